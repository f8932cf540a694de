"""A/B numerics: the RYD_MASKED_ADD=3 build (build_var/ma3.so) must give bit-identical
states to the in-tree library on C2/C3/C4-like batches."""
import ctypes, os, subprocess, sys, warnings
import numpy as np
warnings.simplefilter("ignore")
if len(sys.argv) == 1:
    outs = []
    for lib in ("", os.path.abspath("build_var/ma3.so")):
        env = dict(os.environ, RYD_ENGINE_LIB=lib) if lib else dict(os.environ)
        subprocess.run([sys.executable, __file__, "run", "/tmp/ma3_%d.npz" % len(outs)], env=env, check=True)
        outs.append(np.load("/tmp/ma3_%d.npz" % len(outs)))
    for k in outs[0].files:
        a, b = outs[0][k], outs[1][k]
        print(k, "identical" if np.array_equal(a, b, equal_nan=True) else "max diff %.3e" % np.nanmax(np.abs(a - b)))
else:
    from noisyquantumsimulator_amd import engine as E, sweeps as SW
    eng = E.Engine()
    c2 = E.pack_params(SW.omega_delta_grid(40, 40))
    c3 = SW.c3_four_op_params(SW.pareto_tgate_grid(n_omega=40, n_tau=25))
    r2 = eng.run(c2, "lp_square", "lindblad")
    r3 = eng.run(c3, "smooth_jp", "lindblad", n_steps=300)
    np.savez(sys.argv[2], c2=r2.state, c3=r3.state, s2=r2.status, s3=r3.status)
