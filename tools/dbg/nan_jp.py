import warnings, numpy as np
from noisyquantumsimulator_amd import engine as E, sweeps as SW
from noisyquantumsimulator_amd._native import P
warnings.simplefilter("ignore")
p = SW.c3_four_op_params(SW.pareto_tgate_grid(n_omega=100, n_tau=100))
eng = E.Engine()
for ns in (300, 1000, 3000):
    r = eng.run(p, "smooth_jp", "lindblad", n_steps=ns)
    bad = np.nonzero(r.status)[0]
    print(ns, "bad", len(bad), bad[:10])
    if len(bad):
        i = bad[0]
        tau = p[P["TAU"], i]; om = p[P["OMEGA"], i]
        print(" tau", tau, "Om", om, "V", p[P["V"], i], "dt", tau / ns)
        print(" state col", r.state[:, 4 * i + 3])
        print(" summary", r.summary[:, i])
# (appended) per-point series length and wave max, to correlate with the bad points
