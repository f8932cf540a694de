"""Per-wave phase totals of traj3q_kernel from the RYD_TQ_PROF build variant
(build/libryd_qprof.so: shader-clock sums written over the C5 summary columns).
Usage on the GPU box:
    RYD_ENGINE_LIB=$PWD/build/libryd_qprof.so python tools/traj_qprof.py
"""
import warnings

from noisyquantumsimulator_amd import engine as E
from noisyquantumsimulator_amd import sweeps as SW
from noisyquantumsimulator_amd import trajectories as TR

warnings.simplefilter("ignore")
eng = E.Engine()
params = E.pack_params(SW.blockade_grid_3atom())
db = TR.TrajectoryDeviceBatch(eng, params, "lp_square", TR.plus_state(), n_traj=256, seed=20260215, point_offset=0)
for _ in range(2):
    db.launch()
db.synchronize()
ms = db.launch(timed=True)
r = db.fetch()
tot = r.col("RESERVED")
print(f"C5 quad kernel {ms:.3f} ms, {params.shape[1]} waves; per-wave shader cycles (mean over waves):")
for nm, c in [("pass 1 + setup", "MEAN_JUMPS"), ("walk", "FRAC_JUMPED"), ("  of which service", "NLADDER"),
              ("  of which enter", "NSQUARE"), ("reduce", "MAX_JUMPS")]:
    v = r.col(c)
    print(f"  {nm:20s} {v.mean():12.0f}  ({100 * v.mean() / tot.mean():5.1f} %)")
print(f"  {'total':20s} {tot.mean():12.0f}")
it, ns = r.col("TRACE"), r.col("QUBIT_POP")
use, ex = r.col("ITER_USEFUL"), r.col("ITER_EXEC")
print(f"  loop iterations {it.mean():.1f}, service passes {ns.mean():.1f}, wave-steps {ex.mean() / 16:.1f}, "
      f"useful trajectory-steps {use.mean():.1f}; walk cycles per iteration {r.col('FRAC_JUMPED').mean() / it.mean():.0f}")
