"""Per-wave phase totals of traj3_kernel from the RYD_T_PROF build variant
(build/libryd_tprof.so: shader-clock phase sums written over the C5 summary columns).
Usage on the GPU box:
    RYD_ENGINE_LIB=$PWD/build/libryd_tprof.so python tools/traj_prof.py [ladder]
"""
import os
import sys
import warnings

import numpy as np

from noisyquantumsimulator_amd import engine as E
from noisyquantumsimulator_amd import sweeps as SW
from noisyquantumsimulator_amd import trajectories as TR

warnings.simplefilter("ignore")
L = int(sys.argv[1]) if len(sys.argv) > 1 else TR.resolve_ladder(TR.DEFAULT_LADDER, "lp_square")
shards = int(sys.argv[2]) if len(sys.argv) > 2 else 1          # time rank 0's shard of an N-way split
eng = E.Engine()
b, off = SW.c5_rank_shard(0, shards)
params = E.pack_params(b)
db = TR.TrajectoryDeviceBatch(eng, params, "lp_square", TR.plus_state(), n_traj=256, ladder_levels=L,
                              seed=20260215, point_offset=off)
for _ in range(2):
    db.launch()
db.synchronize()
ms = db.launch(timed=True)
r = db.fetch()
names = ["ladder+no-jump", "classify", "walk", "reduce", "outputs"]
cols = ["MEAN_JUMPS", "FRAC_JUMPED", "MAX_JUMPS", "TRACE", "QUBIT_POP"]
tot = r.col("RESERVED")
print(f"C5 L={L}: kernel {ms:.3f} ms, {params.shape[1]} waves; per-wave cycles (mean over waves):")
for nm, c in zip(names, cols):
    v = r.col(c)
    print(f"  {nm:15s} mean {v.mean():10.0f}  ({100 * v.mean() / tot.mean():5.1f} %)  p90 {np.percentile(v, 90):10.0f}")
print(f"  {'total':15s} mean {tot.mean():10.0f}  max {tot.max():10.0f}")
if L == 0 and os.environ.get("RYD_T_WG", "0") == "1":      # traj3w_kernel: the eigen-decomposition's share of pass 1
    v = r.col("NLADDER")
    print(f"  (of pass 1: eigen-decomposition mean {v.mean():10.0f}  p90 {np.percentile(v, 90):10.0f})")
    trips, ev, jf = r.col("ITER_USEFUL"), r.col("NSQUARE"), r.col("ITER_EXEC")
    print(f"  wave 0 walk: trips mean {trips.mean():.1f} max {trips.max():.0f}; cycles per trip "
          f"{(ev.sum() + jf.sum()) / trips.sum():.0f} (restart + evaluation {ev.sum() / trips.sum():.0f}, "
          f"segments/jumps/ends/fetch {jf.sum() / trips.sum():.0f})")
    sys.exit(0)
if L == 0:                       # traj3e_kernel: the outputs phase's split (range merges)
    arr, mrg = r.col("ITER_USEFUL"), r.col("ITER_EXEC")
    print(f"  (of outputs: the merge's jumper lists mean {arr.mean():.0f} p90 {np.percentile(arr, 90):.0f}; "
          f"merge in all (lists, ket loads, reduction) mean {mrg.mean():.0f} p90 {np.percentile(mrg, 90):.0f})")
    sys.exit(0)
use, ex = r.col("ITER_USEFUL"), r.col("ITER_EXEC")
print(f"  ladder steps useful {use.sum():.3g}, executed {ex.sum():.3g} (exec/useful {ex.sum() / use.sum():.2f}); "
      f"walk cycles per executed wave-step {r.col('MAX_JUMPS').sum() / (ex.sum() / 64):.0f}")
if L != 0 and r.col("NSQUARE").max() < 100:   # the sym kernel's prof build: ladder phase split
    print(f"  ladder build split (pass 1): taylor {r.col('ITER_USEFUL').mean():.0f}  squarings "
          f"{r.col('ITER_EXEC').mean():.0f}  levels {r.col('NLADDER').mean():.0f}  s0 {r.col('NSQUARE').mean():.2f}")
