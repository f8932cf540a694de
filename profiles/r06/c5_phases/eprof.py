import sys, warnings, numpy as np
sys.path.insert(0, '.')
warnings.simplefilter('ignore')
from noisyquantumsimulator_amd import engine as E, sweeps as SW, trajectories as TR
eng = E.Engine()
for shards in (1, 8):
    b, off = SW.c5_rank_shard(0, shards)
    p = E.pack_params(b)
    db = TR.TrajectoryDeviceBatch(eng, p, "lp_square", n_traj=256, seed=20260215, point_offset=off, kernel="lanes")
    for _ in range(2): db.launch()
    db.synchronize()
    ms = db.launch(timed=True)
    r = db.fetch(); db.free()
    tot = r.col("RESERVED")
    names = [("pass1", "MEAN_JUMPS"), ("  jacobi", "ITER_USEFUL"), ("classify", "FRAC_JUMPED"), ("walk", "MAX_JUMPS"),
             ("reduce", "TRACE"), ("outputs", "QUBIT_POP"), ("merge", "ITER_EXEC")]
    print(f"shards {shards}: {ms:.3f} ms, points {p.shape[1]}; cycles per point-writing wave (mean / p90 / max)")
    for nm, c in names:
        v = r.col(c)
        print(f"  {nm:10s} {v.mean():10.0f} {np.percentile(v, 90):10.0f} {v.max():10.0f}")
    print(f"  {'total':10s} {tot.mean():10.0f} {np.percentile(tot, 90):10.0f} {tot.max():10.0f}")
    lt = (r.col("NSQUARE") - r.col("NLADDER")) * 10.0   # ns, 100 MHz clock
    print(f"  wave lifetime ns mean {lt.mean():.0f} max {lt.max():.0f}")
