"""Per-wave start/end (100 MHz realtime) of traj3e on the C5 grid, by order (prof build)."""
import sys, warnings
import numpy as np
from noisyquantumsimulator_amd import engine as E, sweeps as SW, trajectories as TR
warnings.simplefilter("ignore")
order = sys.argv[1]; shards = int(sys.argv[2]) if len(sys.argv) > 2 else 1
eng = E.Engine()
b, off = SW.c5_rank_shard(0, shards, order=order)
params = E.pack_params(b)
db = TR.TrajectoryDeviceBatch(eng, params, "lp_square", TR.plus_state(), n_traj=256, ladder_levels=0, seed=20260215, point_offset=off)
for _ in range(2): db.launch()
db.synchronize(); ms = db.launch(timed=True); r = db.fetch()
t0, t1 = r.col("NLADDER"), r.col("NSQUARE")
base = t0.min(); t0 = (t0 - base) / 100.0; t1 = (t1 - base) / 100.0          # us
om = b["Omega"] / (2e6 * np.pi); vo = b["V_over_Omega"]
print(f"{order} shards={shards}: kernel {ms:.3f} ms; span {t1.max():.1f} us; start range {t0.min():.1f}..{t0.max():.1f}")
dur = t1 - t0
print(f"  wave duration us: mean {dur.mean():.1f} p50 {np.median(dur):.1f} p90 {np.percentile(dur,90):.1f} max {dur.max():.1f}")
idx = np.argsort(-t1)[:10]
for i in idx:
    print(f"  pt {i:5d} Om {om[i]:5.2f} V/Om {vo[i]:7.1f} start {t0[i]:7.1f} end {t1[i]:7.1f} dur {dur[i]:7.1f} jumps {r.col('RESERVED')[i]:.0f}")
hist = np.histogram(t0, bins=10)
print("  start histogram", hist[0].tolist(), np.round(hist[1], 0).tolist())
# duration vs Omega decile
for q in range(0, 64, 8):
    m = (np.round((om - 1) / 9 * 63) >= q) & (np.round((om - 1) / 9 * 63) < q + 8)
    print(f"  Om idx {q:2d}-{q+7:2d}: mean dur {dur[m].mean():7.1f} max {dur[m].max():7.1f}")
