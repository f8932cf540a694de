import sys, warnings, heapq, numpy as np
sys.path.insert(0, '.')
warnings.simplefilter('ignore')
from noisyquantumsimulator_amd import engine as E, sweeps as SW, trajectories as TR
eng = E.Engine()
b, off = SW.c5_rank_shard(0, 1)
p = E.pack_params(b)
db = TR.TrajectoryDeviceBatch(eng, p, "lp_square", n_traj=256, seed=20260215, point_offset=off, kernel="lanes")
for _ in range(2): db.launch()
db.synchronize()
ms = db.launch(timed=True)
r = db.fetch(); db.free()
n = p.shape[1]; npair = n // 2
t0 = r.col("NLADDER"); t1 = r.col("NSQUARE")        # 100 MHz wave start / end of the wave writing the point
# wave b writes points b (slot 0) and 2 npair - 1 - b (slot 1)
w0 = t0[:npair]; w1 = t1[:npair]
dur = (w1 - w0) * 10.0                                # ns
start = w0 - w0.min()
print(f"kernel {ms:.3f} ms; waves {npair}; wave ns mean {dur.mean():.0f} p90 {np.percentile(dur,90):.0f} max {dur.max():.0f}")
print(f"actual span ns {(w1.max() - w0.min()) * 10:.0f}; sum/1024 {dur.sum()/1024:.0f}")
def sim(order, simds=1024):
    h = [0.0] * simds
    heapq.heapify(h)
    end = 0.0
    for k in order:
        s = heapq.heappop(h)
        e = s + dur[k]
        end = max(end, e)
        heapq.heappush(h, e)
    return end
print("FIFO (blockIdx order) simulated ns", round(sim(range(npair))))
print("LPT (longest first) simulated ns", round(sim(np.argsort(-dur))))
# a host-side proxy: the pulse length times the summed decay rates of the pair
tau = p[E.N.P["TAU"]] if hasattr(E, "N") else None
