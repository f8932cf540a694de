import sys, warnings, heapq, numpy as np
sys.path.insert(0, '.')
warnings.simplefilter('ignore')
from noisyquantumsimulator_amd import engine as E, sweeps as SW, trajectories as TR, _native as N
eng = E.Engine()
b, off = SW.c5_rank_shard(0, 1)
p = E.pack_params(b)
db = TR.TrajectoryDeviceBatch(eng, p, "lp_square", n_traj=256, seed=20260215, point_offset=off, kernel="lanes")
for _ in range(2): db.launch()
db.synchronize(); db.launch(timed=True)
r = db.fetch(); db.free()
n = p.shape[1]; npair = n // 2
t0 = r.col("NLADDER"); t1 = r.col("NSQUARE")
dur = (t1[:npair] - t0[:npair]) * 10.0
pa = np.arange(npair); pb = 2 * npair - 1 - pa
tau = p[N.P["TAU"]]
g = p[4:12].sum(axis=0)
prox = {"tau_max": np.maximum(tau[pa], tau[pb]), "tau_sum": tau[pa] + tau[pb],
        "gtau_max": np.maximum((g * tau)[pa], (g * tau)[pb]), "gtau_sum": (g * tau)[pa] + (g * tau)[pb]}
def sim(order, simds=1024):
    h = [0.0] * simds; heapq.heapify(h); end = 0.0
    for k in order:
        s = heapq.heappop(h); e = s + dur[k]; end = max(end, e); heapq.heappush(h, e)
    return end
print("FIFO", round(sim(range(npair))), "oracle LPT", round(sim(np.argsort(-dur))))
for k, v in prox.items():
    print(k, "corr %.3f" % np.corrcoef(v, dur)[0, 1], "LPT-by-proxy", round(sim(np.argsort(-v, kind="stable"))))
