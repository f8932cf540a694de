import sys, warnings, numpy as np
sys.path.insert(0, '.')
warnings.simplefilter('ignore')
from noisyquantumsimulator_amd import engine as E, sweeps as SW, _native as N
eng = E.Engine()
import bench as B
b = SW.c2_rank_shard(0, 1, B.N_DELTA, B.N_OMEGA)
p = E.pack_params(b)
def timeit(pp, k=30):
    db = E.DeviceBatch(eng, pp, "lp_square", "lindblad")
    for _ in range(5): db.launch()
    db.synchronize()
    t = [db.launch(timed=True) for _ in range(k)]
    r = db.fetch(); db.free()
    return float(np.median(t)) * 1e3, r
t0, r = timeit(p)
nsq = r.summary[N.S["NSQUARE"]]; nmv = r.summary[N.S["NMV_EXEC"]]
cost = 3750.0 * nsq + 139.0 * nmv
print("orig us %.2f" % t0, "nsq min/max", nsq.min(), nsq.max(), "nmv min/max", nmv.min(), nmv.max(),
      "cost cv %.3f" % (cost.std() / cost.mean()), flush=True)
# quads of 4 points share a wave: sort points by cost so each quad is homogeneous, heavy first
order = np.argsort(-cost, kind="stable")
t1, r1 = timeit(p[:, order])
print("sorted desc us %.2f" % t1, flush=True)
t2, _ = timeit(p[:, order[::-1]])
print("sorted asc us %.2f" % t2, flush=True)
# bit check: a point's outputs do not depend on its quad neighbours
st = r.state.reshape(r.state.shape[0], -1, 4)
st1 = r1.state.reshape(r1.state.shape[0], -1, 4)
print("row-independent:", np.array_equal(st[:, order], st1))
t3, _ = timeit(p)
print("orig again us %.2f" % t3, flush=True)
