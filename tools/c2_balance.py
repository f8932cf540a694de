"""Per-SIMD load of lindblad_sym16_kernel on the C2 grid, from the RYD_S16_PROF build
variant (see tools/phase_prof.py).  For each wave: its XCD and dispatch slot (inverted
from xcd_block), the SIMD it ran on (HW_ID), its shader cycles, wall start/end and the
squaring levels of its points.  Prints whether dispatch slot k of an XCD lands on a
fixed SIMD (k mod 128), the per-SIMD summed cycles, and which SIMDs end the launch.
Usage on the GPU box:
    RYD_ENGINE_LIB=$PWD/build_var/lib_s16prof.so python tools/c2_balance.py [out.npz]
"""
import sys
import warnings
from collections import defaultdict

import numpy as np

from noisyquantumsimulator_amd import engine as E
from noisyquantumsimulator_amd import sweeps as SW

warnings.simplefilter("ignore")
prm = E.pack_params(SW.omega_delta_grid(100, 100))
n = prm.shape[1]
eng = E.Engine()
db = E.DeviceBatch(eng, prm, "lp_square", "lindblad")
for _ in range(3):
    db.launch()
db.synchronize()
ms = db.launch(timed=True)
S = db.fetch().summary
db.free()
nw = n // 4
nb = nw
full = (nb // 32) * 32
c = np.arange(nw)
# inverse of xcd_block (RYD_XCD_MAP 2): chunk c -> block b = 8 k + x
k = np.where(c < full, (c >> 5) * 4 + (c & 3), c // 8)
x = np.where(c < full, (c >> 2) & 7, c % 8)
b = np.where(c < full, 8 * k + x, c)
k = b // 8
x = b % 8
cyc = S[9, ::4]
t0 = S[10, ::4]
t1 = S[11, ::4]
hw = S[13, ::4].astype(np.int64)
nsq = S[19].reshape(nw, 4).max(1)
se = (hw >> 13) & 7
sh = (hw >> 12) & 1
cu = (hw >> 8) & 15
simd = (hw >> 4) & 3
key = [(int(x[i]), int(se[i]), int(sh[i]), int(cu[i]), int(simd[i])) for i in range(nw)]
rt0 = (t0 - t0.min()) * 0.01
rt1 = (t1 - t0.min()) * 0.01
print(f"C2 n={n} waves={nw} kernel {ms * 1e3:.1f} us; wall end max {rt1.max():.2f} us")
by = defaultdict(list)
for i in range(nw):
    by[key[i]].append(i)
cnt = np.array([len(v) for v in by.values()])
print(f"SIMDs {len(by)}  waves/SIMD hist {np.bincount(cnt).tolist()}")
# slot -> SIMD consistency: waves k, k+128, k+256 of one XCD on one SIMD?
same = tot = 0
for i in range(nw):
    if k[i] >= 128:
        j = np.nonzero((x == x[i]) & (k == k[i] - 128))[0]
        if len(j):
            tot += 1
            same += key[j[0]] == key[i]
print(f"slot k and k-128 of an XCD on the same SIMD: {same}/{tot}")
# third waves: slots
third = [v for v in by.values() if len(v) >= 3]
ks = np.array([sorted(k[v]) for v in third if len(v) == 3])
if len(ks):
    print("3-wave SIMDs: slot ranges", ks.min(0).tolist(), ks.max(0).tolist())
load = {kk: cyc[v].sum() for kk, v in by.items()}
end = {kk: rt1[v].max() for kk, v in by.items()}
L = np.array(list(load.values()))
print(f"per-SIMD cycles: mean {L.mean():.0f} max {L.max():.0f} (3-wave mean "
      f"{np.mean([load[kk] for kk, v in by.items() if len(v) == 3]):.0f}, 2-wave mean "
      f"{np.mean([load[kk] for kk, v in by.items() if len(v) == 2]):.0f})")
print(f"per-wave cycles: mean {cyc.mean():.0f} min {cyc.min():.0f} max {cyc.max():.0f}")
for s in np.unique(nsq):
    m = nsq == s
    print(f"  nsq {int(s)}: {m.sum()} waves, cycles mean {cyc[m].mean():.0f}, wall dur mean "
          f"{(rt1 - rt0)[m].mean():.2f} us")
last = sorted(end, key=end.get)[-12:]
print("latest-ending SIMDs: (end us, waves, slots, nsq, cycles)")
for kk in last:
    v = by[kk]
    print(f"  {end[kk]:.2f} {len(v)} {sorted(k[v].tolist())} {nsq[v].astype(int).tolist()} {cyc[v].astype(int).tolist()}")
if len(sys.argv) > 1:
    np.savez(sys.argv[1], k=k, x=x, cyc=cyc, rt0=rt0, rt1=rt1, hw=hw, nsq=nsq)
