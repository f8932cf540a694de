"""Per-wave phase timeline of lindblad_sym16_kernel from the RYD_S16_PROF build variant
(build/libryd_prof.so: shader-clock timestamps written to the summary's unused Lindblad
columns).  Usage on the GPU box:
    RYD_ENGINE_LIB=$PWD/build/libryd_prof.so python tools/phase_prof.py [c2|c3] [n ...]
"""
import sys
import warnings
from collections import defaultdict

import numpy as np

from noisyquantumsimulator_amd import engine as E
from noisyquantumsimulator_amd import sweeps as SW

warnings.simplefilter("ignore")
w = sys.argv[1] if len(sys.argv) > 1 else "c2"
ns = [int(a) for a in sys.argv[2:]] or [4096, 10000]
if w == "c2":
    full = E.pack_params(SW.omega_delta_grid(200, 200))
    proto, nst = "lp_square", None
else:
    full = SW.c3_four_op_params(SW.pareto_tgate_grid(400, 100))
    proto, nst = "smooth_jp", 300
eng = E.Engine()
names = ["load", "cheb", "square", "transpose", "segments", "epilogue"]
for n in ns:
    idx = np.linspace(0, full.shape[1] - 1, n).round().astype(int) if n != 10000 or w != "c2" else None
    prm = E.pack_params(SW.omega_delta_grid(100, 100)) if idx is None else full[:, idx].copy()
    db = E.DeviceBatch(eng, prm, proto, "lindblad", n_steps=nst)
    for _ in range(3):
        db.launch()
    db.synchronize()
    ms = db.launch(timed=True)
    r = db.fetch()
    S = r.summary
    cyc = S[4:10, ::4]                       # per wave (first point of each wave)
    t0 = S[10, ::4]
    t1 = S[11, ::4]
    hw = S[13, ::4].astype(np.int64)
    xcc = np.zeros_like(hw)                  # (the XCC column carries the staging timestamp)
    stage = S[14, ::4] - S[8, ::4]
    d = np.diff(np.vstack([np.zeros(cyc.shape[1]), cyc]), axis=0)
    print(f"== {w} n={n} waves={n // 4} kernel {ms * 1e3:.1f} us (HIP events)")
    for k, nm in enumerate(names):
        print(f"  {nm:10s} mean {d[k].mean():9.0f} cyc  p10 {np.percentile(d[k], 10):9.0f}  "
              f"p90 {np.percentile(d[k], 90):9.0f}  max {d[k].max():9.0f}")
    print(f"  (epilogue: rotate + LDS staging + state stores {stage.mean():.0f} cyc, summary "
          f"{(cyc[5] - S[14, ::4]).mean():.0f} cyc)")
    tot = cyc[-1]
    print(f"  total      mean {tot.mean():9.0f} cyc  max {tot.max():9.0f}")
    rt0 = (t0 - t0.min()) * 0.01             # 100 MHz -> us
    rt1 = (t1 - t0.min()) * 0.01
    print(f"  wall: start p50 {np.median(rt0):.2f} us max {rt0.max():.2f}; end p50 {np.median(rt1):.2f} "
          f"max {rt1.max():.2f}; wave duration p50 {np.median(rt1 - rt0):.2f} us max {(rt1 - rt0).max():.2f}")
    print(f"  clock: {np.median(tot / np.maximum(rt1 - rt0, 1e-3)) / 1e3:.2f} GHz (cycles / wall)")
    simd = defaultdict(list)
    for k in range(len(hw)):
        key = (int(xcc[k]), (int(hw[k]) >> 13) & 7, (int(hw[k]) >> 12) & 1, (int(hw[k]) >> 8) & 15,
               (int(hw[k]) >> 4) & 3)
        simd[key].append((rt0[k], rt1[k]))
    cnt = np.array([len(v) for v in simd.values()])
    print(f"  SIMDs used {len(simd)}  waves/SIMD min {cnt.min()} max {cnt.max()} "
          f"hist {np.bincount(cnt).tolist()}")
    conc = []
    for v in simd.values():
        ev = sorted([(a, 1) for a, b in v] + [(b, -1) for a, b in v])
        c = m = 0
        for _, e in ev:
            c += e
            m = max(m, c)
        conc.append(m)
    print(f"  max concurrent waves per SIMD hist {np.bincount(conc).tolist()}")
    late = rt0 > 2.0
    if late.any():
        print(f"  waves starting > 2 us after the first: {late.sum()}  (start p50 {np.median(rt0[late]):.2f} us)")
    db.free()
