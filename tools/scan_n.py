"""Kernel time vs batch size for the C2 workload (wave quantisation study).
    python tools/scan_n.py [workload]"""
import sys
import warnings

import numpy as np

from noisyquantumsimulator_amd import engine as E
from noisyquantumsimulator_amd import sweeps as SW

warnings.simplefilter("ignore")
w = sys.argv[1] if len(sys.argv) > 1 else "c2"
if w == "c2":
    full = E.pack_params(SW.omega_delta_grid(200, 200))          # 40k points, C2 ranges
    proto, ns = "lp_square", None
else:
    full = SW.c3_four_op_params(SW.pareto_tgate_grid(400, 100))
    proto, ns = "smooth_jp", 300
eng = E.Engine()
rng = np.random.default_rng(0)
for n in (1024, 2048, 3072, 4096, 6144, 8192, 10000, 12288, 16384, 20000, 24576, 32768, 40000):
    if n > full.shape[1]:
        break
    idx = np.sort(rng.choice(full.shape[1], n, replace=False))
    db = E.DeviceBatch(eng, full[:, idx].copy(), proto, "lindblad", n_steps=ns)
    for _ in range(3):
        db.launch()
    db.synchronize()
    db.mark(0)
    for _ in range(20):
        db.launch()
    db.mark(1)
    ms = db.mark_elapsed() / 20
    print(f"{w} n={n:6d} waves={n // 4:6d} waves/SIMD={n / 4 / 1024:5.2f} kernel {ms * 1e3:8.2f} us  "
          f"{n / ms / 1e3:8.2f} Mpts/s", flush=True)
    db.free()
