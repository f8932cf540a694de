"""Host unpack rate of the host-buffer boundary vs the caller's output allocation
(round-3 probe): fresh np.zeros, fresh np.empty, pre-faulted arrays."""
import sys
import time
import warnings

import numpy as np

sys.path.insert(0, ".")
from noisyquantumsimulator_amd import engine as E  # noqa: E402
from noisyquantumsimulator_amd import sweeps as SW  # noqa: E402

warnings.simplefilter("ignore")
p = E.pack_params(SW.omega_delta_grid())
eng = E.Engine()
real_zeros = np.zeros
for mode in ("zeros", "empty", "prefault", "zeros", "empty"):
    if mode == "empty":
        E.np.zeros = lambda *a, **k: np.empty(*a, **{kk: v for kk, v in k.items()})
    elif mode == "prefault":
        def pf(*a, **k):
            x = np.empty(*a, **k)
            x.fill(0)
            return x
        E.np.zeros = pf
    else:
        E.np.zeros = real_zeros
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        r = eng.run(p, "lp_square", "lindblad")
        ts.append(time.perf_counter() - t0)
        tl = eng.last_timeline()
    E.np.zeros = real_zeros
    print(f"{mode:9s} call {np.median(ts) * 1e3:.3f} ms  pack {tl['pack_ms']:.3f}  unpack {tl['unpack_ms']:.3f} ms "
          f"({9.64e6 / (tl['unpack_ms'] * 1e-3) / 1e9:.1f} GB/s)  d2h {r.d2h_ms:.3f}", flush=True)
import os
for f in ("/sys/kernel/mm/transparent_hugepage/enabled", "/sys/kernel/mm/transparent_hugepage/defrag"):
    try:
        print(f, open(f).read().strip())
    except OSError as e:
        print(f, e)
print("nproc", os.cpu_count(), "OMP", os.environ.get("OMP_NUM_THREADS"))
