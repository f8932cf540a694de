"""CPU timing of the host epilogue (ryd_mixed_phase) with and without the gauge check on
4000 noisy-fixture-derived points (8 threads); compare builds with RYD_ENGINE_LIB=<lib>."""
import os
import sys
import time

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "tests")]
import numpy as np
from test_mixed_phase_host import _noisy_fixture_states
from noisyquantumsimulator_amd import engine as E
blocks = [S for _, S in _noisy_fixture_states()]
rng = np.random.default_rng(1)
n = 4000
st = np.zeros((25, 4 * n))
for i in range(n):
    S = blocks[i % len(blocks)]
    st[:, 4*i:4*i+4] = S * (1.0 + 1e-7 * rng.standard_normal(S.shape)) * (np.abs(S) > 1e-15)
for copies in (0, 1, 4):
    ts = []
    for _ in range(7):
        t0 = time.perf_counter(); E.mixed_phase(st, n, 3, gauge_check=copies > 0, copies=max(copies, 1), n_threads=8); ts.append(time.perf_counter() - t0)
    print(os.environ['RYD_ENGINE_LIB'].split('/')[-1], 'copies', copies, 'median %.1f ms' % (np.median(ts) * 1e3))
