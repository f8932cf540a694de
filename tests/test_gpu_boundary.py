"""The host-buffer boundary (ryd_run_batch): persistent per-slot device workspace and
pinned staging, every slot enqueued before the first wait, host-thread unpack.

* a handle with two slots on the same device range-partitions the batch; both
  slots are enqueued before the first wait (host timeline, ryd_last_timeline) and the
  result is bit-identical to the one-slot handle's;
* the workspace grows and is reused across calls of different sizes without changing
  any result;
* D2H into the pinned staging runs at PCIe speed (no pageable copy)."""
import warnings

import numpy as np
import pytest

from noisyquantumsimulator_amd import engine as E
from noisyquantumsimulator_amd import sweeps as SW

pytestmark = pytest.mark.gpu


def _heavy_params(n_omega=100):
    """10k smooth-JP points, 4-op model (3000 segments: ~0.6 ms kernels per slot)."""
    warnings.simplefilter("ignore")
    return SW.c3_four_op_params(SW.pareto_tgate_grid(n_omega=n_omega, n_tau=100))


def test_two_slot_handle_enqueues_all_before_waiting_and_matches_one_slot():
    p = _heavy_params()
    one = E.Engine(devices=[0])
    two = E.Engine(devices=[0, 0])
    r1 = one.run(p, "smooth_jp", "lindblad", n_steps=3000)
    two.run(p, "smooth_jp", "lindblad", n_steps=3000)           # warm the workspace
    r2 = two.run(p, "smooth_jp", "lindblad", n_steps=3000)
    assert np.all(r1.status == 0) and np.all(r2.status == 0)
    assert np.array_equal(r1.state, r2.state)
    assert np.array_equal(r1.summary, r2.summary, equal_nan=True)   # Lindblad OV rows are NaN
    tl = two.last_timeline()
    s0, s1 = tl["slots"]
    assert s0["points"] + s1["points"] == p.shape[1]
    assert s0["device"] == s1["device"] == 0
    for s in (s0, s1):
        assert s["h2d_start"] <= s["kernel_start"] <= s["kernel_end"] <= s["d2h_end"]
    # deterministic (program order): every slot's parameters were packed in one
    # pass and both kernels were enqueued before the host waited for either slot
    assert max(s0["host_enqueued"], s1["host_enqueued"]) <= min(s0["host_wait"], s1["host_wait"]), tl
    # the device-side overlap is a measurement, reported (bench.py host_path has the same
    # timeline), not asserted: it depends on kernel length against the enqueue gap
    overlap = min(s0["kernel_end"], s1["kernel_end"]) - max(s0["kernel_start"], s1["kernel_start"])
    print(f"timeline {tl}; kernel overlap {overlap:.3f} ms")
    one.close()
    two.close()


def test_workspace_reuse_across_sizes():
    warnings.simplefilter("ignore")
    b = SW.omega_delta_grid(40, 50)               # 2000 points, C2 layout
    p = E.pack_params(b)
    eng = E.Engine()
    ref = {}
    for n in (2000, 300, 2000, 7, 1999):
        r = eng.run(p[:, :n].copy(), "lp_square", "lindblad")
        assert np.all(r.status == 0)
        if n in ref:
            assert np.array_equal(ref[n].state, r.state)
        ref.setdefault(n, r)
    # a prefix of the batch gives the same rows as the whole batch
    assert np.array_equal(ref[300].state, ref[2000].state.reshape(25, 2000, 4)[:, :300].reshape(25, 1200))
    fresh = E.Engine().run(p[:, :1999].copy(), "lp_square", "lindblad")
    assert np.array_equal(fresh.state, ref[1999].state)


def test_pinned_d2h_rate():
    warnings.simplefilter("ignore")
    p = E.pack_params(SW.omega_delta_grid())     # C2, 10k points: 9.6 MB back
    eng = E.Engine()
    eng.run(p, "lp_square", "lindblad")
    r = eng.run(p, "lp_square", "lindblad")
    nbytes = 8 * (25 * 4 + E.N.NSUMMARY) * p.shape[1] + 4 * p.shape[1]
    gbs = nbytes / (r.d2h_ms * 1e-3) / 1e9
    print(f"d2h {r.d2h_ms:.3f} ms = {gbs:.1f} GB/s; timeline {eng.last_timeline()}")
    assert gbs > 10.0
