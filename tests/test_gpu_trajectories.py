"""Three-atom blockade with quantum-jump trajectories (C5) on the GPU, through the
C-ABI (ryd_run_trajectories), against the CPU oracle (oracle/three_atom_oracle.py):

* rates = 0: every trajectory is the Schrodinger ket -> mean rho exact to 1e-10, se = 0;
* atom parked in |0>: equals the two-atom GPU ket engine;
* noisy: mean rho within 5.5 standard errors of the exact 729x729 Liouvillian state;
* single trajectories: same jump count / channels, jump times within the ladder
  quantum, same final ket as the exact-jump-time oracle on the same Philox stream;
* launch-shape independence (bit-exact), bad inputs, full 4096-point C5 grid properties.
"""
import warnings

import numpy as np
import pytest

from noisyquantumsimulator_amd import _native as N
from noisyquantumsimulator_amd import configurations as CF
from noisyquantumsimulator_amd import engine as E
from noisyquantumsimulator_amd import physics as PH
from noisyquantumsimulator_amd import sweeps as SW
from noisyquantumsimulator_amd import trajectories as TR
from oracle import three_atom_oracle as O3

pytestmark = pytest.mark.gpu

KW = dict(species="Rb87", n_rydberg=70, tweezer_power=0.020, tweezer_waist=0.8e-6, temperature=2e-6,
          spacing_factor=2.8, B_field=1e-4, NA=0.5)


@pytest.fixture(scope="module")
def eng():
    return E.Engine()


def _c5(idx, scale=1.0):
    warnings.simplefilter("ignore")
    p = E.pack_params(SW.blockade_grid_3atom(point_slice=slice(0, SW.C5_POINTS)))[:, idx].copy()
    p[4:12] *= scale
    return np.ascontiguousarray(p)


def _two_atom(si, n=2):
    warnings.simplefilter("ignore")
    exc = SW.medium_excitation()
    b = PH.derive_batch(si(excitation=exc), n, **dict(KW, temperature=np.linspace(2e-6, 5e-6, n)))
    return E.pack_params(b)


LADDERS = [16, N.T["EXACT"]]          # the ladder walk and the exact-jump-time kernel
# (ladder_levels, exact-mode kernel): the ladder, traj3e (one trajectory per lane, the
# default) and traj3r (one trajectory per 16-lane DPP row, include/ryd_engine.h RYD_T_FLAG_ROWS)
MODES = [(16, "auto"), (N.T["EXACT"], "lanes"), (N.T["EXACT"], "rows")]
EXACT_KERNELS = ["lanes", "rows"]


@pytest.mark.parametrize("ladder", LADDERS)
@pytest.mark.parametrize("protocol,n_steps,shape", [("lp_square", None, "square"), ("bangbang", None, "square"),
                                                    ("smooth_jp", 60, "square"), ("lp_shaped", 40, "cosine")])
def test_zero_rates_equal_pure_evolution(eng, protocol, n_steps, shape, ladder):
    if ladder == N.T["EXACT"] and protocol == "lp_shaped":
        pytest.skip("a shaped envelope has no constant H_eff: exact mode refuses it (test_bad_inputs)")
    if protocol == "lp_square":
        p = _c5([0, 700, 2100, 4095])
    elif protocol == "bangbang":
        p = _two_atom(CF.JPSimulationInputs)
    elif protocol == "smooth_jp":
        p = _two_atom(CF.SmoothJPSimulationInputs)
    else:
        p = _two_atom(lambda excitation: CF.LPSimulationInputs(excitation=excitation, pulse_shape="cosine"))
    p[4:12] = 0.0
    ns = n_steps if n_steps is not None else E.default_n_steps(protocol, p)
    psi0 = TR.plus_state()
    r = TR.run_trajectories(eng, p, protocol, psi0, n_traj=256, n_steps=ns, shape=shape, ladder_levels=ladder)
    assert np.all(r.status == 0)
    assert np.all(r.col("MEAN_JUMPS") == 0)
    for i in range(p.shape[1]):
        psi = O3.pure_ket(p[:, i], protocol, psi0, n_steps=ns, shape=shape)
        np.testing.assert_allclose(r.rho[i], np.outer(psi, psi.conj()), atol=1e-10, rtol=0, err_msg=f"{protocol}/{i}")
        assert r.se[i].max() < 1e-12
    np.testing.assert_allclose(r.col("TRACE"), 1.0, atol=1e-12)


def test_spectator_atom_matches_two_atom_engine(eng):
    p = _c5([10, 3000])
    p[4:12] = 0.0
    k2 = eng.run(p, "lp_square", "ket").kets()               # two-atom GPU ket path
    one, zero = np.array([0, 1, 0]), np.array([1, 0, 0])
    r = TR.run_trajectories(eng, p, "lp_square", TR.product_ket(one, one, zero), n_traj=256)
    for i in range(2):
        psi = np.kron(k2[i, 3], zero)                        # input |11> (label index 3) (x) |0>
        np.testing.assert_allclose(r.rho[i], np.outer(psi, psi.conj()), atol=1e-10, rtol=0)


@pytest.mark.parametrize("ladder", LADDERS)
def test_noisy_mean_rho_within_standard_error(eng, ladder):
    idx = [5, 1800, 4000]
    p = _c5(idx, scale=30.0)
    psi0 = TR.plus_state()
    r = TR.run_trajectories(eng, p, "lp_square", psi0, n_traj=2048, seed=20260215, ladder_levels=ladder)
    assert np.all(r.status == 0)
    assert np.all(r.col("MEAN_JUMPS") > 0.05)
    np.testing.assert_allclose(r.col("TRACE"), 1.0, atol=1e-12)
    z2 = []
    for i in range(len(idx)):
        ref = O3.exact_rho(p[:, i], "lp_square", psi0)
        d = np.abs(r.rho[i] - ref)
        # rare-channel elements may have no sampled event: Poisson floor sqrt(|rho| / n)
        se = np.maximum(r.se[i], np.sqrt(np.abs(ref) / 2048))
        ok = (d < 1e-9) | (d < 5.5 * se + 1e-8)
        assert ok.all(), (i, (d / np.maximum(se, 1e-300)).max())
        m = r.se[i] > 1e-4
        z2.append(((d[m] / r.se[i][m]) ** 2).mean())
    assert 0.3 < np.mean(z2) < 2.0, z2                        # the errors ARE standard errors


@pytest.mark.parametrize("ladder", LADDERS)
@pytest.mark.parametrize("protocol,n_steps", [("bangbang", None), ("smooth_jp", 12)])
def test_noisy_multi_segment_protocols(eng, protocol, n_steps, ladder):
    """Bang-bang rebuilds the ladder every segment (different lengths) inside the
    jumper rounds; smooth JP rotates the frame every segment."""
    p = _two_atom(CF.JPSimulationInputs if protocol == "bangbang" else CF.SmoothJPSimulationInputs, n=1)
    p[4:12] *= 5.0                                            # ~1-2 jumps per trajectory
    ns = n_steps if n_steps is not None else E.default_n_steps(protocol, p)
    psi0 = TR.plus_state()
    r = TR.run_trajectories(eng, p, protocol, psi0, n_traj=2048, seed=99, n_steps=ns, records=True,
                            ladder_levels=ladder)
    assert r.status[0] == 0 and r.col("MEAN_JUMPS")[0] > 0.05
    ref = O3.exact_rho(p[:, 0], protocol, psi0, n_steps=ns)
    d = np.abs(r.rho[0] - ref)
    se = np.maximum(r.se[0], np.sqrt(np.abs(ref) / 2048))
    assert np.all((d < 1e-9) | (d < 5.5 * se + 1e-8)), (d / se).max()
    # and one-to-one against the exact-jump-time oracle for a few trajectories
    nj, cj, kets = r.n_jumps()[0], r.jump_channels()[0], r.kets()[0]
    exact = ladder == N.T["EXACT"]
    tj = r.jump_times()[0]
    t_total = sum(dt for _, _, dt in O3.schedule(p[:, 0], protocol, ns))
    for t in range(6):
        k, jumps = O3.mc_trajectory(p[:, 0], protocol, psi0, point=0, traj=t, seed=99, n_steps=ns)
        assert nj[t] == len(jumps) and all(cj[t, m] == ch for m, (_, ch) in enumerate(jumps[:4]))
        assert abs(np.vdot(k, kets[t])) > 1 - (1e-12 if exact else 1e-6)
        if exact:     # every segment boundary and phase frame crossed at the oracle's jump times
            assert all(abs(tj[t, m] - tt) <= 1e-10 * t_total for m, (tt, _) in enumerate(jumps[:4]))


def test_trajectories_match_exact_time_oracle(eng):
    """One-to-one: same Philox stream -> same jumps and final ket as the CPU unravelling
    with exact (root-found) jump times; the GPU resolves jump times to dt / 2^L."""
    L = 36
    p = _c5([1200], scale=40.0)
    psi0 = TR.plus_state()
    r = TR.run_trajectories(eng, p, "lp_square", psi0, n_traj=256, seed=77, ladder_levels=L, records=True)
    assert r.status[0] == 0
    nj, tj, cj, kets = r.n_jumps()[0], r.jump_times()[0], r.jump_channels()[0], r.kets()[0]
    dt = p[N.P["TAU"], 0]
    checked = 0
    for t in range(24):
        k, jumps = O3.mc_trajectory(p[:, 0], "lp_square", psi0, point=0, traj=t, seed=77)
        assert nj[t] == len(jumps), t
        for m, (tt, ch) in enumerate(jumps[:N.T["REC_JUMPS"]]):
            assert cj[t, m] == ch
            if m == 0:     # first jump: exactly the quantum that contains the crossing
                assert tt - 1e-20 <= tj[t, m] <= tt + dt * 2.0 ** -L + 1e-20
                checked += 1
            else:          # later ones inherit the O(quantum) shift of the state before them
                assert abs(tj[t, m] - tt) <= 1e-9 * tt
        assert abs(np.vdot(k, kets[t])) > 1 - 1e-8, t
    assert checked > 5


@pytest.mark.parametrize("kernel", EXACT_KERNELS)
@pytest.mark.parametrize("idx,scale", [(1200, 40.0), (77, 60.0), (4095, 40.0)])
def test_exact_jump_times_match_oracle(eng, idx, scale, kernel):
    """ladder_levels = RYD_T_EXACT: every jump time is the root the oracle's brentq finds
    (Newton on the eigen-decomposed H_eff), not the end of a ladder quantum -- so later
    jumps agree as tightly as the first, and so do the final kets."""
    p = _c5([idx], scale=scale)
    psi0 = TR.plus_state()
    r = TR.run_trajectories(eng, p, "lp_square", psi0, n_traj=256, seed=77, ladder_levels=N.T["EXACT"],
                            records=True, kernel=kernel)
    assert r.status[0] == 0
    nj, tj, cj, kets = r.n_jumps()[0], r.jump_times()[0], r.jump_channels()[0], r.kets()[0]
    dt = p[N.P["TAU"], 0]
    checked = 0
    for t in range(32):
        k, jumps = O3.mc_trajectory(p[:, 0], "lp_square", psi0, point=0, traj=t, seed=77)
        assert nj[t] == len(jumps), t
        for m, (tt, ch) in enumerate(jumps[:N.T["REC_JUMPS"]]):
            assert cj[t, m] == ch
            assert abs(tj[t, m] - tt) <= 1e-10 * dt, (t, m, tj[t, m], tt)
            checked += 1
        assert abs(np.vdot(k, kets[t])) > 1 - 1e-12, t
    assert checked > 5


@pytest.mark.parametrize("ladder,kernel", MODES)
def test_launch_shape_and_partition_independence(eng, ladder, kernel):
    p = _c5(list(range(0, 4096, 512)), scale=20.0)
    kw = dict(ladder_levels=ladder, kernel=kernel)
    a = TR.run_trajectories(eng, p, "lp_square", n_traj=256, seed=5, records=True, **kw)
    b = TR.run_trajectories(eng, p, "lp_square", n_traj=512, seed=5, records=True, **kw)
    np.testing.assert_array_equal(a.records, b.records[:, :256])     # a trajectory = its stream
    c = TR.run_trajectories(eng, p, "lp_square", n_traj=256, seed=5, **kw)
    np.testing.assert_array_equal(a.rho, c.rho)                         # deterministic
    np.testing.assert_array_equal(a.se, c.se)
    # device-side range shards with their global offsets == one batch (outputs, standard
    # errors and the per-trajectory records bit for bit)
    outs = []
    for lo, hi in ((0, 3), (3, 4), (4, 8)):
        db = TR.TrajectoryDeviceBatch(eng, p[:, lo:hi], "lp_square", n_traj=256, seed=5, point_offset=lo,
                                      records=True, **kw)
        db.launch()
        db.synchronize()
        outs.append(db.fetch())
        db.free()
    np.testing.assert_array_equal(np.concatenate([o.rho for o in outs]), a.rho)
    np.testing.assert_array_equal(np.concatenate([o.se for o in outs]), a.se)
    np.testing.assert_array_equal(np.concatenate([o.records for o in outs]), a.records)
    d = TR.run_trajectories(eng, p, "lp_square", n_traj=256, seed=6, **kw)
    assert not np.array_equal(d.rho, a.rho)


def test_exact_mode_falls_back_for_a_non_constant_schedule(eng):
    """An LP square with |xi| != 1 has two different |Omega| segments: exact mode sends the
    point through the L = 16 ladder (RYD_STATUS_EXACT_FALLBACK, not BAD_INPUT -- ADVICE r3)
    while its neighbours stay exact."""
    p = _c5([300, 1300, 2300], scale=30.0)
    p[N.P["XI_RE"], 1] *= 0.8
    p[N.P["XI_IM"], 1] *= 0.8
    psi0 = TR.plus_state()
    r = TR.run_trajectories(eng, p, "lp_square", psi0, n_traj=2048, seed=11, ladder_levels=N.T["EXACT"])
    assert r.status[1] == N.STATUS_EXACT_FALLBACK, r.status
    assert r.status[0] == 0 and r.status[2] == 0
    lad = TR.run_trajectories(eng, p, "lp_square", psi0, n_traj=2048, seed=11, ladder_levels=16)
    np.testing.assert_array_equal(r.rho[1], lad.rho[1])              # the ladder kernel's own result
    for i in range(3):
        ref = O3.exact_rho(p[:, i], "lp_square", psi0)
        d = np.abs(r.rho[i] - ref)
        se = np.maximum(r.se[i], np.sqrt(np.abs(ref) / 2048))
        assert np.all((d < 1e-9) | (d < 5.5 * se + 1e-8)), (i, (d / se).max())
    q = p.copy()
    q[4:12] = 0.0                                                    # and without noise: the pure ket
    z = TR.run_trajectories(eng, q, "lp_square", psi0, n_traj=256, ladder_levels=N.T["EXACT"])
    assert z.status[1] == N.STATUS_EXACT_FALLBACK
    psi = O3.pure_ket(q[:, 1], "lp_square", psi0)
    np.testing.assert_allclose(z.rho[1], np.outer(psi, psi.conj()), atol=1e-10, rtol=0)


def test_exact_mode_guard_near_an_exceptional_point(eng):
    """The single-atom block [[delta1 - i hgs, w], [w, -Delta - i hgr]] has an exceptional
    point at Delta = -delta1, hgr - hgs = 2 w: there W e^{-i Lam t} W^T loses every digit.
    Tuned to 1e-10 of it, the eigenbasis is flagged ill-conditioned, the point runs on the
    ladder (RYD_STATUS_EXACT_FALLBACK) and still matches the 729 x 729 Liouvillian."""
    p = _c5([1000, 2000])
    i = 1
    w = 0.5 * p[N.P["OMEGA"], i]
    p[N.P["DELTA"], i] = -p[N.P["DELTA1"], i]
    p[4:12, i] = 0.0
    p[N.P["GPHI_A"], i] = p[N.P["GPHI_B"], i] = 4.0 * w * (1.0 + 1e-10)   # hgr = gphi / 2 = 2 w
    psi0 = TR.plus_state()
    r = TR.run_trajectories(eng, p, "lp_square", psi0, n_traj=2048, seed=3, ladder_levels=N.T["EXACT"])
    assert r.status[0] == 0
    assert r.status[i] == N.STATUS_EXACT_FALLBACK, r.status
    assert r.col("MEAN_JUMPS")[i] > 0.05
    ref = O3.exact_rho(p[:, i], "lp_square", psi0)
    d = np.abs(r.rho[i] - ref)
    se = np.maximum(r.se[i], np.sqrt(np.abs(ref) / 2048))
    assert np.all((d < 1e-9) | (d < 5.5 * se + 1e-8)), (d / se).max()


@pytest.mark.parametrize("ladder", LADDERS)
def test_bad_inputs(eng, ladder):
    p = _c5([1, 2, 3])
    p[N.P["OMEGA"], 1] = 0.0
    r = TR.run_trajectories(eng, p, "lp_square", n_traj=256, ladder_levels=ladder)
    assert r.status[1] & N.STATUS_BAD_INPUT and r.status[0] == 0 and r.status[2] == 0
    assert np.all(r.rho[1] == 0)
    with pytest.raises(N.EngineError):
        TR.run_trajectories(eng, p, "lp_square", n_traj=100)
    with pytest.raises(N.EngineError):
        TR.run_trajectories(eng, p, "lp_square", n_traj=256, ladder_levels=-1)
    with pytest.raises(N.EngineError):                      # exact mode needs a constant H_eff
        TR.run_trajectories(eng, _two_atom(lambda excitation: CF.LPSimulationInputs(
            excitation=excitation, pulse_shape="cosine")), "lp_shaped", n_traj=256, n_steps=40, shape="cosine",
            ladder_levels=N.T["EXACT"])


@pytest.mark.parametrize("ladder,kernel", MODES)
def test_c5_full_grid_properties(eng, ladder, kernel):
    warnings.simplefilter("ignore")
    p = E.pack_params(SW.blockade_grid_3atom())
    r = TR.run_trajectories(eng, p, "lp_square", n_traj=256, seed=20260215, ladder_levels=ladder, kernel=kernel)
    assert r.n == 4096 and np.all(r.status == 0)
    np.testing.assert_allclose(r.col("TRACE"), 1.0, atol=1e-12)
    np.testing.assert_allclose(r.rho, np.conj(np.transpose(r.rho, (0, 2, 1))), atol=0)
    assert np.linalg.eigvalsh(r.rho).min() > -1e-12
    q = r.col("QUBIT_POP")
    assert np.all((q > 0.5) & (q <= 1 + 1e-12))
    assert np.all(np.isfinite(r.se))
    psi0 = TR.plus_state()
    for i in (77, 3333):
        ref = O3.exact_rho(p[:, i], "lp_square", psi0)
        d = np.abs(r.rho[i] - ref)
        assert np.all((d < 1e-9) | (d < 5.5 * np.maximum(r.se[i], np.sqrt(np.abs(ref) / 256)) + 1e-8))
    # the N = 8 strong-scaling shards (sweeps.c5_rank_shard) reproduce the full launch's rows
    for rank in (0, 5):
        b, off = SW.c5_rank_shard(rank, 8)
        db = TR.TrajectoryDeviceBatch(eng, E.pack_params(b), "lp_square", n_traj=256, seed=20260215,
                                      point_offset=off, ladder_levels=ladder, kernel=kernel)
        db.launch()
        db.synchronize()
        o = db.fetch()
        db.free()
        np.testing.assert_array_equal(o.rho, r.rho[off:off + o.n])
        np.testing.assert_array_equal(o.se, r.se[off:off + o.n])
        # (ITER_EXEC counts the issued row-evaluations: scheduling-dependent in the exact kernel)
        det = [N.TS[k] for k in ("MEAN_JUMPS", "FRAC_JUMPED", "MAX_JUMPS", "TRACE", "QUBIT_POP", "ITER_USEFUL")]
        np.testing.assert_array_equal(o.summary[det], r.summary[det][:, off:off + o.n])
    # strided shards (sweeps.c5_strided_shard: points r, r + 8, ...; point_stride keys the
    # random streams by global index) reproduce rows r::8 of the same launch
    for rank in (0, 5):
        b, off, stride = SW.c5_strided_shard(rank, 8)
        db = TR.TrajectoryDeviceBatch(eng, E.pack_params(b), "lp_square", n_traj=256, seed=20260215,
                                      point_offset=off, point_stride=stride, ladder_levels=ladder, kernel=kernel)
        db.launch()
        db.synchronize()
        o = db.fetch()
        db.free()
        np.testing.assert_array_equal(o.rho, r.rho[rank::8])
        np.testing.assert_array_equal(o.se, r.se[rank::8])
        np.testing.assert_array_equal(o.summary[det], r.summary[det][:, rank::8])


def test_exact_kernels_agree(eng):
    """traj3r and traj3e walk the same Philox streams to the same jump times; they differ
    only in the order of the floating-point sums (one row per trajectory vs one lane), so the
    outputs agree to rounding and the jump records exactly in count and channel."""
    warnings.simplefilter("ignore")
    p = E.pack_params(SW.blockade_grid_3atom())[:, ::8].copy()
    kw = dict(n_traj=256, seed=20260215, ladder_levels=N.T["EXACT"], records=True)
    a = TR.run_trajectories(eng, p, "lp_square", kernel="lanes", **kw)
    b = TR.run_trajectories(eng, p, "lp_square", kernel="rows", **kw)
    assert np.all(a.status == 0) and np.all(b.status == 0)
    np.testing.assert_allclose(b.rho, a.rho, atol=1e-12, rtol=0)
    np.testing.assert_allclose(b.se, a.se, atol=1e-12, rtol=0)
    np.testing.assert_array_equal(b.n_jumps(), a.n_jumps())
    np.testing.assert_array_equal(b.jump_channels(), a.jump_channels())
    np.testing.assert_allclose(b.jump_times(), a.jump_times(), atol=1e-12 * float(p[N.P["TAU"]].max()), rtol=0)
