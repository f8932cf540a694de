"""GPU parity: the HIP engine (through the C-ABI) vs the expm oracle.

Tolerances (fp64):
* Lindblad rho elements, ket amplitudes: |d| <= 1e-10 against the exact
  propagator (the engine is exact to ~1e-13; SURVEY.md §7 hard part 1);
* populations / fidelities: <= 1e-10;
* published notebook numbers: to their printed digits.
"""
import warnings

import numpy as np
import pytest

from conftest import states_from_fixture
from golden_configs import derive
from noisyquantumsimulator_amd import _native as N
from noisyquantumsimulator_amd import engine as E
from oracle import lindblad_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-10


@pytest.fixture(scope="module")
def eng():
    return E.Engine()


def _run_cfg(eng, cfg):
    warnings.simplefilter("ignore")
    b = derive(cfg)
    p = E.pack_params(b)
    key = E.protocol_key(b)
    evol = "lindblad" if b.include_noise else "ket"
    shape = b.pulse_shape.lower() if key == "lp_shaped" else "square"
    return b, E.Engine.run(eng, p, key, evol, shape=shape)


FIXTURES = ["lp_medium_nf", "smooth_medium_nf", "lp_high_nf", "lp_low_nf", "smooth_high_nf",
            "smooth_low_nf", "lp_medium_noisy", "smooth_medium_noisy", "bangbang_medium_noisy",
            "bangbang_medium_nf", "lp_cosine_noisy", "lp_gaussian_nf", "lp_cs133_noisy",
            "lp_nonclock_trapoff_noisy", "lp_850nm_hot_noisy", "smooth_override_noisy",
            "lp_override_noisy"]


@pytest.mark.parametrize("name", FIXTURES)
def test_states_match_oracle(eng, evolution_golden, name):
    e = evolution_golden[name]
    b, r = _run_cfg(eng, e["config"])
    assert r.status[0] == 0
    ref = states_from_fixture(e)
    got = r.rho()[0] if r.evolution == "lindblad" else r.kets()[0]
    for k, lab in enumerate(O.LABELS):
        np.testing.assert_allclose(got[k], ref[lab], atol=TOL, rtol=0, err_msg=f"{name}/{lab}")
    # gauge-invariant fidelity outputs
    fid, avg, info = O.cz_fidelity(ref)
    pops = r.populations()[0]
    for k, lab in enumerate(O.LABELS):
        want = fid[lab] if lab != "11" else info["F11_population"]
        assert abs(pops[k] - want) < TOL
    if r.evolution == "ket":
        assert abs(r.col("AVG_F")[0] - avg) < TOL
        assert abs(r.col("PENALTY")[0] - info["cz_phase_fidelity"]) < TOL


@pytest.mark.parametrize("name", ["lp_medium_nf", "smooth_medium_nf", "lp_high_nf", "lp_low_nf",
                                  "smooth_high_nf", "smooth_low_nf"])
def test_published_numbers_through_engine(eng, evolution_golden, name):
    """The reference notebooks' published fidelities, straight from the GPU summary."""
    e = evolution_golden[name]
    b, r = _run_cfg(eng, e["config"])
    got = dict(avg=r.col("AVG_F")[0], F11=r.col("POP0")[0] * 0 + r.summary[N.S["POP0"] + 3][0]
               * r.col("PENALTY")[0], cz_phase_fidelity=r.col("PENALTY")[0],
               phase_error_deg=np.degrees(min(abs(r.col("CTRL_PHASE")[0] - np.pi),
                                              abs(r.col("CTRL_PHASE")[0] + np.pi))),
               controlled_phase_deg=abs(np.degrees(r.col("CTRL_PHASE")[0])))
    for key, (val, digits) in e["published"].items():
        if key in got:
            assert round(float(got[key]), digits) == pytest.approx(val, abs=0.51 * 10 ** (-digits)), key


def test_row5_populations(eng, evolution_golden):
    e = evolution_golden["lp_row5_physics"]
    d = e["derived"]
    p = np.zeros((N.NPARAM, 1))
    p[N.P["OMEGA"]], p[N.P["V"]], p[N.P["DELTA"]] = d["Omega"], d["V"], d["Delta_gate"]
    p[N.P["TAU"]], p[N.P["XI_RE"]], p[N.P["XI_IM"]] = d["tau_single"], d["xi_re"], d["xi_im"]
    r = eng.run(p, "lp_square", "ket")
    pops = r.populations()[0]
    assert round(pops[3], 8) == pytest.approx(0.99999617, abs=6e-9)
    assert round(pops.mean(), 8) == pytest.approx(0.99999904, abs=6e-9)


def _random_points(rng, n, protocol):
    p = np.zeros((N.NPARAM, n))
    Om = 2 * np.pi * rng.uniform(1e6, 10e6, n)
    p[N.P["OMEGA"]] = Om
    p[N.P["V"]] = Om * 10 ** rng.uniform(1, 3, n)
    p[N.P["DELTA1"]] = 2 * np.pi * rng.uniform(0, 3e5, n)
    for k, hi in (("G1", 2e4), ("G0", 5e4), ("GPHI", 1e5), ("GSC", 5e5)):
        p[N.P[k + "_A"]] = rng.uniform(0, hi, n)
        p[N.P[k + "_B"]] = rng.uniform(0, hi, n)
    if protocol == "lp_square":
        dl = rng.uniform(0.3, 0.45, n) * Om
        tau = 4.29268 / Om
        xi = np.exp(1j * rng.uniform(0, 2 * np.pi, n))
        p[N.P["DELTA"]], p[N.P["TAU"]] = dl, tau
        p[N.P["XI_RE"]], p[N.P["XI_IM"]] = xi.real, xi.imag
    elif protocol == "smooth_jp":
        p[N.P["DELTA"]] = -0.0205 * Om
        p[N.P["TAU"]] = rng.uniform(5, 12, n) / Om
        p[N.P["A"]] = 0.311 * np.pi
        p[N.P["OMEGA_MOD"]] = 1.242 * Om
        p[N.P["PHI_OFF"]] = 4.696
    elif protocol == "bangbang":
        p[N.P["OMEGA_TAU"]] = 22.08
        p[N.P["NSEG"]] = 5
        st = np.sort(rng.uniform(0, 22.08, (n, 4)), axis=1)
        st[:, 1] = st[:, 0]            # a zero-length segment (skipped, :1902-1903)
        p[N.P["SWT0"]:N.P["SWT0"] + 4] = st.T
        p[N.P["PHI0"]:N.P["PHI0"] + 5] = rng.uniform(-np.pi, np.pi, (5, n))
    return p


def _oracle_point(p, i, protocol, n_steps=300, shape="cosine"):
    g = lambda k: p[N.P[k], i]
    I3 = np.eye(3)
    ops = []
    for atom in ("A", "B"):
        emb = (lambda o: np.kron(o, I3)) if atom == "A" else (lambda o: np.kron(I3, o))
        for key, op in (("G1", np.outer(np.eye(3)[1], np.eye(3)[2])),
                        ("G0", np.outer(np.eye(3)[0], np.eye(3)[2])),
                        ("GPHI", np.diag([0, 0, 1.0])), ("GSC", np.diag([0, 1.0, 0]))):
            rate = g(f"{key}_{atom}")
            if rate > 0:
                ops.append(np.sqrt(rate) * emb(op.astype(complex)))
    kw = dict(Omega=g("OMEGA"), V=g("V"), delta_zeeman=g("DELTA1"), c_ops=ops)
    if protocol == "lp_square":
        spec = O.PointSpec(protocol="lp_square", Delta=g("DELTA"), tau=g("TAU"),
                           xi=complex(g("XI_RE"), g("XI_IM")), **kw)
    elif protocol == "smooth_jp":
        spec = O.PointSpec(protocol="smooth_jp", Delta=g("DELTA"), tau=g("TAU"), A=g("A"),
                           omega_mod=g("OMEGA_MOD"), phi_offset=g("PHI_OFF"), n_steps=n_steps, **kw)
    else:
        nseg = int(g("NSEG"))
        spec = O.PointSpec(protocol="bangbang", omega_tau=g("OMEGA_TAU"),
                           switching_times=[p[N.P["SWT0"] + k, i] for k in range(nseg - 1)],
                           phases=[p[N.P["PHI0"] + k, i] for k in range(nseg)], **kw)
    return O.run_point(spec)


@pytest.mark.parametrize("protocol", ["lp_square", "smooth_jp", "bangbang"])
def test_random_points_asymmetric_atoms(eng, protocol):
    """Different rates on the two atoms (C1-style single-atom collapse ops)."""
    rng = np.random.default_rng(20260215)
    n = 3
    p = _random_points(rng, n, protocol)
    r = eng.run(p, protocol, "lindblad", n_steps=60 if protocol == "smooth_jp" else None)
    rho = r.rho()
    for i in range(n):
        ref = _oracle_point(p, i, protocol, n_steps=60)
        for k, lab in enumerate(O.LABELS):
            np.testing.assert_allclose(rho[i, k], ref[lab], atol=TOL, rtol=0)


def test_c1_single_collapse_op(eng):
    """C1: one jump sqrt(gamma)(|1><r| (x) I), gamma = 1/140 us (BASELINE.json configs[0])."""
    Om = 2 * np.pi * 5e6
    p = np.zeros((N.NPARAM, 1))
    dl = 0.377371 * Om
    tau = 4.29268 / Om
    from noisyquantumsimulator_amd.protocols import compute_phase_shift_xi
    xi = complex(compute_phase_shift_xi(dl, Om, tau))
    p[N.P["OMEGA"]], p[N.P["V"]], p[N.P["DELTA"]], p[N.P["TAU"]] = Om, 100 * Om, dl, tau
    p[N.P["XI_RE"]], p[N.P["XI_IM"]] = xi.real, xi.imag
    p[N.P["G1_A"]] = 7142.857
    r = eng.run(p, "lp_square", "lindblad")
    ref = _oracle_point(p, 0, "lp_square")
    for k, lab in enumerate(O.LABELS):
        np.testing.assert_allclose(r.rho()[0, k], ref[lab], atol=TOL, rtol=0)


def test_batch_properties_large(eng):
    """Size-independent properties at the C2 bench size (10k points)."""
    rng = np.random.default_rng(7)
    n = 10_000
    p = _random_points(rng, n, "lp_square")
    for k in ("G1", "G0", "GPHI", "GSC"):
        p[N.P[k + "_B"]] = p[N.P[k + "_A"]]
    r = eng.run(p, "lp_square", "lindblad")
    assert np.all(r.status == 0)
    rho = r.rho()
    tr = np.einsum("nkaa->nk", rho)
    np.testing.assert_allclose(tr, 1.0, atol=1e-11)                   # jumps preserve the trace
    np.testing.assert_allclose(rho, np.conj(np.swapaxes(rho, -1, -2)), atol=1e-15)  # Hermitian
    w = np.linalg.eigvalsh(rho[:500])
    assert w.min() > -1e-11                                           # positive
    pops = r.populations()
    assert np.all((pops > -1e-12) & (pops < 1 + 1e-12))
    # batch-position independence (bitwise): a shuffled sub-batch reproduces its rows
    idx = rng.permutation(n)[:777]
    r2 = eng.run(p[:, idx], "lp_square", "lindblad")
    np.testing.assert_array_equal(r2.state, r.state.reshape(25, n, 4)[:, idx, :].reshape(25, -1))
    # spot-check against the oracle
    for i in (0, n // 2, n - 1):
        ref = _oracle_point(p, i, "lp_square")
        for k, lab in enumerate(O.LABELS):
            np.testing.assert_allclose(rho[i, k], ref[lab], atol=TOL, rtol=0)


def test_edge_cases(eng):
    rng = np.random.default_rng(3)
    p = _random_points(rng, 37, "lp_square")          # not a multiple of 16 points
    p[N.P["OMEGA"], 5] = 0.0                            # invalid point -> status bit, batch survives
    p[N.P["TAU"], 9] = -1.0
    r = eng.run(p, "lp_square", "lindblad")
    assert r.status[5] & N.STATUS_BAD_INPUT and r.status[9] & N.STATUS_BAD_INPUT
    ok = np.ones(37, bool)
    ok[[5, 9]] = False
    assert np.all(r.status[ok] == 0)
    e0 = eng.run(np.zeros((N.NPARAM, 0)), "lp_square", "lindblad")   # empty batch
    assert e0.state.shape == (25, 0)
    one = eng.run(p[:, :1], "lp_square", "ket")
    assert one.status[0] == 0 and abs(np.linalg.norm(one.kets()[0, 3]) - 1) < 1e-12


@pytest.mark.parametrize("protocol,n_steps", [("lp_square", None), ("bangbang", None),
                                              ("smooth_jp", 30), ("smooth_jp", 300)])
@pytest.mark.parametrize("symmetric", [True, False])
def test_squaring_and_vector_methods_agree(eng, protocol, n_steps, symmetric):
    """The propagator-squaring kernel and the per-input vector kernel are two
    independent evaluations of the same exact propagator."""
    rng = np.random.default_rng(11)
    p = _random_points(rng, 45, protocol)           # 45 = 4.5 blocks of 10 points: ragged tail
    if symmetric:
        for k in ("G1", "G0", "GPHI", "GSC"):
            p[N.P[k + "_B"]] = p[N.P[k + "_A"]]
    rv = eng.run(p, protocol, "lindblad", n_steps=n_steps, method="cheb_vector")
    rs = eng.run(p, protocol, "lindblad", n_steps=n_steps, method="cheb_squaring")
    assert np.all(rv.status == 0) and np.all(rs.status == 0)
    np.testing.assert_allclose(rs.state, rv.state, atol=1e-11, rtol=0)
    np.testing.assert_allclose(rs.populations(), rv.populations(), atol=1e-11, rtol=0)
    assert np.all(rv.col("NSQUARE") == 0)
    if protocol != "smooth_jp":          # short smooth-JP segments (x < X_BASE) need none
        assert np.all(rs.col("NSQUARE") > 0)
    ref = _oracle_point(p, 44, protocol, n_steps=n_steps or 300)
    for k, lab in enumerate(O.LABELS):
        np.testing.assert_allclose(rs.rho()[44, k], ref[lab], atol=TOL, rtol=0)
    if symmetric:
        # the 16-lane DPP-row kernel (auto method for identical atoms: segment order, inlined
        # sin/cos, angle recurrence, LDS zero words) is a third evaluation of the same map
        r16 = eng.run(p, protocol, "lindblad", n_steps=n_steps, method="chebyshev")
        assert np.all(r16.status == 0)
        np.testing.assert_allclose(r16.state, rv.state, atol=1e-11, rtol=0)
        np.testing.assert_allclose(r16.populations(), rv.populations(), atol=1e-11, rtol=0)


def test_lp_phase_frame_fallback_for_non_unit_xi(eng):
    """LP square runs both pulses off ONE propagator (pulse 2 = pulse 1 in the frame
    rotated by arg xi) when |xi| = 1, as compute_phase_shift_xi guarantees.  An ABI
    caller may pass any xi: a block holding a non-unit xi builds both propagators
    (NSQUARE doubles for its 10 points) and still matches the vector kernel."""
    rng = np.random.default_rng(5)
    p = _random_points(rng, 25, "lp_square")
    base = eng.run(p, "lp_square", "lindblad", method="cheb_squaring")
    q = p.copy()
    q[N.P["XI_RE"], 13] *= 1.01
    q[N.P["XI_IM"], 13] *= 1.01
    rs = eng.run(q, "lp_square", "lindblad", method="cheb_squaring")
    rv = eng.run(q, "lp_square", "lindblad", method="cheb_vector")
    assert np.all(rs.status == 0)
    np.testing.assert_allclose(rs.state, rv.state, atol=1e-11, rtol=0)
    nb, nq = base.col("NSQUARE"), rs.col("NSQUARE")
    blk = (np.arange(25) // 10 == 1) & (np.arange(25) != 13)   # 13's pulse 2 has a new x
    np.testing.assert_array_equal(nq[blk], 2 * nb[blk])
    out = np.arange(25) // 10 != 1
    np.testing.assert_array_equal(nq[out], nb[out])
    others = np.ones(25, bool)
    others[13] = False
    np.testing.assert_allclose(rs.state.reshape(25, 25, 4)[:, others],
                               base.state.reshape(25, 25, 4)[:, others], atol=1e-12, rtol=0)
    ref = _oracle_point(q, 13, "lp_square")
    for k, lab in enumerate(O.LABELS):
        np.testing.assert_allclose(rs.rho()[13, k], ref[lab], atol=TOL, rtol=0)


def test_multi_device_handle_range_partition():
    """ryd_run_batch range-partitions a batch over the handle's devices; on a 1-GPU box
    the same device twice exercises the partition (two streams, two shards)."""
    rng = np.random.default_rng(5)
    p = _random_points(rng, 1001, "lp_square")
    for k in ("G1", "G0", "GPHI", "GSC"):
        p[N.P[k + "_B"]] = p[N.P[k + "_A"]]
    one = E.Engine([0]).run(p, "lp_square", "lindblad")
    two = E.Engine([0, 0]).run(p, "lp_square", "lindblad")
    np.testing.assert_array_equal(one.state, two.state)
    np.testing.assert_array_equal(one.summary, two.summary)


@pytest.mark.parametrize("protocol,n_steps", [("lp_square", None), ("bangbang", None),
                                              ("smooth_jp", 3), ("smooth_jp", 20)])
def test_dopri5_reference_stepper(eng, protocol, n_steps):
    """The adaptive RK45 (Dormand-Prince) mode agrees with the exact propagator to its
    tolerance; the step cap raises the STEP_CAP status bit instead of failing the batch."""
    rng = np.random.default_rng(13)
    p = _random_points(rng, 8, protocol)
    p[N.P["OMEGA"]] = 2 * np.pi * 8e6       # keep the run short: V*tau ~ 1e2-1e3 rad
    if protocol == "lp_square":
        p[N.P["TAU"]] = 4.29268 / p[N.P["OMEGA"]]
    r = eng.run(p, protocol, "lindblad", n_steps=n_steps, method="dopri5", rtol=1e-11, atol=1e-13)
    ex = eng.run(p, protocol, "lindblad", n_steps=n_steps, method="cheb_vector")
    assert np.all(r.status == 0)
    np.testing.assert_allclose(r.state, ex.state, atol=2e-8, rtol=0)
    np.testing.assert_allclose(r.populations(), ex.populations(), atol=2e-9, rtol=0)
    assert r.matvec_useful > 5 * ex.matvec_useful / 4      # stepper needs many more RHS calls
    capped = eng.run(p[:, :2], protocol, "lindblad", n_steps=n_steps, method="dopri5", max_steps=5)
    assert np.all(capped.status & N.STATUS_STEP_CAP)


def test_sym16_invalid_waves_and_phase_range(eng):
    """Identical-atom (sym16) edge cases: a whole wave of invalid points (segment 0 still
    builds, identity rows) beside valid waves; a smooth-JP point whose laser-phase
    argument leaves the inlined sin/cos range (|x| >= 1e15) is flagged NONFINITE alone,
    the rest of its wave unaffected and equal to a clean run."""
    rng = np.random.default_rng(29)
    for protocol, ns in (("lp_square", None), ("bangbang", None)):
        p = _random_points(rng, 12, protocol)
        for k in ("G1", "G0", "GPHI", "GSC"):
            p[N.P[k + "_B"]] = p[N.P[k + "_A"]]
        assert E.symmetric_atoms(p)
        p[N.P["OMEGA"], 4:8] = 0.0                        # the second wave: all invalid
        r = eng.run(p, protocol, "lindblad", n_steps=ns)
        assert np.all(r.status[4:8] & N.STATUS_BAD_INPUT)
        ok = np.r_[0:4, 8:12]
        assert np.all(r.status[ok] == 0)
        clean = eng.run(p[:, ok].copy(), protocol, "lindblad", n_steps=ns)
        np.testing.assert_array_equal(clean.state, r.state.reshape(25, 12, 4)[:, ok].reshape(25, -1))
    p = _random_points(rng, 8, "smooth_jp")
    for k in ("G1", "G0", "GPHI", "GSC"):
        p[N.P[k + "_B"]] = p[N.P[k + "_A"]]
    base = eng.run(p, "smooth_jp", "lindblad", n_steps=60)
    assert np.all(base.status == 0)
    p[N.P["OMEGA_MOD"], 2] = 1e25                          # phase argument ~1e19 rad
    r = eng.run(p, "smooth_jp", "lindblad", n_steps=60)
    assert r.status[2] & N.STATUS_NONFINITE
    others = [i for i in range(8) if i != 2]
    assert np.all(r.status[others] == 0)
    st = r.state.reshape(25, 8, 4)
    np.testing.assert_array_equal(st[:, others], base.state.reshape(25, 8, 4)[:, others])
