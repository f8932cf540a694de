"""The default noise-free ket method (ket_block_kernel: exact 2x2 / 3x3 block
propagators in the phase frame, one lane per point) against the 4-lane Chebyshev
state-vector kernel (method="cheb_vector", the round-2 path) and the expm oracle, for
every protocol, dim 3 and 4, including the step-cap and invalid-input status bits."""
import warnings

import numpy as np
import pytest

from noisyquantumsimulator_amd import configurations as CF
from noisyquantumsimulator_amd import engine as E
from noisyquantumsimulator_amd import physics as PH
from noisyquantumsimulator_amd import sweeps as SW
from oracle import lindblad_oracle as O
import oracle_evaluator as OE

pytestmark = pytest.mark.gpu
TOL = 1e-10


def _grid(kind, n=96, dim=3):
    warnings.simplefilter("ignore")
    exc = SW.medium_excitation(1.0)
    rng = np.random.default_rng(7)
    ref = PH.derive_batch(CF.LPSimulationInputs(excitation=exc), **SW._apparatus_kwargs(), include_noise=False)
    p2 = SW.MEDIUM["laser_2_power"] * (rng.uniform(1, 10, n) / (ref["Omega"][0] / (2e6 * np.pi))) ** 2
    sf = rng.uniform(2.0, 5.0, n)
    kw = dict(**SW._apparatus_kwargs(spacing_factor=sf), include_noise=False, hilbert_space_dim=dim)
    if kind == "lp_square":
        si = CF.LPSimulationInputs(excitation=exc)
        over = dict(laser_2_power=p2, delta_over_omega=rng.uniform(0.2, 0.5, n), omega_tau=rng.uniform(3.5, 5.5, n))
    elif kind in ("cosine", "gaussian"):
        si = CF.LPSimulationInputs(excitation=exc, pulse_shape=kind)
        over = dict(laser_2_power=p2)
    elif kind == "smooth_jp":
        si = CF.SmoothJPSimulationInputs(excitation=exc)
        over = dict(laser_2_power=p2, omega_tau=rng.uniform(5, 25, n), A=rng.uniform(0.2, 3.0, n))
    else:
        si = CF.JPSimulationInputs(excitation=exc)
        over = dict(laser_2_power=p2)
    return PH.derive_batch(si, n=n, overrides=over, **kw)


@pytest.mark.parametrize("kind", ["lp_square", "smooth_jp", "bangbang", "cosine", "gaussian"])
@pytest.mark.parametrize("dim", [3, 4])
def test_block_kets_match_chebyshev_kets(kind, dim):
    b = _grid(kind, dim=dim)
    p = E.pack_params(b)
    key = E.protocol_key(b)
    shape = b.pulse_shape.lower() if key == "lp_shaped" else "square"
    eng = E.Engine()
    rb = eng.run(p, key, "ket", shape=shape, dim=dim)
    rc = eng.run(p, key, "ket", shape=shape, dim=dim, method="cheb_vector")
    assert np.all(rb.status == 0) and np.all(rc.status == 0)
    assert np.abs(rb.state - rc.state).max() < TOL
    for c in ("POP0", "AVG_POP", "AVG_F", "PENALTY", "TRACE11"):
        np.testing.assert_allclose(rb.col(c), rc.col(c), atol=TOL, rtol=0, err_msg=c)
    cp = np.angle(np.exp(1j * (rb.col("CTRL_PHASE") - rc.col("CTRL_PHASE"))))
    assert np.abs(cp).max() < 1e-9
    assert np.all(rb.col("NSQUARE") >= 1)                      # propagator builds per point
    if key in ("lp_square", "smooth_jp"):
        assert np.all(rb.col("NSQUARE") == 1)                  # phase frame: one build


@pytest.mark.parametrize("kind", ["lp_square", "smooth_jp", "bangbang"])
def test_block_kets_match_oracle(kind):
    b = _grid(kind, n=6)
    p = E.pack_params(b)
    key = E.protocol_key(b)
    r = E.Engine().run(p, key, "ket")
    kets = r.kets()
    for i in range(b.n):
        ref = O.run_point(OE.point_spec(b, i, n_steps=300))
        for k, lab in enumerate(O.LABELS):
            assert np.abs(kets[i, k] - ref[lab]).max() < TOL, (kind, i, lab)


def test_block_kets_status_bits():
    b = _grid("lp_square", n=4)
    p = E.pack_params(b)
    P = E.N.P
    p[P["TAU"], 1] = 1e3                       # 2e6 rad cap (mesolve nsteps analogue)
    p[P["OMEGA"], 2] = -1.0                    # invalid input
    eng = E.Engine()
    rb = eng.run(p, "lp_square", "ket")
    rc = eng.run(p, "lp_square", "ket", method="cheb_vector")
    np.testing.assert_array_equal(rb.status, rc.status)
    assert rb.status[1] & E.N.STATUS_STEP_CAP and rb.status[2] & E.N.STATUS_BAD_INPUT
    assert rb.status[0] == 0 and rb.status[3] == 0
