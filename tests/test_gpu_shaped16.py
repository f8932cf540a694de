"""LP shaped (RG/simulation.py:2099-2231) on the 16-lane DPP-row kernel (ryd_shaped16.inc,
round 5) against the expm oracle and against the one-lane-per-input Chebyshev kernel it
replaces (RYD_SHAPED16=0), on a ragged batch with per-point series lengths.  Tolerance
1e-10 absolute on rho elements, as the other parity tests."""
import os
import warnings

import numpy as np
import pytest

import oracle_evaluator as OE
from noisyquantumsimulator_amd import configurations as CF
from noisyquantumsimulator_amd import engine as E
from noisyquantumsimulator_amd import physics as PH
from oracle import lindblad_oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-10


@pytest.fixture(scope="module")
def eng():
    return E.Engine()


def _batch(n, shape="cosine"):
    warnings.simplefilter("ignore")
    return PH.derive_batch(CF.LPSimulationInputs(pulse_shape=shape), n, species="Rb87", n_rydberg=70,
                           temperature=np.linspace(2e-6, 4e-5, n), spacing_factor=2.8,
                           overrides=dict(laser_2_power=np.geomspace(0.02, 2.0, n)))


@pytest.mark.parametrize("shape", ["cosine", "gaussian"])
def test_shaped16_matches_oracle_and_old_kernel(eng, shape):
    n = 7                                                   # two waves, the second ragged
    b = _batch(n, shape)
    p = E.pack_params(b)
    r = eng.run(p, "lp_shaped", "lindblad", shape=shape)      # the reference's 500 steps
    assert np.all(r.status == 0)
    os.environ["RYD_SHAPED16"] = "0"
    try:
        old = eng.run(p, "lp_shaped", "lindblad", shape=shape)
    finally:
        del os.environ["RYD_SHAPED16"]
    np.testing.assert_allclose(r.state, old.state, atol=TOL, rtol=0)
    np.testing.assert_allclose(r.populations(), old.populations(), atol=TOL, rtol=0)
    rho = r.rho()
    for i in (0, n - 1):
        ref = O.run_point(OE.point_spec(b, i))
        for k, lab in enumerate(O.LABELS):
            np.testing.assert_allclose(rho[i, k], ref[lab], atol=TOL, rtol=0, err_msg=f"{shape}/{i}/{lab}")


def test_shaped16_rows_independent_of_their_wave(eng):
    b = _batch(6)
    p = E.pack_params(b)
    r = eng.run(p, "lp_shaped", "lindblad", shape="cosine", n_steps=40)
    for i in (1, 5):
        one = eng.run(p[:, i:i + 1].copy(), "lp_shaped", "lindblad", shape="cosine", n_steps=40)
        np.testing.assert_array_equal(one.state[:, :4], r.state[:, 4 * i:4 * i + 4])


@pytest.mark.parametrize("n_steps", [3, 40])
def test_shaped16_coarse_schedule_substeps(eng, n_steps):
    """Segments whose series argument exceeds SH_XSUB are taken in equal sub-steps (rows of a
    wave with different counts): same states as the per-lane kernel, no STEP_CAP."""
    b = _batch(7)
    p = E.pack_params(b)
    r = eng.run(p, "lp_shaped", "lindblad", shape="cosine", n_steps=n_steps)
    assert np.all(r.status == 0)
    os.environ["RYD_SHAPED16"] = "0"
    try:
        old = eng.run(p, "lp_shaped", "lindblad", shape="cosine", n_steps=n_steps)
    finally:
        del os.environ["RYD_SHAPED16"]
    np.testing.assert_allclose(r.state, old.state, atol=TOL, rtol=0)


@pytest.mark.parametrize("shape,n_steps", [("square", 2), ("blackman", 2), ("cosine", 2), ("blackman", 500)])
def test_shaped16_every_shape_and_the_shortest_schedule(eng, shape, n_steps):
    """The four envelope names (square / gaussian / blackman take the scalar-t envelope 1,
    RG/simulation.py:2179-2220) and n_steps = 2 (one segment per pulse, sub-stepped): the
    same states as the per-lane kernel."""
    b = _batch(5)
    p = E.pack_params(b)
    r = eng.run(p, "lp_shaped", "lindblad", shape=shape, n_steps=n_steps)
    assert np.all(r.status == 0)
    os.environ["RYD_SHAPED16"] = "0"
    try:
        old = eng.run(p, "lp_shaped", "lindblad", shape=shape, n_steps=n_steps)
    finally:
        del os.environ["RYD_SHAPED16"]
    np.testing.assert_allclose(r.state, old.state, atol=TOL, rtol=0)
