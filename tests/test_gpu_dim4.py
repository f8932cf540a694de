"""hilbert_space_dim=4 (|0>, |1>, |r+>, |r->; SURVEY.md §8 a2/a3 dim-4 notes) on the GPU
against the expm oracle: the 36-dim Lindblad sector kernel, the embedded ket path,
and the simulate_CZ_gate drop-in."""
import warnings

import numpy as np
import pytest

import oracle_evaluator as OE
from noisyquantumsimulator_amd import configurations as CF
from noisyquantumsimulator_amd import engine as E
from noisyquantumsimulator_amd import physics as PH
from noisyquantumsimulator_amd import simulation as SIM
from oracle import lindblad_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-10
KW = dict(species="Rb87", n_rydberg=70, tweezer_power=0.020, tweezer_waist=0.8e-6, temperature=2e-6,
          spacing_factor=2.8, B_field=1e-4, NA=0.5)


def _exc(purity=0.95):
    return CF.TwoPhotonExcitationConfig(
        laser_1=CF.LaserParameters(power=50e-6, waist=50e-6, polarization="pi", polarization_purity=purity),
        laser_2=CF.LaserParameters(power=0.3, waist=50e-6, polarization="sigma+", polarization_purity=purity))


@pytest.fixture(scope="module")
def eng():
    return E.Engine()


@pytest.mark.parametrize("si", [CF.LPSimulationInputs, CF.SmoothJPSimulationInputs, CF.JPSimulationInputs])
@pytest.mark.parametrize("noisy", [True, False])
def test_dim4_states_match_oracle(eng, si, noisy):
    warnings.simplefilter("ignore")
    b = PH.derive_batch(si(excitation=_exc()), 3, hilbert_space_dim=4, include_noise=noisy,
                        **dict(KW, temperature=np.array([1e-6, 5e-6, 2e-5])))
    if noisy:
        assert np.all(b["mJ_leakage_rate"] > 0)
    key = E.protocol_key(b)
    r = eng.run(E.pack_params(b), key, "lindblad" if noisy else "ket", dim=4,
                n_steps=60 if key == "smooth_jp" else None)
    assert np.all(r.status == 0)
    got = r.rho() if noisy else r.kets()
    for i in range(b.n):
        spec = OE.point_spec(b, i, n_steps=60)
        ref = O.run_point(spec)
        for k, lab in enumerate(O.LABELS):
            np.testing.assert_allclose(got[i, k], ref[lab], atol=TOL, rtol=0, err_msg=f"{key}/{i}/{lab}")


def test_dim4_asymmetric_rates_and_trace(eng):
    """Different mJ rates on the two atoms; trace and positivity of every rho."""
    warnings.simplefilter("ignore")
    b = PH.derive_batch(CF.LPSimulationInputs(excitation=_exc()), 64, hilbert_space_dim=4,
                        **dict(KW, temperature=np.linspace(1e-6, 3e-5, 64)))
    p = E.pack_params(b)
    p[E.N.P["GMJ_B"]] *= 3.0
    r = eng.run(p, "lp_square", "lindblad", dim=4)
    rho = r.rho()
    np.testing.assert_allclose(np.einsum("nkaa->nk", rho), 1.0, atol=1e-11)
    assert np.linalg.eigvalsh(rho).min() > -1e-11
    # the r- populations are fed only by mJ mixing: positive, and larger on atom B
    pm = rho[..., 3 * 4 + 0, 3 * 4 + 0].real          # |r- 0> population of input |10>-type states
    assert np.all(pm[:, 2:] >= -1e-15)


def test_simulate_cz_gate_dim4_drop_in():
    warnings.simplefilter("ignore")
    si = CF.LPSimulationInputs(excitation=_exc(0.99))
    res = SIM.simulate_CZ_gate(si, hilbert_space_dim=4, **KW)
    assert res.hilbert_space_dim == 4 and res.results["11"].shape == (16, 16)
    assert res.noise_breakdown["n_collapse_ops"] == len(res.c_ops) == 30
    assert res.H1.shape == (16, 16)
    b = PH.derive_batch(si, hilbert_space_dim=4, **KW)
    ref = O.run_point(OE.point_spec(b, 0))
    for lab in O.LABELS:
        np.testing.assert_allclose(res.results[lab], ref[lab], atol=TOL, rtol=0)
    fid, avg, info = O.cz_fidelity(ref, dim=4)
    for lab in ("00", "01", "10"):
        assert abs(res.fidelities[lab] - fid[lab]) < TOL
    # noise-free dim 4 = dim 3 embedded (|r-> never driven)
    r4 = SIM.simulate_CZ_gate(si, hilbert_space_dim=4, include_noise=False, **KW)
    r3 = SIM.simulate_CZ_gate(si, hilbert_space_dim=3, include_noise=False, **KW)
    assert abs(r4.avg_fidelity - r3.avg_fidelity) < 1e-13


def test_dim4_rows_are_independent_of_their_wave(eng):
    """The DPP-row kernel holds 4 points per wave with per-row squaring depths: a ragged
    batch of 9 points (Omega spread over a decade: different depths in one wave) gives each
    point the bits it gets alone, and the oracle's states at 1e-10."""
    warnings.simplefilter("ignore")
    n = 9
    b = PH.derive_batch(CF.LPSimulationInputs(excitation=_exc()), n, hilbert_space_dim=4,
                        **dict(KW, temperature=np.linspace(1e-6, 3e-5, n)),
                        overrides=dict(laser_2_power=np.geomspace(0.03, 3.0, n)))
    p = E.pack_params(b)
    r = eng.run(p, "lp_square", "lindblad", dim=4)
    assert np.all(r.status == 0)
    assert len(set(r.col("NSQUARE").tolist())) > 1              # different depths in the batch
    for i in (0, 4, 8):
        one = eng.run(p[:, i:i + 1].copy(), "lp_square", "lindblad", dim=4)
        np.testing.assert_array_equal(one.state[:, :4], r.state[:, 4 * i:4 * i + 4])
        ref = O.run_point(OE.point_spec(b, i))
        for k, lab in enumerate(O.LABELS):
            np.testing.assert_allclose(r.rho()[i, k], ref[lab], atol=TOL, rtol=0, err_msg=f"{i}/{lab}")
