"""simulate_CZ_gate / simulate_CZ_gate_batch end to end on the GPU engine."""
import warnings

import numpy as np
import pytest

from conftest import states_from_fixture
from golden_configs import simulate_kwargs, simulation_inputs
from noisyquantumsimulator_amd import configurations as CF
from noisyquantumsimulator_amd import simulation as SIM
from oracle import lindblad_oracle as O

pytestmark = pytest.mark.gpu


def test_published_lp_medium(evolution_golden):
    warnings.simplefilter("ignore")
    cfg = evolution_golden["lp_medium_nf"]["config"]
    r = SIM.simulate_CZ_gate(simulation_inputs(cfg), **simulate_kwargs(cfg))
    assert isinstance(r, SIM.SimulationResult)
    assert round(r.avg_fidelity, 6) == 0.994423
    assert round(r.fidelities["11"], 6) == 0.977897
    assert round(r.phase_info["cz_phase_fidelity"], 6) == 0.978587
    assert round(r.phase_info["phase_error_from_pi_deg"], 2) == 16.83
    assert round(r.gate_time_us, 3) == 0.379
    assert round(r.V_over_Omega, 1) == 342.5
    assert round(r.Omega_MHz, 3) == 3.602
    assert r.n_pulses == 2 and r.protocol == "levine_pichler" and r.H1.shape == (9, 9)
    assert r.results["11"].shape == (9,)          # kets (no c_ops)


def test_noisy_point_matches_fixture(evolution_golden):
    warnings.simplefilter("ignore")
    e = evolution_golden["lp_medium_noisy"]
    cfg = e["config"]
    r = SIM.simulate_CZ_gate(simulation_inputs(cfg), **simulate_kwargs(cfg), eigh="numpy")
    ref = states_from_fixture(e)
    for lab in O.LABELS:
        assert r.results[lab].shape == (9, 9)
        np.testing.assert_allclose(r.results[lab], ref[lab], atol=1e-10)
    assert len(r.c_ops) == 14 and r.noise_breakdown["n_collapse_ops"] == 14
    assert r.phase_info["F11_population"] == pytest.approx(ref["11"][4, 4].real, abs=1e-10)
    # The mixed-state phase penalty takes the phase of LAPACK's dominant eigenvector,
    # a gauge that flips under 1e-14 perturbations of rho (SURVEY.md hard part 3;
    # observed on MI355X hosts: fixture states -> 0.9514, GPU states equal to 1e-14
    # -> 0.9057).  The reference's own avg_fidelity is ill-conditioned there, so the
    # pipeline is graded for consistency: the oracle's compute_CZ_fidelity on OUR
    # states, plus every gauge-invariant output against the fixture.
    _, avg_ours, _ = O.cz_fidelity(r.results, eigh=np.linalg.eigh)
    assert r.avg_fidelity == pytest.approx(avg_ours, abs=1e-12)
    pops = [r.phase_info["pop_00"], r.phase_info["pop_01"]]
    np.testing.assert_allclose(pops, [e["fidelities"]["00"], e["fidelities"]["01"]], atol=1e-10)


def test_dict_return_and_defaults():
    warnings.simplefilter("ignore")
    for si in (CF.LPSimulationInputs(), CF.SmoothJPSimulationInputs(), CF.JPSimulationInputs()):
        d = SIM.simulate_CZ_gate(si, return_dataclass=False)
        assert 0.0 < d["avg_fidelity"] <= 1.0
        assert d["gate_time_us"] == pytest.approx(d["tau_total"] * 1e6)


def test_batch_equals_single_points():
    warnings.simplefilter("ignore")
    T = np.array([2e-6, 10e-6, 50e-6])
    Ptw = np.array([0.01, 0.03, 0.06])
    si = CF.LPSimulationInputs()
    br = SIM.simulate_CZ_gate_batch(si, temperature=T, tweezer_power=Ptw, eigh="numpy")
    for i in range(3):
        r = SIM.simulate_CZ_gate(si, temperature=T[i], tweezer_power=Ptw[i], eigh="numpy")
        assert br.avg_fidelity[i] == pytest.approx(r.avg_fidelity, abs=1e-12)
        np.testing.assert_allclose(br.populations[i],
                                   [r.phase_info["pop_00"], r.phase_info["pop_01"],
                                    np.real(r.results["10"][3, 3]), r.phase_info["F11_population"]],
                                   atol=1e-13)


def test_shape_errors_like_reference():
    warnings.simplefilter("ignore")
    with pytest.raises(TypeError):
        SIM.simulate_CZ_gate(CF.LPSimulationInputs(pulse_shape="drag"))
    with pytest.raises(ValueError):
        SIM.simulate_CZ_gate(CF.LPSimulationInputs(pulse_shape="time_optimal"))
    with pytest.raises(TypeError):
        SIM.simulate_CZ_gate(object())
