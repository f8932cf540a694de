"""The gauge-invariant noisy figure of merit on the product surface (VERDICT r2
missing #5 / weak #6): BatchResult / SimulationResult carry the process and average
gate fidelity to CZ up to local Z phases (noise_models.gate_fidelity), checked against
the oracle's 81x81 process map; the optimiser can minimise it (cost="process_fidelity"),
which makes a noisy DE run a continuous function of its inputs, and the default
(reference-cost) run reports how many simulated candidates were gauge-flagged."""
import importlib
import warnings

import numpy as np
import pytest

import oracle_evaluator as OE
from noisyquantumsimulator_amd import noise_models as NM
from noisyquantumsimulator_amd import simulation as SIM
from oracle import lindblad_oracle as O

OC = importlib.import_module("noisyquantumsimulator_amd.optimize_cz_gate")
pytestmark = pytest.mark.gpu


def _inputs(noisy):
    a = OC.ApparatusConstraints()
    exc = a.make_excitation_config(0.99 if noisy else 1.0)
    noise = a.make_full_noise() if noisy else a.make_noiseless()
    return a, exc, noise


@pytest.mark.parametrize("proto,noisy", [("lp", True), ("smooth_jp", True), ("jp_bangbang", True),
                                         ("lp", False), ("smooth_jp", False)])
def test_batch_process_fidelity_matches_oracle_map(proto, noisy):
    warnings.simplefilter("ignore")
    a, exc, noise = _inputs(noisy)
    space = OC._param_space(proto, 5 if proto == "jp_bangbang" else None)
    rng = np.random.default_rng(11)
    lo, hi = np.array(space.bounds).T
    X = np.vstack([space.x0, lo + (hi - lo) * rng.random((2, len(lo)))])
    si, over = space.inputs(X, exc, noise)
    br = SIM.simulate_CZ_gate_batch(si, X.shape[0], include_noise=noisy, overrides=over, process_fidelity=True,
                                    **a.simulate_kwargs())
    assert br.ok.all()
    S = np.stack([O.process_map(OE.point_spec(br.batch, i)) for i in range(br.n)])
    fpro, favg = NM.gate_fidelity(S)
    np.testing.assert_allclose(br.process_fidelity, fpro, atol=1e-10, rtol=0)
    np.testing.assert_allclose(br.avg_gate_fidelity, favg, atol=1e-10, rtol=0)
    assert np.all(br.avg_gate_fidelity <= 1 + 1e-12)


def test_simulation_result_carries_invariant_fidelity():
    warnings.simplefilter("ignore")
    a, exc, noise = _inputs(True)
    si = OC._build_lp_inputs(OC._param_space("lp").x0, exc, noise)
    r0 = SIM.simulate_CZ_gate(si, include_noise=True, **a.simulate_kwargs())
    assert r0.process_fidelity is None and r0.avg_gate_fidelity is None        # not requested
    r = SIM.simulate_CZ_gate(si, include_noise=True, process_fidelity=True, **a.simulate_kwargs())
    br = SIM.simulate_CZ_gate_batch(si, 1, include_noise=True, process_fidelity=True, **a.simulate_kwargs())
    assert r.process_fidelity == br.process_fidelity[0] and r.avg_gate_fidelity == br.avg_gate_fidelity[0]
    assert 0.9 < r.avg_gate_fidelity < 1.0 and r.avg_fidelity == r0.avg_fidelity


def test_invariant_cost_de_is_continuous_in_its_inputs():
    """A noisy DE run on cost="process_fidelity" returns the same best candidate when an
    apparatus input moves by one part in 1e12 (the reference cost cannot promise this:
    its noisy phase penalty is gauge-flagged on most points)."""
    warnings.simplefilter("ignore")
    runs = []
    for scale in (1.0, 1.0 + 1e-12):
        a = OC.ApparatusConstraints()
        a.laser_2_power *= scale
        runs.append(OC.optimize_cz_gate("lp", a, include_noise=True, maxiter=3, popsize=5, seed=7,
                                        cache=OC.SimulationCache(), verbose=False, cost="process_fidelity"))
    r0, r1 = runs
    assert r0.cost == "process_fidelity" and r0.n_simulated > 0
    np.testing.assert_allclose(r0.best_params, r1.best_params, rtol=1e-6, atol=0)
    assert abs(r0.best_cost - r1.best_cost) <= 1e-8 * abs(r0.best_cost)
    assert np.isfinite(r0.best_metrics["avg_gate_fidelity"]) and r0.best_metrics["avg_gate_fidelity"] > 0.9


def test_reference_cost_run_reports_gauge_flags():
    warnings.simplefilter("ignore")
    a = OC.ApparatusConstraints()
    r = OC.optimize_cz_gate("lp", a, include_noise=True, maxiter=2, popsize=5, seed=3,
                            cache=OC.SimulationCache(), verbose=False)
    assert r.cost == "reference" and r.n_simulated > 0
    assert 0 < r.gauge_flagged <= r.n_simulated
    assert "Gauge-flagged" in repr(r)
