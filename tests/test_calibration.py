"""Calibration-data writer: CPU layout / round trip on a
synthetic batch result, GPU end to end."""
import warnings

import numpy as np

from noisyquantumsimulator_amd._native import STATUS_FAIL_MASK
import pytest

from noisyquantumsimulator_amd import calibration as CAL
from noisyquantumsimulator_amd import configurations as CF
from noisyquantumsimulator_amd import physics as PH
from noisyquantumsimulator_amd.simulation import BatchResult


def _fake_result(n=3):
    warnings.simplefilter("ignore")
    b = PH.derive_batch(CF.LPSimulationInputs(), n, temperature=np.linspace(1e-6, 3e-6, n))
    F = np.tile([1.0, 0.99, 0.99, 0.97], (n, 1))
    return BatchResult(batch=b, avg_fidelity=F.mean(1), fidelities=F, populations=F,
                       controlled_phase=np.full(n, np.pi - 0.1), cz_phase_fidelity=np.full(n, 0.99),
                       status=np.zeros(n, np.uint32), is_mixed=np.ones(n, bool))


def test_records_and_roundtrip(tmp_path):
    br = _fake_result()
    recs = CAL.records(br, {"temperature": np.linspace(1e-6, 3e-6, 3), "tweezer_power": 0.03})
    assert len(recs) == 3
    r = recs[1]
    assert r["parameters"]["temperature"] == pytest.approx(2e-6)
    assert r["error_rates"]["avg_infidelity"] == pytest.approx(1 - br.avg_fidelity[1])
    assert r["error_rates"]["phase_error_deg"] == pytest.approx(np.degrees(0.1))
    assert r["durations"]["gate_time_us"] == pytest.approx(br.batch["tau_total"][1] * 1e6)
    path = CAL.calibration_path(str(tmp_path), "Rb87", 70, "levine_pichler")
    assert path.endswith("neutral_atoms/rydberg_cz/n70_Rb87_levine_pichler.json")
    CAL.write_calibration(path, recs, "Rb87", 70, "levine_pichler", {"note": "test"})
    doc = CAL.load_calibration(path)
    assert doc["points"] == recs and doc["metadata"]["n_points"] == 3 and doc["metadata"]["note"] == "test"
    bad = tmp_path / "bad.json"
    bad.write_text('{"schema": "other"}')
    with pytest.raises(ValueError):
        CAL.load_calibration(str(bad))


@pytest.mark.gpu
def test_calibrate_cz_on_gpu(tmp_path):
    from noisyquantumsimulator_amd.simulation import simulate_CZ_gate_batch
    warnings.simplefilter("ignore")
    si = CF.LPSimulationInputs()
    sp = np.array(["Rb87", "Rb87", "Cs133"])
    T = np.array([1e-6, 5e-6, 2e-6])
    paths = CAL.calibrate_cz(si, str(tmp_path), species=sp, n_rydberg=70, temperature=T)
    assert len(paths) == 2
    rb = CAL.load_calibration(CAL.calibration_path(str(tmp_path), "Rb87", 70, "levine_pichler"))
    cs = CAL.load_calibration(CAL.calibration_path(str(tmp_path), "Cs133", 70, "levine_pichler"))
    assert len(rb["points"]) == 2 and len(cs["points"]) == 1
    br = simulate_CZ_gate_batch(si, species=sp, n_rydberg=70, temperature=T)
    for doc, idx in ((rb, [0, 1]), (cs, [2])):
        for rec, i in zip(doc["points"], idx):
            assert rec["status"] & STATUS_FAIL_MASK == 0 and rec["status"] == int(br.status[i])
            assert rec["error_rates"]["avg_infidelity"] == pytest.approx(1 - br.avg_fidelity[i], abs=1e-12)
            e = rec["error_rates"]
            pauli = sum(e["pauli_error_probs"].values())
            assert 0 < pauli < 1 and 0 <= e["leakage"] < 1
            assert 0 < e["avg_gate_infidelity"] < 0.2
