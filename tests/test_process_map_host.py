"""Host side of the process-map layer (noise_models.py) on CPU: assembly from the
engine's output rows, Choi / Kraus / PTM against the oracle's textbook definitions,
the CZ phase fit, and known-answer channels.  SURVEY.md §8 a12 has no reference
oracle (the reference module is a stub): these pin the definitions."""
import numpy as np
import pytest

from noisyquantumsimulator_amd import noise_models as NM
from oracle import lindblad_oracle as O
from process_map_util import rows_from_map, spec_from_params, unitary_map


def _random_params(seed):
    from noisyquantumsimulator_amd import _native as N
    rng = np.random.default_rng(seed)
    p = np.zeros((N.NPARAM, 1))
    Om = 2 * np.pi * 4e6
    p[N.P["OMEGA"]], p[N.P["V"]], p[N.P["DELTA1"]] = Om, 30 * Om, 2 * np.pi * 2e5
    for k, hi in (("G1", 2e5), ("G0", 3e5), ("GPHI", 4e5), ("GSC", 2e5)):
        p[N.P[k + "_A"]] = rng.uniform(0, hi)
        p[N.P[k + "_B"]] = rng.uniform(0, hi)
    p[N.P["DELTA"]], p[N.P["TAU"]] = 0.377 * Om, 4.29268 / Om
    xi = np.exp(1j * rng.uniform(0, 2 * np.pi))
    p[N.P["XI_RE"]], p[N.P["XI_IM"]] = xi.real, xi.imag
    return p


@pytest.fixture(scope="module")
def noisy_map():
    return O.process_map(spec_from_params(_random_params(4), 0, "lp_square"))


def test_assembly_from_engine_rows(noisy_map):
    state, coh = rows_from_map(noisy_map)
    S = NM.assemble_maps(state, coh)[0]
    np.testing.assert_allclose(S, noisy_map, atol=1e-15)


def test_choi_ptm_match_oracle_definitions(noisy_map):
    S = noisy_map[None]
    np.testing.assert_allclose(NM.choi(S)[0], O.choi_matrix(noisy_map), atol=1e-15)
    np.testing.assert_allclose(NM.ptm(S)[0], O.pauli_transfer_matrix(noisy_map), atol=1e-15)
    w = np.linalg.eigvalsh(NM.choi(S)[0])
    assert w.min() > -1e-12                                  # completely positive


def test_kraus_reproduce_map(noisy_map):
    pm = NM.analyse(noisy_map[None], with_kraus=True)
    K = pm.kraus_ops[0]
    for a in range(4):
        for b in range(4):
            X = np.zeros((4, 4), dtype=complex)
            X[a, b] = 1
            np.testing.assert_allclose(sum(k @ X @ k.conj().T for k in K), O.apply_map(noisy_map, X),
                                       atol=1e-13)
    # trace non-increasing: sum K^dag K <= I (leakage out of the qubit block)
    assert np.linalg.eigvalsh(np.eye(4) - sum(k.conj().T @ k for k in K)).min() > -1e-12


def test_phase_fit_is_the_maximum(noisy_map):
    pm = NM.analyse(noisy_map[None])
    g = np.linspace(-np.pi, np.pi, 361)
    A, B = np.meshgrid(g, g, indexing="ij")
    F = NM.process_fidelity(np.broadcast_to(noisy_map, (A.size, 16, 16)), NM.ideal_cz(A.ravel(), B.ravel()))
    assert pm.process_fidelity[0] >= F.max() - 1e-12
    # leakage = 1 - Tr E(I/4); Pauli probabilities sum to the surviving weight
    tr = np.mean([np.trace(O.apply_map(noisy_map, np.diag(np.eye(4)[x]).astype(complex))).real
                  for x in range(4)])
    assert pm.leakage[0] == pytest.approx(1 - tr, abs=1e-14)
    assert pm.pauli_probs[0].sum() == pytest.approx(1 - pm.leakage[0], abs=1e-13)


def test_ideal_cz_with_local_phases():
    a, b = 0.7, -1.9
    U = np.diag([1, np.exp(1j * b), np.exp(1j * a), -np.exp(1j * (a + b))])
    pm = NM.analyse(unitary_map(U)[None], with_kraus=True)
    assert pm.process_fidelity[0] == pytest.approx(1.0, abs=1e-14)
    assert pm.avg_gate_fidelity[0] == pytest.approx(1.0, abs=1e-14)
    assert pm.kraus_rank[0] == 1 and pm.leakage[0] == pytest.approx(0, abs=1e-15)
    assert pm.alpha[0] == pytest.approx(a) and pm.beta[0] == pytest.approx(b)
    assert pm.pauli_error[0] == pytest.approx(0, abs=1e-14)


def test_depolarised_cz_known_answer():
    """E = (1-p) CZ + p * (complete depolarisation): PTM diagonal 1-p on non-identity
    Paulis of the error channel, uniform Pauli probabilities p/16 + ..."""
    p = 0.03
    U = np.diag([1, 1, 1, -1]).astype(complex)
    S = (1 - p) * unitary_map(U)
    for a in range(4):
        S[5 * np.arange(4), 5 * a] += p / 4                   # |a><a| -> I/4 ; coherences -> 0
    pm = NM.analyse(S[None])
    np.testing.assert_allclose(pm.pauli_probs[0, 1:], p / 16, atol=1e-15)
    assert pm.pauli_probs[0, 0] == pytest.approx(1 - 15 * p / 16)
    assert pm.process_fidelity[0] == pytest.approx(1 - 15 * p / 16)
    assert pm.avg_gate_fidelity[0] == pytest.approx((4 * (1 - 15 * p / 16) + 1) / 5)


def test_ket_maps_and_gate_fidelity_of_ideal_cz():
    """noise_models.ket_maps + gate_fidelity (the gauge-invariant figure of merit on
    BatchResult / SimulationResult): an exact CZ with arbitrary local Z phases and a
    global phase has process fidelity 1; a swap of the |11> sign (identity) has 0.25."""
    rng = np.random.default_rng(5)
    for d in (3, 4):
        a, b, g = rng.uniform(-np.pi, np.pi, 3)
        q = [0, 1, d, d + 1]
        psi = np.zeros((2, 4, d * d), complex)
        u = np.exp(1j * g) * np.array([1, np.exp(1j * b), np.exp(1j * a), -np.exp(1j * (a + b))])
        for x in range(4):
            psi[0, x, q[x]] = u[x]
            psi[1, x, q[x]] = 1.0
        fpro, favg = NM.gate_fidelity(NM.ket_maps(psi, d))
        np.testing.assert_allclose(fpro, [1.0, 0.25], atol=1e-12)
        np.testing.assert_allclose(favg, [1.0, 0.4], atol=1e-12)


def test_gate_fidelity_equals_analyse_on_noisy_map(noisy_map):
    S = noisy_map[None]
    fpro, favg = NM.gate_fidelity(S)
    pm = NM.analyse(S)
    np.testing.assert_array_equal(fpro, pm.process_fidelity)
    np.testing.assert_array_equal(favg, pm.avg_gate_fidelity)
