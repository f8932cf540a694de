"""Process maps on the GPU (ryd_run_coherences + the diagonal sector) against the
oracle's full-Liouvillian definition.  Tolerance 1e-10 on every
map element, as the state parity tests."""
import numpy as np
import pytest

from noisyquantumsimulator_amd import _native as N
from noisyquantumsimulator_amd import engine as E
from noisyquantumsimulator_amd import noise_models as NM
from oracle import lindblad_oracle as O
from process_map_util import spec_from_params
from test_gpu_parity import _random_points

pytestmark = pytest.mark.gpu
TOL = 1e-10
QI = O.QUBIT_INDEX


@pytest.fixture(scope="module")
def eng():
    return E.Engine()


@pytest.mark.parametrize("protocol,n_steps", [("lp_square", None), ("smooth_jp", 30), ("bangbang", None)])
def test_process_map_matches_oracle(eng, protocol, n_steps):
    rng = np.random.default_rng(99)
    p = _random_points(rng, 5, protocol)                 # asymmetric atoms, random rates
    pm = NM.gate_process_maps(p, protocol, n_steps=n_steps, engine=eng, with_kraus=True)
    assert np.all(pm.status == 0)
    for i in range(5):
        ref = O.process_map(spec_from_params(p, i, protocol, n_steps=n_steps or 300))
        np.testing.assert_allclose(pm.S[i], ref, atol=TOL, rtol=0)
    assert np.all(pm.kraus_rank > 1)                      # noisy: not a unitary channel


def test_noise_free_map_is_the_ket_unitary(eng):
    """Zero rates: the coherence kernels and the ket kernel are independent routes to
    the same qubit-block unitary, S = U_q (x) conj(U_q)."""
    rng = np.random.default_rng(5)
    p = _random_points(rng, 40, "lp_square")
    for k in ("G1", "G0", "GPHI", "GSC"):
        p[N.P[k + "_A"]] = p[N.P[k + "_B"]] = 0.0
    pm = NM.gate_process_maps(p, "lp_square", engine=eng, with_kraus=True)
    psi = eng.run(p, "lp_square", "ket").kets()           # (n, 4 inputs, 9)
    Uq = psi[:, :, QI].transpose(0, 2, 1)                 # U_q[c, a] = <c|psi_a>
    S_ket = np.einsum("nca,ndb->ncdab", Uq, np.conj(Uq)).reshape(-1, 16, 16)
    np.testing.assert_allclose(pm.S, S_ket, atol=TOL, rtol=0)
    assert np.all(pm.kraus_rank == 1)


def test_large_batch_channel_properties(eng):
    rng = np.random.default_rng(8)
    n = 2000
    p = _random_points(rng, n, "lp_square")
    pm = NM.gate_process_maps(p, "lp_square", engine=eng)
    assert np.all(pm.status == 0)
    w = np.linalg.eigvalsh(pm.choi)
    assert w.min() > -1e-10                               # completely positive
    # trace non-increasing: Tr_out J <= I_in
    T = np.einsum("nacbc->nab", pm.choi.reshape(n, 4, 4, 4, 4))
    assert np.linalg.eigvalsh(np.eye(4) - T).min() > -1e-10
    assert np.all((pm.process_fidelity <= 1 + 1e-12) & (pm.leakage >= -1e-12))
    np.testing.assert_allclose(pm.pauli_probs.sum(axis=1), 1 - pm.leakage, atol=1e-11)
    for i in (0, n - 1):
        ref = O.process_map(spec_from_params(p, i, "lp_square"))
        np.testing.assert_allclose(pm.S[i], ref, atol=TOL, rtol=0)


def test_coherence_rows_are_independent_of_their_wave(eng):
    """4 points per wave, each row (and each quad bank) with its own squaring depth: a
    ragged batch gives every point the bits it gets alone."""
    rng = np.random.default_rng(17)
    p = _random_points(rng, 7, "lp_square")
    coh, st = eng.run_coherences(p, "lp_square")
    assert np.all(st == 0)
    for i in (0, 3, 6):
        c1, s1 = eng.run_coherences(p[:, i:i + 1].copy(), "lp_square")
        np.testing.assert_array_equal(c1[:, 0], coh[:, i])
