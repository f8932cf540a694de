"""Input checks of the generic evolve_state seam (RG/simulation.py:647-690) that run
before any GPU call: segment lengths must be finite and non-negative and H Hermitian
(the kernel's Gershgorin bound assumes it), so such inputs raise instead of returning
the input state or an unflagged wrong one."""
import numpy as np
import pytest

from noisyquantumsimulator_amd import simulation as SIM


def _h(d=3):
    rng = np.random.default_rng(1)
    a = rng.normal(size=(d, d)) + 1j * rng.normal(size=(d, d))
    return a + a.conj().T


@pytest.mark.parametrize("T", [-1e-6, np.nan, np.inf])
def test_bad_segment_length_raises(T):
    with pytest.raises(ValueError, match="segment lengths"):
        SIM.evolve_state_batch(_h()[None], np.eye(3)[:1], np.array([T]))


def test_non_hermitian_hamiltonian_raises():
    H = _h()
    H[0, 1] += 1e-3
    with pytest.raises(ValueError, match="Hermitian"):
        SIM.evolve_state_batch(H[None], np.eye(3)[:1], np.array([1.0]))
    with pytest.raises(ValueError, match="Hermitian"):
        SIM.evolve_state(H, np.eye(3)[0], [0.0, 1.0])


def test_non_finite_hamiltonian_raises():
    H = _h()
    H[1, 1] = np.nan
    with pytest.raises(ValueError, match="Hermitian"):
        SIM.evolve_state_batch(H[None], np.eye(3)[:1], np.array([1.0]))
