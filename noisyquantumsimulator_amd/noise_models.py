"""Gate process maps: Choi, Kraus, Pauli transfer matrix and Pauli error rates
of the noisy Rydberg CZ gate.

The reference promises this layer (README.md:20, docs/ARCHITECTURE.md:102-111)
but ships only a stub (src/qpu_simulator/noise_models/__init__.py:1-22).  Here
it sits on the GPU engine:

* the 4 diagonal qubit inputs |x><x| come from the Lindblad state of
  ``ryd_run_batch`` (the real 25-dim sector);
* the 6 upper off-diagonal qubit matrix units come from ``ryd_run_coherences``
  (each evolved in its own excitation-number sector, see the kernel comment in
  csrc/ryd_engine.hip); the other 6 are adjoints.

From those 36 numbers per point the host assembles (vectorised over points):

``S[n, 4c+d, 4a+b] = <c| E(|a><b|) |d>`` the qubit-block map (basis 00,01,10,11;
atom A is the first qubit), its Choi matrix, Kraus operators, PTM, the process
and average gate fidelity to CZ up to the best single-qubit Z phases (a
gauge-invariant, phase-sensitive figure of merit, unlike the reference's
eigenvector-phase penalty), the leakage out of the qubit subspace, and the
Pauli error probabilities of the twirled error channel U_CZ^-1 o E.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _native as N

QUBIT_E = (0, 1)   # e00 = |0><0|, e11 = |1><1| in the single-atom sector basis

_P1 = (np.eye(2, dtype=complex), np.array([[0, 1], [1, 0]], dtype=complex),
       np.array([[0, -1j], [1j, 0]]), np.array([[1, 0], [0, -1]], dtype=complex))
PAULI_LABELS = tuple(a + b for a in "IXYZ" for b in "IXYZ")
PAULI2 = np.array([np.kron(P, Q) for P in _P1 for Q in _P1])          # (16, 4, 4)
# (-1)^[P_i, P_j anticommute]
_CHI = np.array([[1.0 if np.allclose(Pi @ Pj, Pj @ Pi) else -1.0 for Pj in PAULI2] for Pi in PAULI2])


def assemble_maps(state: np.ndarray, coh: np.ndarray) -> np.ndarray:
    """S (n, 16, 16) complex from the Lindblad state rows (25, 4n) of the diagonal
    inputs and the coherence rows (NCOH, n)."""
    n = coh.shape[1]
    R = state.reshape(25, n, 4)                                     # [e_A*5 + e_B][point][input x]
    S = np.zeros((n, 16, 16), dtype=complex)
    for x in range(4):
        for y in range(4):                                          # <y|E(|x><x|)|y>
            ya, yb = QUBIT_E[y >> 1], QUBIT_E[y & 1]
            S[:, 5 * y, 5 * x] = R[5 * ya + yb, :, x]
    c = lambda row: coh[row] + 1j * coh[row + 1]
    pairs = ((N.C["K0"], ((0, 1), (2, 3))),     # inputs |00><01|, |10><11| ; outputs the same pair
             (N.C["K1"], ((0, 2), (1, 3))))     # inputs |00><10|, |01><11|
    for base, units in pairs:
        for s, (a, b) in enumerate(units):
            for o, (cc, dd) in enumerate(units):
                S[:, 4 * cc + dd, 4 * a + b] = c(base + 4 * s + 2 * o)
    S[:, 4 * 0 + 3, 4 * 0 + 3] = c(N.C["K2"])                        # |00><11|
    S[:, 4 * 1 + 2, 4 * 1 + 2] = c(N.C["K3"])                        # |01><10|
    # adjoint inputs: E(|b><a|) = E(|a><b|)^dag  ->  S[dc, ba] = conj S[cd, ab]
    idx = np.arange(16)
    swap = 4 * (idx % 4) + idx // 4
    for a in range(4):
        for b in range(a + 1, 4):
            col = 4 * a + b
            S[:, swap, 4 * b + a] = np.conj(S[:, :, col])
    return S


def choi(S: np.ndarray) -> np.ndarray:
    """J[(a,c),(b,d)] = <c|E(|a><b|)|d>, input factor first: (n, 16, 16)."""
    n = S.shape[0]
    T = S.reshape(n, 4, 4, 4, 4)                                    # [c, d, a, b]
    return T.transpose(0, 3, 1, 4, 2).reshape(n, 16, 16)            # [a, c, b, d]


def kraus(J: np.ndarray, rtol: float = 1e-12):
    """Kraus operators from the Choi matrix: K_k[c, a] = sqrt(lam_k) v_k[4a + c].
    Returns (K (n, 16, 4, 4), rank (n,)); eigenvalues below rtol*max are dropped."""
    w, V = np.linalg.eigh(J)
    w = np.where(w > rtol * w.max(axis=1, keepdims=True), w, 0.0)
    K = (np.sqrt(w)[:, None, :] * V)                                # column k = sqrt(lam) v_k
    K = K.reshape(-1, 4, 4, 16).transpose(0, 3, 2, 1)               # [n, k, c, a]
    return K[:, ::-1], (w > 0).sum(axis=1)


def ptm(S: np.ndarray) -> np.ndarray:
    """R[n, i, j] = Tr(P_i E(P_j)) / 4 (real for Hermiticity-preserving maps)."""
    vP = PAULI2.reshape(16, 16)                                     # row j = vec(P_j), 4a+b
    vPT = PAULI2.transpose(0, 2, 1).reshape(16, 16)                 # row i = vec(P_i^T)
    return np.real(np.einsum("ik,nkl,jl->nij", vPT, S, vP)) / 4


def _coh(S, a, b):
    return S[:, 4 * a + b, 4 * a + b]


def cz_phase_fit(S: np.ndarray, iters: int = 30):
    """Single-qubit Z phases (alpha on atom A, beta on atom B) maximising the process
    fidelity to U = diag(1, e^{i beta}, e^{i alpha}, -e^{i(alpha+beta)}); coordinate
    ascent, each step exact (F is a + Re(e^{i alpha} C(beta)) in alpha and vice versa)."""
    s01 = _coh(S, 0, 1) - _coh(S, 2, 3)
    s10 = _coh(S, 0, 2) - _coh(S, 1, 3)
    s11 = _coh(S, 0, 3)
    sx = _coh(S, 1, 2)
    al = -np.angle(s10)
    be = -np.angle(s01)
    for _ in range(iters):
        Ca = s10 - np.exp(1j * be) * s11 + np.exp(-1j * be) * sx
        al = -np.angle(Ca)
        Cb = s01 - np.exp(1j * al) * s11 + np.exp(-1j * al) * np.conj(sx)
        be = -np.angle(Cb)
    return al, be


def ideal_cz(alpha: np.ndarray, beta: np.ndarray) -> np.ndarray:
    """Diagonal of U (n, 4)."""
    return np.stack([np.ones_like(alpha, dtype=complex), np.exp(1j * beta), np.exp(1j * alpha),
                     -np.exp(1j * (alpha + beta))], axis=1)


def process_fidelity(S: np.ndarray, u: np.ndarray) -> np.ndarray:
    """F_pro = Tr(S_U^dag S) / 16 with S_U[(c,d),(a,b)] = d_ca d_db u_a conj(u_b)."""
    diag = np.einsum("na,nb->nab", np.conj(u), u).reshape(-1, 16)   # conj(u_a) u_b at 4a+b
    return np.real(np.einsum("nk,nk->n", diag, np.einsum("nkk->nk", S))) / 16


def ket_maps(psi: np.ndarray, dim: int = 3) -> np.ndarray:
    """S (n, 16, 16) of a unitary (noise-free) evolution from the output kets psi[n, 4, D]
    of the 4 basis inputs: <c|E(|a><b|)|d> = psi_a[c] conj(psi_b[d]) on the qubit block."""
    q = np.array([0, 1, dim, dim + 1])                              # |00>, |01>, |10>, |11> in D
    P = psi[:, :, q]                                                # [n, a, c]
    return np.einsum("nac,nbd->ncdab", P, np.conj(P)).reshape(psi.shape[0], 16, 16)


def gate_fidelity(S: np.ndarray):
    """(process fidelity, average gate fidelity) to CZ up to the fitted local Z phases:
    a function of the map alone, so unlike the reference's eigenvector-phase penalty it
    does not depend on the eigensolver's gauge."""
    al, be = cz_phase_fit(S)
    fpro = process_fidelity(S, ideal_cz(al, be))
    surv = np.real(S[:, ::5, ::5].sum(axis=(1, 2))) / 4
    return fpro, (4 * fpro + surv) / 5


@dataclass
class ProcessMaps:
    S: np.ndarray                 # (n, 16, 16) qubit-block map on matrix units
    choi: np.ndarray              # (n, 16, 16)
    ptm: np.ndarray               # (n, 16, 16)
    process_fidelity: np.ndarray  # to CZ up to the fitted local Z phases
    avg_gate_fidelity: np.ndarray
    leakage: np.ndarray           # mean over basis inputs of the weight outside the qubit block
    alpha: np.ndarray             # fitted Z phase on atom A
    beta: np.ndarray              # fitted Z phase on atom B
    pauli_probs: np.ndarray       # (n, 16): twirled U^-1 o E, order PAULI_LABELS
    status: np.ndarray
    kraus_ops: Optional[np.ndarray] = None
    kraus_rank: Optional[np.ndarray] = None

    @property
    def pauli_error(self) -> np.ndarray:
        """Total Pauli error (all non-identity terms) of the twirled channel."""
        return self.pauli_probs[:, 1:].sum(axis=1)


def analyse(S: np.ndarray, status: Optional[np.ndarray] = None, with_kraus: bool = False) -> ProcessMaps:
    n = S.shape[0]
    J = choi(S)
    R = ptm(S)
    al, be = cz_phase_fit(S)
    u = ideal_cz(al, be)
    fpro = process_fidelity(S, u)
    surv = np.real(S[:, ::5, ::5].sum(axis=(1, 2))) / 4             # Tr E(I/4) = sum_xy <y|E(|x><x|)|y>/4
    favg = (4 * fpro + surv) / 5
    # error channel E' = U^dag o E: S'[(c,d),:] = conj(u_c) u_d S[(c,d),:]
    Sp = np.einsum("na,nb->nab", np.conj(u), u).reshape(n, 16, 1) * S
    f = np.einsum("nii->ni", ptm(Sp))                                # Pauli fidelities
    probs = f @ _CHI.T / 16
    out = ProcessMaps(S=S, choi=J, ptm=R, process_fidelity=fpro, avg_gate_fidelity=favg,
                      leakage=1.0 - surv, alpha=al, beta=be, pauli_probs=probs,
                      status=status if status is not None else np.zeros(n, np.uint32))
    if with_kraus:
        out.kraus_ops, out.kraus_rank = kraus(J)
    return out


def gate_process_maps(params: np.ndarray, protocol: str, n_steps: Optional[int] = None,
                      shape: str = "square", engine=None, with_kraus: bool = False) -> ProcessMaps:
    """Process maps of a batch of packed points (engine.pack_params layout) on the GPU."""
    from . import engine as E
    eng = engine if engine is not None else E.Engine()
    diag = eng.run(params, protocol, "lindblad", n_steps=n_steps, shape=shape)
    coh, cst = eng.run_coherences(params, protocol, n_steps=n_steps, shape=shape)
    S = assemble_maps(diag.state, coh)
    return analyse(S, diag.status | cst, with_kraus=with_kraus)
