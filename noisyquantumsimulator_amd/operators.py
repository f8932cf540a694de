"""Dense two-atom operators for SimulationResult.H1/H2/c_ops (numpy, no QuTiP).

The GPU engine never materialises these: it builds the generator from scalars.
They are returned so callers that inspect ``result.H1`` / ``result.c_ops`` keep
working.  Conventions follow RG/hamiltonians.py:584-1274 (H) and
RG/noise_models.py:1199-1620 (c_ops, same order); atom 1 is the slow tensor index.
"""
from __future__ import annotations

import math
from typing import Dict, List

import numpy as np


def _k(d, i):
    v = np.zeros(d, dtype=complex)
    v[i] = 1
    return v


def _count(d: int, level: int) -> np.ndarray:
    """Diagonal of P_level (x) I + I (x) P_level: atoms in ``level`` per two-atom basis state."""
    one = np.arange(d) == level
    return (one[:, None].astype(float) + one[None, :].astype(float)).ravel()


def hamiltonian(Omega: complex, Delta: float, V: float, dim: int = 3, delta1: float = 0.0) -> np.ndarray:
    """H = sum_atoms [(Omega/2)|r><1| + h.c. - Delta P_r + delta1 P_1] + V sum P_r P_r', entry
    by entry (the single-atom terms touch one atom index at a time) with the arithmetic
    of the kron-product form: Rabi terms, then -Delta per Rydberg level, +V, +delta1."""
    d = dim
    D = d * d
    H = np.zeros((D, D), dtype=complex)
    hu, hd = 0.5 * (Omega * 1.0 + np.conj(Omega) * 0.0), 0.5 * (Omega * 0.0 + np.conj(Omega) * 1.0)
    for o in range(d):                          # the other atom's level
        H[2 * d + o, 1 * d + o] += hu            # atom 1: |r><1| (x) I
        H[1 * d + o, 2 * d + o] += hd
        H[o * d + 2, o * d + 1] += hu            # atom 2: I (x) |r><1|
        H[o * d + 1, o * d + 2] += hd
    rys = [2] if d == 3 else [2, 3]
    diag = np.zeros(D, dtype=complex)
    for r in rys:
        diag -= Delta * _count(d, r)
    for r in rys:
        for q in rys:
            diag[r * d + q] += V
    if delta1 != 0:
        diag += delta1 * _count(d, 1)
    H[np.arange(D), np.arange(D)] += diag
    return H


def collapse_operators(rates: Dict[str, float], dim: int = 3, branching_1: float = 0.5) -> List[np.ndarray]:
    """The reference's c_op list and order (RG/noise_models.py:1575-1592), each
    sqrt(rate) |a><b| (x) I then sqrt(rate) I (x) |a><b|, set entry by entry."""
    g = lambda k: float(rates.get(k, 0.0) or 0.0)
    d = dim
    D = d * d
    rys = [2] if d == 3 else [2, 3]
    out: List[np.ndarray] = []

    def both(a: int, b: int, rate: float):
        c = math.sqrt(rate)
        m1 = np.zeros((D, D), dtype=complex)
        m2 = np.zeros((D, D), dtype=complex)
        for o in range(d):
            m1[a * d + o, b * d + o] = c
            m2[o * d + a, o * d + b] = c
        out.extend([m1, m2])
    if g("gamma_r") > 0:
        for r in rys:
            both(1, r, g("gamma_r") * branching_1)
            both(0, r, g("gamma_r") * (1 - branching_1))
    if g("gamma_bbr") > 0:
        for r in rys:
            both(0, r, g("gamma_bbr"))
    if d == 4 and g("mJ_leakage_rate") > 0:
        both(3, 2, g("mJ_leakage_rate"))
        both(2, 3, g("mJ_leakage_rate"))
    gphi = g("gamma_phi_laser") + g("gamma_phi_thermal") + g("gamma_phi_zeeman")
    if gphi > 0:
        for r in rys:
            both(r, r, gphi)
    for key in ("gamma_loss_antitrap", "gamma_loss_background"):
        if g(key) > 0:
            for r in rys:
                both(0, r, g(key))
    if g("gamma_scatter_intermediate") > 0:
        both(1, 1, g("gamma_scatter_intermediate"))
    if g("gamma_leakage") > 0:
        for r in rys:
            both(0, r, g("gamma_leakage"))
    return out


def basis_kets(dim: int = 3) -> Dict[str, np.ndarray]:
    out = {}
    for lab, (a, b) in (("00", (0, 0)), ("01", (0, 1)), ("10", (1, 0)), ("11", (1, 1))):
        v = np.zeros(dim * dim, dtype=complex)
        v[a * dim + b] = 1.0
        out[lab] = v
    return out
