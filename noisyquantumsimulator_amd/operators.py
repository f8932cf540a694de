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


def hamiltonian(Omega: complex, Delta: float, V: float, dim: int = 3, delta1: float = 0.0) -> np.ndarray:
    d = dim
    I = np.eye(d, dtype=complex)
    up = np.outer(_k(d, 2), _k(d, 1))
    Ha = 0.5 * (Omega * up + np.conj(Omega) * up.conj().T)
    rys = [2] if d == 3 else [2, 3]
    H = np.kron(Ha, I) + np.kron(I, Ha)
    for r in rys:
        P = np.outer(_k(d, r), _k(d, r))
        H -= Delta * (np.kron(P, I) + np.kron(I, P))
    for r in rys:
        for s in rys:
            H += V * np.kron(np.outer(_k(d, r), _k(d, r)), np.outer(_k(d, s), _k(d, s)))
    P1 = np.outer(_k(d, 1), _k(d, 1))
    if delta1 != 0:
        H += delta1 * (np.kron(P1, I) + np.kron(I, P1))
    return H


def collapse_operators(rates: Dict[str, float], dim: int = 3, branching_1: float = 0.5) -> List[np.ndarray]:
    g = lambda k: float(rates.get(k, 0.0) or 0.0)
    d = dim
    I = np.eye(d, dtype=complex)
    rys = [2] if d == 3 else [2, 3]
    out: List[np.ndarray] = []

    def both(op, rate):
        out.extend([math.sqrt(rate) * np.kron(op, I), math.sqrt(rate) * np.kron(I, op)])
    tr = lambda a, b: np.outer(_k(d, a), _k(d, b))
    if g("gamma_r") > 0:
        for r in rys:
            both(tr(1, r), g("gamma_r") * branching_1)
            both(tr(0, r), g("gamma_r") * (1 - branching_1))
    if g("gamma_bbr") > 0:
        for r in rys:
            both(tr(0, r), g("gamma_bbr"))
    if d == 4 and g("mJ_leakage_rate") > 0:
        both(tr(3, 2), g("mJ_leakage_rate"))
        both(tr(2, 3), g("mJ_leakage_rate"))
    gphi = g("gamma_phi_laser") + g("gamma_phi_thermal") + g("gamma_phi_zeeman")
    if gphi > 0:
        for r in rys:
            both(tr(r, r), gphi)
    for key in ("gamma_loss_antitrap", "gamma_loss_background"):
        if g(key) > 0:
            for r in rys:
                both(tr(0, r), g(key))
    if g("gamma_scatter_intermediate") > 0:
        both(tr(1, 1), g("gamma_scatter_intermediate"))
    if g("gamma_leakage") > 0:
        for r in rys:
            both(tr(0, r), g("gamma_leakage"))
    return out


def basis_kets(dim: int = 3) -> Dict[str, np.ndarray]:
    b0, b1 = _k(dim, 0), _k(dim, 1)
    return {"00": np.kron(b0, b0), "01": np.kron(b0, b1), "10": np.kron(b1, b0), "11": np.kron(b1, b1)}
