"""CZ protocol parameter tables and formulas (vectorised).

Restates RG/protocols.py:
* LP V/Omega lookup with log-interpolation, clamped to [10, 1000]   (:369-379, :562-651)
* compute_phase_shift_xi                                             (:747-819)
* smooth-JP defaults                                                 (:447-473)
* bang-bang JP defaults (validated 5-segment)                        (:299-301, :324-332)
"""
from __future__ import annotations

import numpy as np

# (V/Omega, delta_over_omega, omega_tau_single) -- LP_PARAMS_BY_V_OMEGA
_LP_KEYS = np.array([10.0, 25.0, 50.0, 100.0, 200.0, 500.0, 1000.0])
_LP_DOM = np.array([0.340, 0.360, 0.370, 0.375, 0.377, 0.3773, 0.37737])
_LP_OT = np.array([4.45, 4.35, 4.32, 4.30, 4.293, 4.2927, 4.29268])

LP_OMEGA_TAU_DEFAULT = 4.29268
LP_DELTA_OVER_OMEGA_DEFAULT = 0.377371
LP_XI_DEFAULT = 3.90242

SMOOTH_JP_DEFAULTS = {
    "A": 0.311 * np.pi,
    "omega_mod_ratio": 1.242,
    "phi_offset": 4.696,
    "delta_over_omega": 0.0205,
    "omega_tau": 10.09,
}

JP_BANGBANG_OMEGA_TAU = 22.08
JP_BANGBANG_SWITCHING_TIMES = (2.214, 8.823, 13.258, 19.867)
JP_BANGBANG_PHASES = (np.pi / 2, 0.0, -np.pi / 2, 0.0, np.pi / 2)

PROTOCOL_NAMES = {"levine_pichler": "levine_pichler", "smooth_jp": "smooth_jp",
                  "jandura_pupillo": "jandura_pupillo"}


def lp_adaptive_params(v_over_omega):
    """(delta_over_omega, omega_tau) for LP at the given V/Omega (array).

    get_adaptive_protocol_params: clamp to [10, 1000]; exact table hits are
    returned verbatim, otherwise linear interpolation in log(V/Omega).
    """
    v = np.atleast_1d(np.asarray(v_over_omega, dtype=float)).copy()
    v = np.where(v < 10, 10.0, np.where(v > 1000, 1000.0, v))
    hi = np.searchsorted(_LP_KEYS, v, side="left")          # first key >= v
    hi = np.clip(hi, 0, len(_LP_KEYS) - 1)
    exact = _LP_KEYS[hi] == v
    lo = np.where(exact, hi, np.clip(hi - 1, 0, len(_LP_KEYS) - 1))
    klo, khi = _LP_KEYS[lo], _LP_KEYS[hi]
    with np.errstate(divide="ignore", invalid="ignore"):
        t = (np.log(v) - np.log(klo)) / (np.log(khi) - np.log(klo))
    dom = np.where(exact, _LP_DOM[hi], _LP_DOM[lo] + t * (_LP_DOM[hi] - _LP_DOM[lo]))
    ot = np.where(exact, _LP_OT[hi], _LP_OT[lo] + t * (_LP_OT[hi] - _LP_OT[lo]))
    return dom, ot


def compute_phase_shift_xi(Delta, Omega, tau):
    """e^{i xi} for the second LP pulse (RG/protocols.py:747-819), vectorised."""
    Delta = np.asarray(Delta, dtype=float)
    Om = np.abs(np.asarray(Omega, dtype=float))
    tau = np.asarray(tau, dtype=float)
    with np.errstate(divide="ignore", invalid="ignore"):
        y = Delta / Om
        s = Om * tau
        a = np.sqrt(y ** 2 + 1)
        b = s * a / 2
        num = a * np.cos(b) + 1j * y * np.sin(b)
        den = -a * np.cos(b) + 1j * y * np.sin(b)
        xi = num / den
    bad = (Om < 1e-10) | (np.abs(den) < 1e-12)
    return np.where(bad, 1.0 + 0j, xi)
