"""Alkali species data and the per-species formulas the CZ path needs.

The numbers are the reference's atom database entries (RG/atom_database.py:104
ATOM_DB), stored as the exact float64 values it evaluates to, so every derived
quantity matches.  Only the fields on the simulate_CZ_gate path are kept.
All functions accept numpy arrays (vectorised over sweep points).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict

import numpy as np

from .constants import C, HBAR, RY_JOULES


@dataclass(frozen=True)
class Species:
    name: str
    mass: float                     # kg
    alpha_ground: float             # static ground polarisability, SI (C m^2/V)
    trap_wavelength: float          # default tweezer wavelength, m
    n_ref: int
    C6_ref: float                   # (rad/s) m^6 at n_ref
    tau_0K_ref: float               # s
    tau_ref: float                  # s (300 K)
    alpha_rydberg_ref: float        # SI at n_ref, 1064 nm
    dipole_er_ref: float            # intermediate -> Rydberg dipole at n_ref, C m
    qd_S: float                     # S quantum defect
    intermediate: str               # default intermediate state
    dipole_1e: float                # ground -> intermediate dipole, C m
    gamma_e: float                  # intermediate linewidth, rad/s
    f_ground_to_e: float            # Hz
    E_ionization: float             # J
    omega_D1: float                 # rad/s (two-resonance polarisability model)
    omega_D2: float
    K_quad_zeeman: float            # Hz/G^2 used by calculate_zeeman_shift
    K_quad_noise: float             # Hz/G^2 used for the Zeeman dephasing rate
    stark_hz_per_mK: float          # qubit differential light shift
    g_F_lower: float                # for non-clock Zeeman shifts
    F_lower: int
    exp_C6: float = 11.0
    exp_tau0: float = 3.0
    exp_tau_bbr: float = 2.0
    exp_alpha: float = 7.0
    exp_dipole: float = -1.5


RB87 = Species(
    name="Rb87", mass=1.443160648e-25, alpha_ground=1.1332046206678246e-38,
    trap_wavelength=1.064e-06, n_ref=70, C6_ref=5.420441132650756e-24,
    tau_0K_ref=0.00028, tau_ref=0.00014, alpha_rydberg_ref=-3.297554548720572e-36,
    dipole_er_ref=1.1869695075757072e-31, qd_S=3.1311807, intermediate="5P3/2",
    dipole_1e=3.586343583603744e-29, gamma_e=38107518.88804419,
    f_ground_to_e=384230484468000.0, E_ionization=6.692496878827151e-19,
    omega_D1=2 * np.pi * 377.107e12, omega_D2=2 * np.pi * 384.230e12,
    K_quad_zeeman=575.0, K_quad_noise=575.0, stark_hz_per_mK=70e3,
    g_F_lower=-0.5, F_lower=1,
)

CS133 = Species(
    name="Cs133", mass=2.20694657e-25, alpha_ground=1.6487772743602862e-38,
    trap_wavelength=1.064e-06, n_ref=70, C6_ref=8.796459430051418e-24,
    tau_0K_ref=0.00032, tau_ref=0.00016, alpha_rydberg_ref=-4.946331823080859e-36,
    dipole_er_ref=1.017402435064892e-31, qd_S=4.0493532, intermediate="6P3/2",
    dipole_1e=3.806780777867804e-29, gamma_e=32886191.897777956,
    f_ground_to_e=351725718509000.0, E_ionization=6.2387155951326e-19,
    omega_D1=2 * np.pi * 335.116e12, omega_D2=2 * np.pi * 351.726e12,
    K_quad_zeeman=2000.0, K_quad_noise=427.0, stark_hz_per_mK=200e3,
    g_F_lower=-0.25, F_lower=3,
)

SPECIES: Dict[str, Species] = {"Rb87": RB87, "Cs133": CS133}


def get(name: str) -> Species:
    try:
        return SPECIES[name]
    except KeyError:
        raise ValueError(f"Unknown species: {name}. Available: {list(SPECIES)}") from None


def n_star(sp: Species, n):
    return np.asarray(n, dtype=float) - sp.qd_S


def C6(sp: Species, n):
    """RG/atom_database.py:662-719 -- C6 ∝ n*^11, (rad/s) m^6."""
    return sp.C6_ref * (n_star(sp, n) / (sp.n_ref - sp.qd_S)) ** sp.exp_C6


def rydberg_lifetime(sp: Species, n, temperature: float = 300.0):
    """RG/atom_database.py:722-789 -- 0 K radiative + BBR (T^4 scaled)."""
    ratio = n_star(sp, n) / (sp.n_ref - sp.qd_S)
    tau_0K = sp.tau_0K_ref * ratio ** sp.exp_tau0
    if temperature < 1:
        return tau_0K
    tau_bbr_ref = sp.tau_ref * sp.tau_0K_ref / (sp.tau_0K_ref - sp.tau_ref)
    tau_bbr = tau_bbr_ref * ratio ** sp.exp_tau_bbr
    tau_bbr = tau_bbr * (300.0 / temperature) ** 4
    return 1.0 / (1.0 / tau_0K + 1.0 / tau_bbr)


def dipole_to_rydberg(sp: Species, n):
    """Leg-2 dipole scaled as (n/n_ref)^-1.5 (RG/simulation.py:2905-2907)."""
    return sp.dipole_er_ref * (np.asarray(n, dtype=float) / sp.n_ref) ** (-1.5)


def ground_polarizability_at(sp: Species, wavelength_nm):
    """RG/trap_physics.py:85-207, ground branch: two-resonance correction when
    red-detuned of D1, static value otherwise."""
    lam = np.asarray(wavelength_nm, dtype=float) * 1e-9
    w = 2 * np.pi * C / lam
    corr = 1.0 + 0.3 * w ** 2 / (sp.omega_D1 ** 2 - w ** 2)
    return np.where(w < sp.omega_D1, sp.alpha_ground * corr, sp.alpha_ground)


def rydberg_polarizability_at(sp: Species, wavelength_nm, n):
    """RG/trap_physics.py:85-207, Rydberg branch: n*^7 scaling with the
    ponderomotive (lambda/1064 nm)^2 wavelength factor."""
    lam = np.asarray(wavelength_nm, dtype=float) * 1e-9
    a_static = sp.alpha_rydberg_ref * (n_star(sp, n) / (sp.n_ref - sp.qd_S)) ** sp.exp_alpha
    return a_static * (lam / 1064e-9) ** 2


def excitation_wavelengths_nm(sp: Species, n):
    """AtomicConfiguration.excitation_wavelength_{1,2}_nm (RG/configurations.py:640-966)."""
    lam1 = C / sp.f_ground_to_e * 1e9
    E_bind = -RY_JOULES / n_star(sp, n) ** 2
    E_photon1 = HBAR * 2 * np.pi * sp.f_ground_to_e
    f2 = (sp.E_ionization + E_bind - E_photon1) / (HBAR * 2 * np.pi)
    return lam1, C / f2 * 1e9
