"""Vectorised host-side parameter derivation for simulate_CZ_gate (hot-path row a1).

Every function takes numpy arrays over sweep points.  Together they restate
steps 0-8 of simulate_CZ_gate (RG/simulation.py:2761-3355) and the helpers it
calls:

    tweezer_spacing                       RG/trap_physics.py:265
    laser_E0 / single/two_photon_rabi     RG/laser_physics.py:111, :191, :265
    rydberg_blockade                      RG/laser_physics.py:427
    compute_trap_dependent_noise          RG/trap_physics.py:1614-1848
      trap_depth/trap_frequencies/...     RG/trap_physics.py:347-1365
    calculate_zeeman_shift                RG/trap_physics.py:1851-1965
    calculate_qubit_stark_shift           RG/trap_physics.py:2050-2142
    zeeman_dephasing_rate                 RG/noise_models.py:483
    intermediate_state_scattering_rate    RG/noise_models.py:561
    leakage_rate_to_adjacent_states       RG/noise_models.py:732
    mJ_mixing_rate / rydberg_zeeman_split RG/noise_models.py:856, :913
    build_all_noise_operators (rates)     RG/noise_models.py:1449-1620

The output is a ``DerivedBatch``: the physics-level columns the GPU engine
consumes (Omega, Delta, V, light shift, per-atom channel rates, schedule
parameters) plus the diagnostic fields SimulationResult reports.
"""
from __future__ import annotations

import warnings
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from . import protocols as P
from ._native import (STATUS_DARK_STATE_SIGN, STATUS_OMEGA_RANGE,
                      STATUS_WEAK_BLOCKADE)
from . import species as S
from .constants import C, EPS0, HBAR, KB, MU_B

# ---------------------------------------------------------------------------
# elementary formulas
# ---------------------------------------------------------------------------


def laser_E0(power, waist):
    I_peak = 2 * power / (np.pi * waist ** 2)
    return np.sqrt(2 * I_peak / (EPS0 * C))


def trap_depth(power, waist, alpha):
    I0 = 2 * power / (np.pi * waist ** 2)
    return np.abs(alpha) * I0 / (2 * EPS0 * C)


def thermal_dephasing_rate(dVV, V0, Omega):
    """RG/trap_physics.py:1118-1203 (weak / strong blockade with smoothstep blend)."""
    Omega = np.where((Omega <= 0), 2 * np.pi * 5e6, Omega)
    vo = np.abs(V0) / np.abs(Omega)
    g_weak = (dVV ** 2) * (vo ** 2) * np.abs(Omega) / (2 * np.pi)
    g_strong = (dVV ** 2) * (np.abs(Omega) / np.abs(V0)) ** 2 * np.abs(Omega) / (2 * np.pi)
    x = np.clip((vo - 3) / 7, 0, 1)
    sm = 3 * x ** 2 - 2 * x ** 3
    g_mid = g_weak * (1 - sm) + g_strong * sm
    g = np.where(vo < 3, g_weak, np.where(vo > 10, g_strong, g_mid))
    return np.minimum(g, 10e6)


def effective_antitrap_loss_rate(gate_time, U0, alpha_ratio, mass, waist, temperature,
                                 rydberg_fraction=0.3):
    """effective_loss_rate + atom_loss_probability (RG/trap_physics.py:865-1061),
    trap on during the Rydberg excursion."""
    t_ryd = rydberg_fraction * gate_time
    w_trap = np.sqrt(4 * U0 / (mass * waist ** 2))
    v_th = np.sqrt(KB * temperature / mass)
    capture = 2.0 * waist
    w_anti = np.sqrt(4 * alpha_ratio * U0 / (mass * waist ** 2))
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        sig0 = np.sqrt(KB * temperature / (mass * w_trap ** 2))
        sp = sig0 * np.cosh(w_anti * t_ryd)
        sv = (v_th / w_anti) * np.sinh(w_anti * t_ryd)
        sig = np.sqrt(sp ** 2 + sv ** 2)
        P_loss = np.where(sig > 0, 1.0 - np.exp(-(capture / sig) ** 2 / 2), 0.0)
    P_loss = np.where((w_anti > 0) & (t_ryd > 0), P_loss, 0.0)
    P_loss = np.clip(P_loss, 0.0, 1.0)
    with np.errstate(divide="ignore", invalid="ignore"):
        g = np.where(P_loss >= 0.99, 5.0 / gate_time,
                     np.where(P_loss > 0, -np.log(1 - np.minimum(P_loss, 0.99)) / gate_time, 0.0))
        max_rate = np.where(gate_time > 0, 1.0 / gate_time, 1e6)
    return np.minimum(g, max_rate)


def leakage_rate(Omega, Delta_leak, pulse_shape: str, tau, gamma_r):
    """leakage_rate_to_adjacent_states (RG/noise_models.py:732-853)."""
    x = Delta_leak * tau / (2 * np.pi)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        if pulse_shape == "square":
            sf = (np.sin(np.pi * x) / (np.pi * x)) ** 2
        elif pulse_shape == "gaussian":
            sf = np.exp(-(Delta_leak * tau / 8) ** 2)
        elif pulse_shape == "cosine":
            sf = np.where(np.abs(np.abs(x) - 0.5) < 1e-10, 0.25,
                          (np.sin(np.pi * x) / (np.pi * x * (1 - x ** 2))) ** 2)
        elif pulse_shape == "blackman":
            sf = np.exp(-3 * np.abs(x)) * 0.1
        elif pulse_shape == "drag":
            sf = np.exp(-(Delta_leak * tau / 8) ** 2) * 0.1
        else:   # smooth_sinusoidal, bangbang, ...
            sf = (np.sin(np.pi * x) / (np.pi * x + 1e-10)) ** 2
    sf = np.where(np.abs(x) < 1e-10, 1.0, sf)
    sf = np.clip(sf, 0, 1)
    g = (Omega / Delta_leak) ** 2 * gamma_r * sf
    zero = (np.abs(Delta_leak) < 1e-6) | (np.abs(Omega) < 1e-6)
    return np.where(zero, 0.0, g)


def zeeman_shift(B_field, qubit_0, qubit_1, sp: S.Species):
    """calculate_zeeman_shift (RG/trap_physics.py:1851-1965)."""
    F0, mF0 = qubit_0
    F1, mF1 = qubit_1
    if mF0 == 0 and mF1 == 0:
        B_G = np.asarray(B_field, dtype=float) * 1e4
        return sp.K_quad_zeeman * B_G ** 2 * 2 * np.pi
    g_lo, F_lo = sp.g_F_lower, sp.F_lower
    gF0 = g_lo if F0 == F_lo else -g_lo
    gF1 = g_lo if F1 == F_lo else -g_lo
    return (gF1 * mF1 - gF0 * mF0) * MU_B * np.asarray(B_field, dtype=float) / HBAR


def rydberg_zeeman_splitting(B_field):
    """S_1/2 Rydberg mJ splitting with g_J = 2 + 0.002 (RG/noise_models.py:913-963)."""
    gJ = 1 + (0.5 * 1.5 + 0.5 * 1.5 - 0) / (2 * 0.5 * 1.5) + 0.002
    return gJ * MU_B * np.asarray(B_field, dtype=float) / HBAR


# ---------------------------------------------------------------------------
# batch derivation
# ---------------------------------------------------------------------------

RATE_FIELDS = ("gamma_r", "gamma_bbr", "gamma_phi_laser", "gamma_phi_thermal",
               "gamma_phi_zeeman", "gamma_loss_antitrap", "gamma_loss_background",
               "gamma_scatter_intermediate", "gamma_leakage", "mJ_leakage_rate")


@dataclass
class DerivedBatch:
    """SoA result of the host derivation for N points of one protocol."""
    protocol: str                 # levine_pichler | jandura_pupillo | smooth_jp
    pulse_shape: str
    dim: int
    include_noise: bool
    trap_laser_on: bool
    n: int
    cols: Dict[str, np.ndarray] = field(default_factory=dict)
    bangbang_times: Optional[np.ndarray] = None     # (n, nseg-1) dimensionless
    bangbang_phases: Optional[np.ndarray] = None    # (n, nseg)
    warnings: list = field(default_factory=list)
    noise_config: Any = None                        # the NoiseSourceConfig the points share
    status_bits: Optional[np.ndarray] = None        # (n,) RYD_STATUS_* warning bits per point

    def __getitem__(self, k):
        return self.cols[k]

    def channel_rates(self):
        """Per-atom Lindblad channel rates (|1><r|, |0><r|, P_r, P_1), identical on both
        atoms.  D[sqrt(a)X] + D[sqrt(b)X] = D[sqrt(a+b)X], so the reference's 14 c_ops
        (RG/noise_models.py:1575-1592) collapse exactly onto these 4 channels per atom;
        the reference's ``rate > 0`` guards are applied per term."""
        c = self.cols
        pos = lambda a: np.where(a > 0, a, 0.0)
        b = 0.5
        g_r = pos(c["gamma_r"])
        g1 = g_r * b
        g0 = (g_r * (1 - b) + pos(c["gamma_bbr"]) + pos(c["gamma_loss_antitrap"])
              + pos(c["gamma_loss_background"]) + pos(c["gamma_leakage"]))
        gphi = pos(c["gamma_phi_laser"] + c["gamma_phi_thermal"] + c["gamma_phi_zeeman"])
        gsc = pos(c["gamma_scatter_intermediate"])
        if not self.include_noise:
            z = np.zeros(self.n)
            return z, z, z, z
        return g1, g0, gphi, gsc

    def mj_rate(self):
        """dim 4: rate of each of the two mJ-mixing channels |r-><r+|, |r+><r-| per atom
        (RG/noise_models.py:1287-1295); zero otherwise."""
        if not self.include_noise or self.dim != 4:
            return np.zeros(self.n)
        g = self.cols["mJ_leakage_rate"]
        return np.where(g > 0, g, 0.0)


def _bc(x, n):
    return np.broadcast_to(np.asarray(x, dtype=float), (n,)).astype(float)


# derive_batch's apparatus arguments that may be per-point arrays
POINT_ARGS = ("species", "n_rydberg", "tweezer_power", "tweezer_waist", "tweezer_wavelength_nm",
              "temperature", "B_field", "NA", "spacing_factor", "background_loss_rate_hz")


def _per_point(key, v):
    # bang-bang switching_times / phases given as one 1-D schedule are shared by all points
    return np.ndim(v) > 0 and not (key in ("switching_times", "phases") and np.ndim(v) == 1)


def batch_size(overrides=None, **kw) -> int:
    """The point count derive_batch infers when ``n`` is None: the longest array argument."""
    sizes = [np.size(v) for k, v in kw.items() if k in POINT_ARGS and v is not None and np.ndim(v) > 0]
    sizes += [np.shape(v)[0] for k, v in (overrides or {}).items() if _per_point(k, v)]
    return max(sizes) if sizes else 1


def slice_inputs(kw: Dict[str, Any], n: int, lo: int, hi: int) -> Dict[str, Any]:
    """derive_batch keyword arguments for points lo .. hi - 1 of an n-point call: every
    per-point array (length n along its first axis) is sliced, everything else (scalars,
    length-1 arrays that broadcast, shared schedules) passes through.  The derivation is
    elementwise, so the slice's columns are the call's rows lo .. hi - 1."""
    out = {}
    for k, v in kw.items():
        if k == "overrides" and v is not None:
            out[k] = {ok: (ov[lo:hi] if _per_point(ok, ov) and np.shape(ov)[0] == n else ov)
                      for ok, ov in v.items()}
        elif k in POINT_ARGS and v is not None and np.ndim(v) > 0 and np.shape(v)[0] == n:
            out[k] = v[lo:hi]
        else:
            out[k] = v
    return out


def concat_batches(parts: List["DerivedBatch"]) -> "DerivedBatch":
    """One DerivedBatch from consecutive slices of a call (slice_inputs)."""
    if len(parts) == 1:
        return parts[0]
    b0 = parts[0]
    cat = lambda xs: None if xs[0] is None else np.concatenate(xs)
    flags = []
    for b in parts:
        flags += [f for f in b.warnings if f not in flags]
    return DerivedBatch(protocol=b0.protocol, pulse_shape=b0.pulse_shape, dim=b0.dim,
                        include_noise=b0.include_noise, trap_laser_on=b0.trap_laser_on,
                        n=sum(b.n for b in parts),
                        cols={k: np.concatenate([b.cols[k] for b in parts]) for k in b0.cols},
                        bangbang_times=cat([b.bangbang_times for b in parts]),
                        bangbang_phases=cat([b.bangbang_phases for b in parts]),
                        warnings=flags, noise_config=b0.noise_config,
                        status_bits=cat([b.status_bits for b in parts]))


def derive_batch(simulation_inputs, n: Optional[int] = None, *, species="Rb87",
                 n_rydberg=70, qubit_0=(1, 0), qubit_1=(2, 0), hilbert_space_dim: int = 3,
                 tweezer_power=30e-3, tweezer_waist=1.0e-6, tweezer_wavelength_nm=None,
                 temperature=2e-6, B_field=1e-4, NA=0.5, spacing_factor=2.8,
                 include_noise: bool = True, background_loss_rate_hz=None,
                 trap_laser_on: bool = True, overrides: Optional[Dict[str, Any]] = None
                 ) -> DerivedBatch:
    """Derive physics columns for N points sharing one ``simulation_inputs`` object.

    Any apparatus argument may be an array (broadcast to N).  ``overrides`` may
    hold per-point arrays replacing simulation-input fields
    (laser_1_power, laser_2_power, laser_1_waist, laser_2_waist,
    laser_1_linewidth_hz, laser_2_linewidth_hz, Delta_e, delta_over_omega,
    omega_tau, A, omega_mod_ratio, phi_offset; bang-bang switching_times (n, k)
    and phases (n, k+1)) -- the batched equivalent of building one
    simulation_inputs object per point.
    """
    from .configurations import (JPSimulationInputs, LPSimulationInputs,
                                 SmoothJPSimulationInputs)
    ov = dict(overrides or {})
    si = simulation_inputs
    if isinstance(si, LPSimulationInputs):
        protocol, pulse_shape = "levine_pichler", si.pulse_shape
    elif isinstance(si, SmoothJPSimulationInputs):
        protocol, pulse_shape = "smooth_jp", "smooth_sinusoidal"
    elif isinstance(si, JPSimulationInputs):
        protocol, pulse_shape = "jandura_pupillo", "bangbang"
    else:
        raise TypeError("simulation_inputs must be LPSimulationInputs, JPSimulationInputs, "
                        f"or SmoothJPSimulationInputs, got {type(si).__name__}")
    if hilbert_space_dim not in (3, 4):
        raise ValueError(f"Unsupported Hilbert space dimension: {hilbert_space_dim}. Use 3 or 4.")

    if n is None:
        n = batch_size(species=species, n_rydberg=n_rydberg, tweezer_power=tweezer_power,
                       tweezer_waist=tweezer_waist, tweezer_wavelength_nm=tweezer_wavelength_nm,
                       temperature=temperature, B_field=B_field, NA=NA, spacing_factor=spacing_factor,
                       overrides=ov)
    exc, noise = si.excitation, si.noise
    L1, L2 = exc.laser_1, exc.laser_2
    P1 = _bc(ov.get("laser_1_power", L1.power), n)
    P2 = _bc(ov.get("laser_2_power", L2.power), n)
    w1 = _bc(ov.get("laser_1_waist", L1.waist), n)
    w2 = _bc(ov.get("laser_2_waist", L2.waist), n)
    Delta_e = _bc(ov.get("Delta_e", exc.Delta_e), n)
    nR = _bc(n_rydberg, n)
    Ptw, wtw = _bc(tweezer_power, n), _bc(tweezer_waist, n)
    T, B = _bc(temperature, n), _bc(B_field, n)
    NA_, sf_ = _bc(NA, n), _bc(spacing_factor, n)

    # combined laser linewidth (RG/simulation.py:2854): hypot of the two legs
    lw1 = ov.get("laser_1_linewidth_hz", L1.linewidth_hz)
    lw2 = ov.get("laser_2_linewidth_hz", L2.linewidth_hz)
    if lw1 is not None and lw2 is not None:
        lw = np.sqrt(_bc(lw1, n) ** 2 + _bc(lw2, n) ** 2)
    elif lw1 is not None:
        lw = _bc(lw1, n)
    elif lw2 is not None:
        lw = _bc(lw2, n)
    else:
        lw = np.full(n, 1000.0)
    if Delta_e is None or np.any(np.isnan(Delta_e)):
        raise TypeError("TwoPhotonExcitationConfig.Delta_e must be a number")

    sp_names = np.broadcast_to(np.asarray(species), (n,))
    cols: Dict[str, np.ndarray] = {}
    out_keys = ("Omega1", "Omega", "V", "R", "U0", "omega_r", "sigma_r", "dVV", "g_thermal",
                "g_scatter", "alpha_g", "alpha_r", "alpha_ratio", "g_antitrap_raw", "diff_shift",
                "enhancement", "k_eff", "v_thermal", "g_doppler", "g_intensity", "gamma_r",
                "wavelength_nm", "tau_single", "tau_total", "Delta_gate", "delta_over_omega",
                "omega_tau", "delta_zeeman", "delta_stark", "mass")
    for k in out_keys:
        cols[k] = np.zeros(n)
    flags = []
    for name in np.unique(sp_names):
        m = sp_names == name
        sp = S.get(str(name))
        nn = nR[m]
        # step 1/3: trap wavelength (RG/simulation.py:2869-2878)
        if tweezer_wavelength_nm is not None:
            lam = _bc(tweezer_wavelength_nm, n)[m] * 1e-9
        else:
            lam = np.full(m.sum(), sp.trap_wavelength)
        wl_nm = lam * 1e9
        # step 2: spacing
        R = sf_[m] * (lam / (2 * NA_[m]))
        # step 3: Rabi frequencies
        E01, E02 = laser_E0(P1[m], w1[m]), laser_E0(P2[m], w2[m])
        d_er = S.dipole_to_rydberg(sp, nn)
        Om1 = sp.dipole_1e * E01 / HBAR
        Om2 = d_er * E02 / HBAR
        Om = Om1 * Om2 / (2 * Delta_e[m])
        # step 4: blockade
        V = S.C6(sp, nn) / R ** 6
        vo = np.where(Om > 0, V / np.where(Om > 0, Om, 1.0), np.inf)
        # step 5: protocol parameters
        if protocol == "levine_pichler":
            dom_t, ot_t = P.lp_adaptive_params(vo)
            dom = _bc(ov.get("delta_over_omega", si.delta_over_omega), m.sum()) \
                if (ov.get("delta_over_omega", si.delta_over_omega) is not None) else dom_t
            ot = _bc(ov.get("omega_tau", si.omega_tau), m.sum()) \
                if (ov.get("omega_tau", si.omega_tau) is not None) else ot_t
            tau_s = ot / Om
            tau_t = 2 * tau_s
            Dg = dom * Om
        elif protocol == "jandura_pupillo":
            otv = ov.get("omega_tau", si.omega_tau)
            ot = _bc(otv if otv is not None else P.JP_BANGBANG_OMEGA_TAU, m.sum())
            tau_s = ot / Om
            tau_t = tau_s
            Dg = np.zeros(m.sum())
            dom = np.zeros(m.sum())
        else:
            otv = ov.get("omega_tau", si.omega_tau)
            ot = _bc(otv if otv is not None else P.SMOOTH_JP_DEFAULTS["omega_tau"], m.sum())
            tau_s = ot / Om
            tau_t = tau_s
            Dg = np.zeros(m.sum())
            dv = ov.get("delta_over_omega", si.delta_over_omega)
            dom = _bc(dv if dv is not None else P.SMOOTH_JP_DEFAULTS["delta_over_omega"], m.sum())
        # step 6: trap-dependent noise (compute_trap_dependent_noise)
        U0 = trap_depth(Ptw[m], wtw[m], sp.alpha_ground)
        w_r = np.sqrt(4 * U0 / (sp.mass * wtw[m] ** 2))
        sig = np.sqrt(KB * T[m] / (sp.mass * w_r ** 2))
        dVV = 6 * (np.sqrt(2) * sig) / R
        g_th = thermal_dephasing_rate(dVV, V, Om)
        g_sc = np.where((Om1 > 0) & (Delta_e[m] > 0),
                        sp.gamma_e * (Om1 / 2) ** 2 / (Delta_e[m] ** 2 + (sp.gamma_e / 2) ** 2), 0.0)
        a_g = S.ground_polarizability_at(sp, wl_nm)
        a_r = S.rydberg_polarizability_at(sp, wl_nm, nn)
        a_ratio = np.where(np.abs(a_g) > 1e-50, np.abs(a_r / a_g), 0.0)
        g_anti = np.where((a_ratio > 0) & (tau_t > 0),
                          effective_antitrap_loss_rate(tau_t, U0, a_ratio, sp.mass, wtw[m], T[m]), 0.0)
        I_c = np.where(np.abs(a_g) > 1e-50, 2 * EPS0 * C * np.abs(U0) / np.abs(a_g), 0.0)
        dshift = np.abs(a_r - a_g) * I_c / (2 * EPS0 * C * HBAR * 2 * np.pi)
        enh = 1.0 / (1.0 + np.abs(1.0 - np.where(np.abs(a_g) > 1e-50, a_r / a_g, 0.0)))
        lam1_nm, lam2_nm = S.excitation_wavelengths_nm(sp, nn)
        if noise.include_doppler_dephasing:
            k1 = 2 * np.pi / (lam1_nm * 1e-9)
            k2 = 2 * np.pi / (lam2_nm * 1e-9)
            keff = np.abs(k1 - k2) if exc.counter_propagating else k1 + k2
            g_dop = np.where(tau_t > 0, (keff * np.sqrt(KB * T[m] / sp.mass)) ** 2 * tau_t, 0.0)
            keff = np.where(tau_t > 0, keff, 0.0)
        else:
            keff = np.zeros(m.sum())
            g_dop = np.zeros(m.sum())
        if noise.include_intensity_noise and noise.intensity_noise_frac > 0:
            g_int = (U0 / HBAR) * noise.intensity_noise_frac * np.minimum(enh, 0.1)
        else:
            g_int = np.zeros(m.sum())
        g_r = 1.0 / S.rydberg_lifetime(sp, nn, 300.0)
        # step 6b: Zeeman and Stark shifts
        dz = _bc(zeeman_shift(B[m], qubit_0, qubit_1, sp), m.sum())
        if trap_laser_on:
            depth_mK = (U0 / KB * 1e6) / 1000
            ds = np.where(depth_mK > 0, sp.stark_hz_per_mK * depth_mK,
                          2.4 * 1.6488e-41 * (2 * Ptw[m] / (np.pi * wtw[m] ** 2))
                          / (4 * np.pi * EPS0 * C * HBAR)) * 2 * np.pi
        else:
            ds = np.zeros(m.sum())
        for k, v in (("Omega1", Om1), ("Omega", Om), ("V", V), ("R", R), ("U0", U0),
                     ("omega_r", w_r), ("sigma_r", sig), ("dVV", dVV), ("g_thermal", g_th),
                     ("g_scatter", g_sc), ("alpha_g", a_g), ("alpha_r", a_r),
                     ("alpha_ratio", a_ratio), ("g_antitrap_raw", g_anti), ("diff_shift", dshift),
                     ("enhancement", enh), ("k_eff", keff),
                     ("v_thermal", np.sqrt(KB * T[m] / sp.mass)), ("g_doppler", g_dop),
                     ("g_intensity", g_int), ("gamma_r", g_r), ("wavelength_nm", wl_nm),
                     ("tau_single", tau_s), ("tau_total", tau_t), ("Delta_gate", Dg),
                     ("delta_over_omega", dom), ("omega_tau", ot), ("delta_zeeman", dz),
                     ("delta_stark", ds), ("mass", np.full(m.sum(), sp.mass))):
            cols[k][m] = v
        cols.setdefault("K_quad_noise", np.zeros(n))[m] = sp.K_quad_noise

    Om = cols["Omega"]
    cols["V_over_Omega"] = np.where(Om > 0, cols["V"] / np.where(Om > 0, Om, 1.0), np.inf)
    # the reference's UserWarnings, per point (include/ryd_engine.h RYD_STATUS_* warning bits)
    bits = np.zeros(n, dtype=np.uint32)
    om_range = (Om > 2 * np.pi * 100e6) | (Om < 2 * np.pi * 0.1e6)      # RG/simulation.py:2930-2946
    bits[om_range] |= STATUS_OMEGA_RANGE
    if np.any(Om > 2 * np.pi * 100e6):
        flags.append("omega_above_physical_limit")
        warnings.warn("Ω/2π exceeds physical limit (~100 MHz). Results may be unphysical.",
                      UserWarning)
    if np.any(Om < 2 * np.pi * 0.1e6):
        flags.append("omega_very_low")
        warnings.warn("Ω/2π is very low. Gate will be very slow and susceptible to decoherence.",
                      UserWarning)
    if protocol == "levine_pichler":              # get_adaptive_protocol_params (RG/protocols.py:615-619)
        weak = cols["V_over_Omega"] < 10
        bits[weak] |= STATUS_WEAK_BLOCKADE
        if np.any(weak):
            flags.append("weak_blockade")
            warnings.warn("V/Ω < 10. Blockade too weak for reliable CZ gate!", UserWarning)

    # LP: second-pulse phase factor (RG/simulation.py:3192)
    if protocol == "levine_pichler":
        xi = P.compute_phase_shift_xi(cols["Delta_gate"], Om, cols["tau_single"])
        cols["xi_re"], cols["xi_im"] = np.real(xi), np.imag(xi)
    else:
        cols["xi_re"], cols["xi_im"] = np.ones(n), np.zeros(n)

    # smooth JP parameters (RG/simulation.py:3455-3483): `x or default` falls back
    # on 0 as well as None (reference quirk), delta sign opposite to sign(Delta_e)
    bb_t = bb_p = None
    if protocol == "smooth_jp":
        d = P.SMOOTH_JP_DEFAULTS
        def _or(key, attr):
            v = ov.get(key, getattr(si, attr))
            v = _bc(v if v is not None else 0.0, n)
            return np.where(v != 0, v, d[attr])
        cols["A"] = _or("A", "A")
        cols["omega_mod"] = _or("omega_mod_ratio", "omega_mod_ratio") * Om
        cols["phi_offset"] = _or("phi_offset", "phi_offset")
        raw = ov.get("delta_over_omega", si.delta_over_omega)
        mag = np.abs(_bc(raw if raw is not None else d["delta_over_omega"], n))
        sdom = np.where(Delta_e > 0, -mag, mag)
        if "smooth_delta_over_omega" in ov:      # ABI-level override of the signed value
            sdom = _bc(ov["smooth_delta_over_omega"], n).astype(float)
        cols["smooth_delta_over_omega"] = sdom
        # evolve_smooth_sinusoidal_jp's checks (RG/simulation.py:1631-1647, :1670-1676)
        dark_ok = np.where(Delta_e > 0, sdom < 0, sdom > 0)
        dark_bad = ~dark_ok & (sdom != 0)
        bits[dark_bad] |= STATUS_DARK_STATE_SIGN
        if np.any(dark_bad):
            flags.append("dark_state_sign")
            warnings.warn("Dark state condition violated! The two-photon detuning has the wrong sign "
                          "for the intermediate-state detuning. This will increase scattering error.",
                          UserWarning)
        weak = cols["V_over_Omega"] < 5
        bits[weak] |= STATUS_WEAK_BLOCKADE
        if np.any(weak):
            flags.append("weak_blockade")
            warnings.warn("V/Ω may be too weak for reliable CZ operation. Recommend V/Ω > 10 for "
                          "high-fidelity gates.", UserWarning)
        cols["Delta_seg"] = sdom * Om
        otv = ov.get("omega_tau", si.omega_tau)
        cols["tau_total"] = _bc(otv if otv is not None else d["omega_tau"], n) / Om
        cols["tau_single"] = cols["tau_total"].copy()
    elif protocol == "jandura_pupillo":
        # `getattr(si, ..., None) or default` (RG/simulation.py:3025-3028): an empty
        # list falls back to the defaults; per-point (n, k) arrays pass through
        def _or_default(v, default):
            if isinstance(v, np.ndarray):
                return v if v.size else list(default)
            return v or list(default)
        st = _or_default(ov.get("switching_times", si.switching_times), P.JP_BANGBANG_SWITCHING_TIMES)
        ph = _or_default(ov.get("phases", si.phases), P.JP_BANGBANG_PHASES)
        bb_t = np.broadcast_to(np.atleast_2d(np.asarray(st, dtype=float)), (n, np.shape(st)[-1])).copy()
        bb_p = np.broadcast_to(np.atleast_2d(np.asarray(ph, dtype=float)), (n, np.shape(ph)[-1])).copy()
        if bb_p.shape[1] != bb_t.shape[1] + 1:
            raise AssertionError(f"Need len(phases) = len(switching_times) + 1, got "
                                 f"{bb_p.shape[1]} phases and {bb_t.shape[1]} switching times")
        cols["Delta_seg"] = np.zeros(n)
    else:
        cols["Delta_seg"] = cols["Delta_gate"].copy()

    # step 8: noise rates (RG/simulation.py:3230-3334)
    cols["gamma_r_trap"] = cols["gamma_r"].copy()
    for k in RATE_FIELDS:
        cols[k] = np.zeros(n)
    if include_noise:
        cols["gamma_r"] = cols["gamma_r_trap"].copy()
        cols["gamma_phi_laser"] = np.pi * lw
        cols["gamma_loss_background"] = (_bc(background_loss_rate_hz, n)
                                         if background_loss_rate_hz is not None else np.full(n, 1e3))
        g_mot = cols["g_thermal"] if noise.include_motional_dephasing else np.zeros(n)
        cols["gamma_phi_thermal"] = g_mot + cols["g_doppler"] + cols["g_intensity"]
        B_rms = np.maximum(0.01 * B * 1e4, 1e-3)
        clock = qubit_0[1] == 0 and qubit_1[1] == 0
        df = 2 * cols["K_quad_noise"] * 1.0 * B_rms if clock else 700e3 * B_rms
        cols["gamma_phi_zeeman"] = 2 * np.pi * df
        tf = np.minimum(1.0, (cols["tau_total"] / 1e-6) ** 2)
        cols["gamma_loss_antitrap"] = cols["g_antitrap_raw"] * 0.3 * tf
        cols["anti_trap_time_factor"] = tf
        # Delta_leak = 2 pi 50 MHz (compute_leakage_detuning, fine_structure target,
        # RG/pulse_shaping.py:573-658); tau = step-5 tau_single
        cols["gamma_leakage"] = leakage_rate(Om, 2 * np.pi * 50e6, pulse_shape,
                                             cols["tau_single"], cols["gamma_r"])
        cols["gamma_scatter_intermediate"] = cols["g_scatter"]
        if hilbert_space_dim == 4:
            dZ = rydberg_zeeman_splitting(B)
            pur = min(L1.polarization_purity, L2.polarization_purity)
            eps = 1.0 - pur
            cols["mJ_leakage_rate"] = np.where(np.abs(dZ) < 1e-10, eps ** 2 * np.abs(Om),
                                               eps ** 2 * Om ** 2 / np.where(np.abs(dZ) < 1e-10, 1, np.abs(dZ)))
            cols["Delta_zeeman_rydberg"] = dZ
            cols["combined_polarization_purity"] = np.full(n, pur)
    return DerivedBatch(protocol=protocol, pulse_shape=pulse_shape, dim=hilbert_space_dim,
                        include_noise=include_noise, trap_laser_on=trap_laser_on, n=n, cols=cols,
                        bangbang_times=bb_t, bangbang_phases=bb_p, warnings=flags,
                        noise_config=noise, status_bits=bits)


@dataclass
class DeriveInputs:
    """Inputs of the device derivation (ryd_derive): the descriptor (shared values,
    flags, species table) and the per-point input block [k][n] of the fields that vary."""
    desc: Any                       # _native.DeriveDesc
    cols: np.ndarray                # (k, n) float64
    n: int
    protocol: str                   # lp_square | lp_shaped | smooth_jp | bangbang (engine key)
    shape: str
    dim: int
    include_noise: bool


_NONE = float("nan")


def derive_inputs(simulation_inputs, n: Optional[int] = None, *, species="Rb87",
                  n_rydberg=70, qubit_0=(1, 0), qubit_1=(2, 0), hilbert_space_dim: int = 3,
                  tweezer_power=30e-3, tweezer_waist=1.0e-6, tweezer_wavelength_nm=None,
                  temperature=2e-6, B_field=1e-4, NA=0.5, spacing_factor=2.8,
                  include_noise: bool = True, background_loss_rate_hz=None,
                  trap_laser_on: bool = True, overrides: Optional[Dict[str, Any]] = None) -> DeriveInputs:
    """The arguments of ``derive_batch`` as ryd_derive inputs: every argument that is an
    array becomes a row of the input block, every scalar a descriptor value (so a C4 sweep
    ships only its species, T and P_tweezer columns).  Same validation and defaults as
    ``derive_batch``; the device evaluates the same formulas (csrc/ryd_derive.inc)."""
    from . import _native as N
    from .configurations import (JPSimulationInputs, LPSimulationInputs,
                                 SmoothJPSimulationInputs)
    ov = dict(overrides or {})
    si = simulation_inputs
    if isinstance(si, LPSimulationInputs):
        pulse_shape = si.pulse_shape
        shape = pulse_shape.lower()
        if shape == "drag":
            raise TypeError("pulse_envelope_drag() missing 1 required positional argument: 'Delta_leak'")
        if shape not in N.SHAPE:
            raise ValueError(f"Unknown pulse shape: {pulse_shape}. "
                             f"Available shapes: ['square', 'gaussian', 'cosine', 'blackman', 'drag']")
        proto = "lp_square" if shape == "square" else "lp_shaped"
    elif isinstance(si, SmoothJPSimulationInputs):
        proto, pulse_shape, shape = "smooth_jp", "smooth_sinusoidal", "square"
    elif isinstance(si, JPSimulationInputs):
        proto, pulse_shape, shape = "bangbang", "bangbang", "square"
    else:
        raise TypeError("simulation_inputs must be LPSimulationInputs, JPSimulationInputs, "
                        f"or SmoothJPSimulationInputs, got {type(si).__name__}")
    if hilbert_space_dim not in (3, 4):
        raise ValueError(f"Unsupported Hilbert space dimension: {hilbert_space_dim}. Use 3 or 4.")
    exc, noise = si.excitation, si.noise
    L1, L2 = exc.laser_1, exc.laser_2
    De = ov.get("Delta_e", exc.Delta_e)
    if De is None or np.any(np.isnan(np.asarray(De, dtype=float))):
        raise TypeError("TwoPhotonExcitationConfig.Delta_e must be a number")
    names = list(S.SPECIES)
    sp_arr = np.asarray(species)
    if np.issubdtype(sp_arr.dtype, np.integer):        # indices into the species table (sweeps)
        if sp_arr.size and (sp_arr.min() < 0 or sp_arr.max() >= len(names)):
            raise ValueError(f"species index out of range: the table is {names}")
        sp_idx = sp_arr.astype(float) if sp_arr.ndim else float(sp_arr)
    elif sp_arr.ndim:
        u, inv = np.unique(sp_arr, return_inverse=True)
        sp_idx = np.array([names.index(S.get(str(nm)).name) for nm in u], dtype=float)[inv.ravel()]
    else:
        sp_idx = float(names.index(S.get(str(species)).name))
    fields = {
        "SPECIES": sp_idx, "N_RYD": n_rydberg,
        "P1": ov.get("laser_1_power", L1.power), "P2": ov.get("laser_2_power", L2.power),
        "W1": ov.get("laser_1_waist", L1.waist), "W2": ov.get("laser_2_waist", L2.waist),
        "DELTA_E": ov.get("Delta_e", exc.Delta_e),
        "LW1": ov.get("laser_1_linewidth_hz", L1.linewidth_hz), "LW2": ov.get("laser_2_linewidth_hz", L2.linewidth_hz),
        "TW_POWER": tweezer_power, "TW_WAIST": tweezer_waist, "TW_WL_NM": tweezer_wavelength_nm,
        "TEMPERATURE": temperature, "B_FIELD": B_field, "NA": NA, "SPACING": spacing_factor,
        "BG_LOSS": background_loss_rate_hz,
    }
    dv_ = ov.get("delta_over_omega", getattr(si, "delta_over_omega", None))
    otv = ov.get("omega_tau", si.omega_tau)
    fields["DOM"], fields["OMEGA_TAU"] = dv_, otv
    nseg = 0
    if proto == "smooth_jp":
        for key, attr, f in (("A", "A", "SJP_A"), ("omega_mod_ratio", "omega_mod_ratio", "SJP_OMR"),
                             ("phi_offset", "phi_offset", "SJP_PHI_OFF")):
            v = ov.get(key, getattr(si, attr))
            fields[f] = v if v is not None else 0.0
        fields["SJP_SDOM"] = ov.get("smooth_delta_over_omega")
    elif proto == "bangbang":
        def _or_default(v, default):
            if isinstance(v, np.ndarray):
                return v if v.size else list(default)
            return v or list(default)
        st = np.asarray(_or_default(ov.get("switching_times", si.switching_times), P.JP_BANGBANG_SWITCHING_TIMES),
                        dtype=float)
        ph = np.asarray(_or_default(ov.get("phases", si.phases), P.JP_BANGBANG_PHASES), dtype=float)
        if ph.shape[-1] != st.shape[-1] + 1:
            raise AssertionError(f"Need len(phases) = len(switching_times) + 1, got "
                                 f"{ph.shape[-1]} phases and {st.shape[-1]} switching times")
        nseg = ph.shape[-1]
        if nseg > 8:
            raise ValueError("bang-bang schedules with more than 8 segments are not supported")
        for k in range(nseg - 1):
            fields[f"BB_SWT{k}"] = st[..., k]
        for k in range(nseg):
            fields[f"BB_PHI{k}"] = ph[..., k]
    sizes = [np.shape(v)[0] for v in fields.values() if v is not None and np.ndim(v) > 0]
    if n is None:
        n = max(sizes) if sizes else 1
    desc = N.DeriveDesc()
    desc.abi_version = N.RYD_ABI_VERSION
    desc.protocol = N.PROTO[proto]
    desc.shape = N.SHAPE[shape]
    desc.leak_shape = N.DV_LEAK.get(pulse_shape, N.DV_LEAK_OTHER)
    desc.dim = hilbert_space_dim
    fl = N.DV_FLAG
    desc.flags = ((fl["NOISE"] if include_noise else 0) | (fl["TRAP_ON"] if trap_laser_on else 0)
                  | (fl["DOPPLER"] if noise.include_doppler_dephasing else 0)
                  | (fl["INTENSITY"] if noise.include_intensity_noise else 0)
                  | (fl["COUNTERPROP"] if exc.counter_propagating else 0)
                  | (fl["MOTIONAL"] if noise.include_motional_dephasing else 0))
    desc.n_species = len(names)
    desc.bb_nseg = nseg
    desc.qubit[:] = [float(qubit_0[0]), float(qubit_0[1]), float(qubit_1[0]), float(qubit_1[1])]
    desc.intensity_noise_frac = float(noise.intensity_noise_frac)
    desc.polarization_purity = float(min(L1.polarization_purity, L2.polarization_purity))
    for r, nm in enumerate(names):
        spc = S.SPECIES[nm]
        for c, k in enumerate(N.DV_SPC):
            desc.species[r][c] = float(getattr(spc, k))
    rows = []
    for k in range(N.DV_NFIELD):
        desc.col[k] = -1
        desc.value[k] = 0.0
    idx = {}
    for k, v in N.DV.items():
        idx[k] = v
    for k in range(7):
        idx[f"BB_SWT{k}"] = N.DV["BB_SWT0"] + k
    for k in range(8):
        idx[f"BB_PHI{k}"] = N.DV["BB_PHI0"] + k
    for k, v in fields.items():
        f = idx[k]
        if v is None:
            desc.value[f] = _NONE
        elif np.ndim(v) > 0:
            a = np.broadcast_to(np.asarray(v, dtype=float), (n,))
            desc.col[f] = len(rows)
            rows.append(a)
        else:
            desc.value[f] = float(v)
    if proto == "smooth_jp" and np.ndim(fields["DOM"]) == 0 and fields["DOM"] is None:
        desc.value[N.DV["DOM"]] = _NONE
    cols = np.ascontiguousarray(np.stack(rows)) if rows else np.zeros((0, n))
    return DeriveInputs(desc=desc, cols=cols, n=n, protocol=proto, shape=shape, dim=hilbert_space_dim,
                        include_noise=include_noise)


def area_correction_factor(pulse_shape: str, tau) -> np.ndarray:
    """Peak-Omega scale of a shaped LP pulse (RG/pulse_shaping.py:795-842): the
    square area tau over the trapezoid area of the envelope on linspace(0, tau, 1000).
    Gaussian/blackman are normalised by their grid maximum (:127-186, :239-293)."""
    tau = np.atleast_1d(np.asarray(tau, dtype=float))
    if pulse_shape == "square":
        return np.ones_like(tau)
    if pulse_shape == "drag":
        raise TypeError("pulse_envelope_drag() missing 1 required positional argument: 'Delta_leak'")
    out = np.empty_like(tau)
    for s in range(0, tau.size, 2048):
        tt = tau[s:s + 2048, None]
        t = np.linspace(0.0, 1.0, 1000)[None, :] * 0 + np.linspace(0, tt[:, 0], 1000).T
        if pulse_shape == "gaussian":
            sig = tt / 3.0
            env = np.exp(-(t - tt / 2) ** 2 / (2 * sig ** 2))
            env = env / env.max(axis=1, keepdims=True)
        elif pulse_shape == "cosine":
            env = np.sin(np.pi * t / tt) ** 2
        elif pulse_shape == "blackman":
            env = 0.42 - 0.5 * np.cos(2 * np.pi * t / tt) + 0.08 * np.cos(4 * np.pi * t / tt)
            env = env / env.max(axis=1, keepdims=True)
        else:
            raise ValueError(f"Unknown pulse shape: {pulse_shape}")
        area = np.trapezoid(np.abs(env), t, axis=1)
        out[s:s + 2048] = np.where(area < 1e-15, 1.0, tt[:, 0] / area)
    return out
