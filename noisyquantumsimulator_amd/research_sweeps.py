"""The parameter-sweep driver of examples/research_parameter_sweeps.py on the engine.

The reference loops in Python: for every value of one parameter it calls
``run_single_simulation`` twice -- Levine-Pichler (pulse shape from DEFAULT_PARAMS,
"square") and Jandura-Pupillo bang-bang -- each a full ``simulate_CZ_gate``
(:81-135, :138-195).  Here ``run_sweep`` keeps that contract (same arguments, same
``SweepResult``, same defaults and quirks) and evaluates all values of a protocol in
ONE ``simulate_CZ_gate_batch`` call:

* ``run_single_simulation``'s inputs (:81-135): laser 1 waist 1 um and laser 2 waist
  10 um whatever the sweep, both legs with LaserParameters' default polarisation,
  ``NoiseSourceConfig(include_motional_dephasing=True)``, DEFAULT_PARAMS (:63-78) for
  anything not swept or fixed, ``tweezer_waist`` 1 um unless given;
* a value whose reference call raises (``Delta_e=None`` -> TypeError in
  two_photon_rabi, an unknown pulse shape -> ValueError, ...) or whose engine point
  fails becomes a NaN row with an empty noise breakdown (:133-135, :164-181) instead of
  an exception;
* unknown parameter names are ignored, as ``params.get`` ignores them.

Extra fields beyond the reference's SweepResult: per-point status bits
(include/ryd_engine.h RYD_STATUS_*) for both protocols.
"""
from __future__ import annotations

import warnings
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import numpy as np

from . import _native as N
from .configurations import (JPSimulationInputs, LaserParameters, LPSimulationInputs, NoiseSourceConfig,
                             TwoPhotonExcitationConfig)

# examples/research_parameter_sweeps.py:63-78
DEFAULT_PARAMS: Dict[str, Any] = {
    "species": "Rb87",
    "n_rydberg": 70,
    "temperature": 20e-6,
    "laser_linewidth_hz": 100.0,
    "Delta_e": 2 * np.pi * 1e9,
    "spacing_factor": 1.5,
    "rydberg_power_1": 2.5e-3,
    "rydberg_power_2": 1.0,
    "tweezer_power": 10e-3,
    "NA": 0.5,
    "B_field": 0.0,
    "pulse_shape": "square",
    "include_noise": True,
    "verbose": False,
}

# the sweeps of main() (:644-813), in SI units
DEFAULT_SWEEPS: Dict[str, np.ndarray] = {
    "temperature": np.array([5, 10, 20, 40, 80, 150]) * 1e-6,
    "laser_linewidth_hz": np.array([10, 50, 100, 500, 1000, 5000], dtype=float),
    "Delta_e": 2 * np.pi * np.array([0.5, 1, 2, 5, 10]) * 1e9,
    "spacing_factor": np.array([1.2, 1.5, 2.0, 2.5, 3.0]),
    "n_rydberg": np.array([50, 60, 70, 80, 90]),
    "rydberg_power_2": np.array([0.1, 0.3, 0.5, 1.0, 2.0, 5.0]),
    "tweezer_power": np.array([1, 3, 5, 10, 20, 50]) * 1e-3,
    "NA": np.array([0.3, 0.4, 0.5, 0.6, 0.7]),
}

_APPARATUS = ("species", "n_rydberg", "temperature", "spacing_factor", "tweezer_power", "tweezer_waist",
              "B_field", "NA")
_OVERRIDES = {"rydberg_power_1": ("laser_1_power",), "rydberg_power_2": ("laser_2_power",),
              "laser_linewidth_hz": ("laser_1_linewidth_hz", "laser_2_linewidth_hz"),
              "Delta_e": ("Delta_e",)}


@dataclass
class SweepResult:
    """examples/research_parameter_sweeps.py:48-59 (+ per-point status bits)."""
    param_values: np.ndarray
    fidelities_lp: np.ndarray
    fidelities_jp: np.ndarray
    gate_times_lp: np.ndarray
    gate_times_jp: np.ndarray
    v_over_omega_lp: np.ndarray
    v_over_omega_jp: np.ndarray
    noise_breakdowns_lp: list
    noise_breakdowns_jp: list
    status_lp: Optional[np.ndarray] = None
    status_jp: Optional[np.ndarray] = None


def _inputs(protocol: str, params: Dict[str, Any]):
    """run_single_simulation's simulation_inputs (:88-115).  Laser powers, linewidths and
    Delta_e enter the batch as per-point overrides; these are the shared defaults."""
    lw = params.get("laser_linewidth_hz", 100.0)
    l1 = LaserParameters(power=params.get("rydberg_power_1", 2.5e-3), waist=1.0e-6,
                         linewidth_hz=lw if np.ndim(lw) == 0 else 100.0)
    l2 = LaserParameters(power=params.get("rydberg_power_2", 1.0), waist=10e-6,
                         linewidth_hz=lw if np.ndim(lw) == 0 else 100.0)
    de = params.get("Delta_e", None)
    exc = TwoPhotonExcitationConfig(laser_1=l1, laser_2=l2, Delta_e=de if np.ndim(de) == 0 else 2 * np.pi * 1e9)
    noise = NoiseSourceConfig(include_motional_dephasing=True)
    if protocol.lower() in ("levine_pichler", "lp"):
        return LPSimulationInputs(excitation=exc, noise=noise, pulse_shape=params.get("pulse_shape", "time_optimal"))
    return JPSimulationInputs(excitation=exc, noise=noise)


SWEEP_GAUGE_COPIES = 4


def _batch_call(protocol: str, rows: List[Dict[str, Any]], devices=None):
    """One simulate_CZ_gate_batch over rows that share every non-array setting."""
    from .simulation import simulate_CZ_gate_batch
    p0 = rows[0]
    n = len(rows)
    kw: Dict[str, Any] = {}
    for k in _APPARATUS:
        vals = [r.get(k, {"tweezer_waist": 1e-6, "species": "Rb87", "n_rydberg": 70, "temperature": 5e-6,
                          "spacing_factor": 3.0, "tweezer_power": 30e-3, "B_field": 1e-4, "NA": 0.5}[k])
                for r in rows]
        kw[k] = np.asarray(vals) if k != "species" else np.asarray(vals, dtype=object).astype(str)
    ov: Dict[str, Any] = {}
    for src, dsts in _OVERRIDES.items():
        vals = np.asarray([r.get(src, DEFAULT_PARAMS.get(src)) for r in rows], dtype=float)
        for d in dsts:
            ov[d] = vals
    si = _inputs(protocol, p0)
    # 4 gauge probes instead of 16: the flag stays a proof where set
    return simulate_CZ_gate_batch(si, n, include_noise=bool(p0.get("include_noise", True)), overrides=ov,
                                  devices=devices, gauge_copies=SWEEP_GAUGE_COPIES, **kw)


def _fails_like_reference(protocol: str, row: Dict[str, Any]) -> Optional[str]:
    """The exception the reference's simulate_CZ_gate would raise for this row, if any
    (those rows become NaN, examples/research_parameter_sweeps.py:133-135)."""
    de = row.get("Delta_e", None)
    if de is None or not np.isfinite(float(de)):
        return "two_photon_rabi: Delta_e is None (TypeError)"
    if row.get("species", "Rb87") not in ("Rb87", "Cs133"):
        return f"unknown species {row.get('species')!r}"
    if protocol.lower() in ("levine_pichler", "lp"):
        shape = str(row.get("pulse_shape", "time_optimal")).lower()
        if shape == "drag":
            return "pulse_envelope_drag() missing 1 required positional argument: 'Delta_leak'"
        if shape not in ("square", "gaussian", "cosine", "blackman"):
            return f"Unknown pulse shape: {shape}"
    return None


def _evaluate(protocol: str, rows: List[Dict[str, Any]], devices=None):
    """Per row: (avg_fidelity, gate_time_us, V_over_Omega, noise_breakdown, status)."""
    from .simulation import noise_breakdown_row
    n = len(rows)
    F, T, VO = np.full(n, np.nan), np.full(n, np.nan), np.full(n, np.nan)
    NB: List[Dict[str, Any]] = [{} for _ in range(n)]
    ST = np.zeros(n, np.uint32)
    ok = [i for i in range(n) if _fails_like_reference(protocol, rows[i]) is None]
    # rows that share the settings a batch cannot vary go together
    groups: Dict[Any, List[int]] = {}
    for i in ok:
        r = rows[i]
        key = (str(r.get("pulse_shape", "time_optimal")).lower(), bool(r.get("include_noise", True)))
        groups.setdefault(key, []).append(i)
    for idx in groups.values():
        try:
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                br = _batch_call(protocol, [rows[i] for i in idx], devices)
        except Exception as e:             # the reference would have raised for these rows
            print(f"  Warning: {protocol} simulation failed: {e}")
            continue
        c = br.batch.cols
        for k, i in enumerate(idx):
            ST[i] = br.status[k]
            if not br.ok[k]:
                continue
            F[i] = br.avg_fidelity[k]
            T[i] = c["tau_total"][k] * 1e6
            VO[i] = c["V_over_Omega"][k]
            NB[i] = noise_breakdown_row(br.batch, k)
    return F, T, VO, NB, ST


def run_single_simulation(protocol: str, **kwargs):
    """examples/research_parameter_sweeps.py:81-135: one point, SimulationResult or None."""
    from .simulation import simulate_CZ_gate
    params = DEFAULT_PARAMS.copy()
    params.update(kwargs)
    try:
        why = _fails_like_reference(protocol, params)
        if why:
            raise TypeError(why)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            lw = params.get("laser_linewidth_hz", 100.0)
            exc = TwoPhotonExcitationConfig(
                laser_1=LaserParameters(power=params.get("rydberg_power_1", 2.5e-3), waist=1.0e-6, linewidth_hz=lw),
                laser_2=LaserParameters(power=params.get("rydberg_power_2", 1.0), waist=10e-6, linewidth_hz=lw),
                Delta_e=params.get("Delta_e", None))
            noise = NoiseSourceConfig(include_motional_dephasing=True)
            if protocol.lower() in ("levine_pichler", "lp"):
                si = LPSimulationInputs(excitation=exc, noise=noise,
                                        pulse_shape=params.get("pulse_shape", "time_optimal"))
            else:
                si = JPSimulationInputs(excitation=exc, noise=noise)
            return simulate_CZ_gate(
                simulation_inputs=si, species=params.get("species", "Rb87"),
                n_rydberg=params.get("n_rydberg", 70), temperature=params.get("temperature", 5e-6),
                spacing_factor=params.get("spacing_factor", 3.0), tweezer_power=params.get("tweezer_power", 30e-3),
                tweezer_waist=params.get("tweezer_waist", 1e-6), B_field=params.get("B_field", 1e-4),
                NA=params.get("NA", 0.5), include_noise=params.get("include_noise", True),
                verbose=params.get("verbose", False))
    except Exception as e:
        print(f"  Warning: {protocol} simulation failed: {e}")
        return None


def run_sweep(param_name: str, param_values, verbose: bool = True, devices=None, **fixed_kwargs) -> SweepResult:
    """examples/research_parameter_sweeps.py:138-195, one engine call per protocol."""
    values = list(param_values)
    rows = []
    for v in values:
        p = DEFAULT_PARAMS.copy()
        p.update(fixed_kwargs)
        p[param_name] = v
        rows.append(p)
    if verbose:
        print(f"\nSweeping {param_name} ({len(values)} points)...")
    f_lp, t_lp, vo_lp, nb_lp, st_lp = _evaluate("levine_pichler", rows, devices)
    f_jp, t_jp, vo_jp, nb_jp, st_jp = _evaluate("jandura_pupillo", rows, devices)
    if verbose:
        for i, v in enumerate(values):
            vs = f"{v:.4g}" if isinstance(v, (int, float, np.number)) else str(v)
            print(f"  [{i + 1}/{len(values)}] {param_name}={vs}: LP={f_lp[i]:.4f}, JP={f_jp[i]:.4f}")
    return SweepResult(param_values=np.asarray(param_values), fidelities_lp=f_lp, fidelities_jp=f_jp,
                       gate_times_lp=t_lp, gate_times_jp=t_jp, v_over_omega_lp=vo_lp, v_over_omega_jp=vo_jp,
                       noise_breakdowns_lp=nb_lp, noise_breakdowns_jp=nb_jp, status_lp=st_lp, status_jp=st_jp)


def run_default_sweeps(verbose: bool = False, devices=None) -> Dict[str, SweepResult]:
    """The eight one-parameter sweeps of main() (:655-770) and the species comparison
    (:772-784), without the plotting."""
    out = {name: run_sweep(name, vals, verbose=verbose, devices=devices) for name, vals in DEFAULT_SWEEPS.items()}
    t = np.array([10, 20, 40, 80]) * 1e-6
    out["species_Rb87"] = run_sweep("temperature", t, verbose=verbose, devices=devices, species="Rb87")
    out["species_Cs133"] = run_sweep("temperature", t, verbose=verbose, devices=devices, species="Cs133")
    return out
