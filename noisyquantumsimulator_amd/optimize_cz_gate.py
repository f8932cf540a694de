"""Protocol-parameter optimiser for the CZ gate, evaluated a whole population per
GPU launch.

Drop-in for RG/optimize_cz_gate.py (RG = src/qpu_simulator/micro_physics/
neutral_atoms/rydberg_gates): the same public names, arguments and results --
``ApparatusConstraints`` (:153-277), ``SimulationCache`` (:284-355, same key
format), ``compute_cost`` (:362-431), ``extract_metrics`` (:434-451), the
parameter builders / default bounds (:458-643), ``warm_start_bounds``
(:646-704), ``OptimizationResult`` (:712-779), ``optimize_cz_gate``
(:786-1324) and ``run_baseline`` (:1331-1407).

What changes is how the objective is evaluated.  The reference calls
``simulate_CZ_gate`` once per candidate (≈0.2-1 s of QuTiP each); here
``differential_evolution(vectorized=True)`` hands the objective the whole
population, which becomes ONE ``simulate_CZ_gate_batch`` call (one engine launch
per generation).  The per-candidate semantics are unchanged: the cache is
consulted per member with the reference's keys, a failed point costs 1e6, and
the metrics are the reference's.  Vectorised DE implies ``updating='deferred'``
(scipy's rule); the reference uses scipy's default ``'immediate'``, so with
``vectorized=False`` this module evaluates one candidate per call and follows the
reference's DE trajectory exactly (still on the GPU engine).
"""
from __future__ import annotations

import hashlib
import inspect
import json
import os
import time
import warnings
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
from scipy.optimize import differential_evolution

from . import protocols as PR
from .configurations import (JPSimulationInputs, LaserParameters, LPSimulationInputs,
                             NoiseSourceConfig, SmoothJPSimulationInputs,
                             TwoPhotonExcitationConfig)

# validated / literature parameter sets (RG/protocols.py:299-306, :350-366, :447-473)
JP_SWITCHING_TIMES_VALIDATED = list(PR.JP_BANGBANG_SWITCHING_TIMES)
JP_PHASES_VALIDATED = list(PR.JP_BANGBANG_PHASES)
JP_OMEGA_TAU_VALIDATED = PR.JP_BANGBANG_OMEGA_TAU
JP_SWITCHING_TIMES_DEFAULT = [0.3328, 0.5859, 3.4340, 3.5530, 4.1204, 6.7431]
JP_PHASES_DEFAULT = [np.pi / 2, 0.0, -np.pi / 2, -np.pi / 2, 0.0, np.pi / 2, 0.0]

FAIL_COST = 1e6


# ---------------------------------------------------------------------------
# apparatus, cache, cost
# ---------------------------------------------------------------------------

@dataclass
class ApparatusConstraints:
    """Fixed hardware the optimiser cannot change (RG/optimize_cz_gate.py:153-213)."""
    laser_1_power: float = 50e-6
    laser_1_waist: float = 50e-6
    laser_2_power: float = 0.3
    laser_2_waist: float = 50e-6
    Delta_e: float = 2 * np.pi * 1e9
    laser_1_linewidth_hz: float = 100.0
    laser_2_linewidth_hz: float = 100.0
    temperature: float = 2e-6
    spacing_factor: float = 2.8
    n_rydberg: int = 70
    species: str = "Rb87"
    tweezer_power: float = 0.020
    tweezer_waist: float = 0.8e-6
    B_field: float = 1e-4
    NA: float = 0.5
    counter_propagating: bool = True

    def fingerprint(self) -> str:
        """12-hex md5 of the rounded apparatus tuple (:215-225); part of cache keys."""
        vals = (round(self.laser_1_power, 8), round(self.laser_1_waist, 8),
                round(self.laser_2_power, 8), round(self.laser_2_waist, 8),
                round(self.Delta_e, 2), self.n_rydberg, round(self.spacing_factor, 4),
                round(self.temperature, 10), self.species, round(self.tweezer_power, 6),
                round(self.tweezer_waist, 8), round(self.NA, 3))
        return hashlib.md5(str(vals).encode()).hexdigest()[:12]

    def make_excitation_config(self, pol_purity: float = 1.0) -> TwoPhotonExcitationConfig:
        leg = lambda p, w, pol, lw: LaserParameters(power=p, waist=w, polarization=pol,
                                                    polarization_purity=pol_purity, linewidth_hz=lw)
        return TwoPhotonExcitationConfig(
            laser_1=leg(self.laser_1_power, self.laser_1_waist, "pi", self.laser_1_linewidth_hz),
            laser_2=leg(self.laser_2_power, self.laser_2_waist, "sigma+", self.laser_2_linewidth_hz),
            Delta_e=self.Delta_e, counter_propagating=self.counter_propagating)

    @staticmethod
    def make_noiseless() -> NoiseSourceConfig:
        return NoiseSourceConfig(include_spontaneous_emission=False, include_intermediate_scattering=False,
                                 include_motional_dephasing=False, include_doppler_dephasing=False,
                                 include_intensity_noise=False, intensity_noise_frac=0.0,
                                 include_laser_dephasing=False, include_magnetic_dephasing=False)

    @staticmethod
    def make_full_noise() -> NoiseSourceConfig:
        return NoiseSourceConfig(include_spontaneous_emission=True, include_intermediate_scattering=True,
                                 include_motional_dephasing=True, include_doppler_dephasing=True,
                                 include_intensity_noise=True, intensity_noise_frac=0.01,
                                 include_laser_dephasing=True, include_magnetic_dephasing=True)

    def simulate_kwargs(self, spacing_factor=None) -> Dict[str, Any]:
        """The apparatus arguments the reference objective passes to simulate_CZ_gate
        (:1117-1130)."""
        return dict(species=self.species, n_rydberg=self.n_rydberg,
                    spacing_factor=self.spacing_factor if spacing_factor is None else spacing_factor,
                    temperature=self.temperature, tweezer_power=self.tweezer_power,
                    tweezer_waist=self.tweezer_waist, B_field=self.B_field, NA=self.NA)


class SimulationCache:
    """(cost, metrics) memo keyed by rounded parameter tuples (:284-355).  Keys,
    JSON layout and hit/miss accounting are the reference's, so cache files are
    interchangeable."""

    def __init__(self, precision: int = 4):
        self._store: Dict[str, Tuple[float, Dict]] = {}
        self.precision = precision
        self.hits = 0
        self.misses = 0

    def make_key(self, protocol: str, params: list, apparatus_hash: str = "") -> str:
        rounded = tuple(round(float(p), self.precision) for p in params)
        return f"{apparatus_hash}|{protocol}|{rounded}"

    def __contains__(self, key: str) -> bool:
        return key in self._store

    def __getitem__(self, key: str) -> Tuple[float, Dict]:
        self.hits += 1
        return self._store[key]

    def __setitem__(self, key: str, value: Tuple[float, Dict]):
        self._store[key] = value

    def __len__(self) -> int:
        return len(self._store)

    @property
    def hit_rate(self) -> float:
        tot = self.hits + self.misses
        return self.hits / tot if tot else 0.0

    def save(self, path: str):
        with open(path, "w") as f:
            json.dump({"precision": self.precision,
                       "entries": {k: {"cost": c, "metrics": m} for k, (c, m) in self._store.items()}},
                      f, indent=2, default=str)

    def load(self, path: str):
        if not os.path.exists(path):
            return
        with open(path) as f:
            data = json.load(f)
        self.precision = data.get("precision", self.precision)
        for k, v in data.get("entries", {}).items():
            self._store[k] = (v["cost"], v["metrics"])


_global_cache = SimulationCache(precision=4)


COST_KINDS = ("reference", "process_fidelity")
# probes of the gauge check in the optimiser and sweep paths (the full 16-probe
# check doubles the epilogue); a flag set by any probe is still a proof, an unset one says
# less
OPT_GAUGE_COPIES = 4


def compute_cost(metrics: Dict[str, float], gate_time_us: float = 0.0, time_weight: float = 0.01,
                 cost: str = "reference") -> float:
    """Percentage-infidelity cost (:362-431): 10 (1-F)^2 + 5 (1-F11)^2 + 2 (1-p)^2 in
    % units, + time_weight x t_gate; 1e6 for NaN or F < 0.5.  ``cost="process_fidelity"``:
    10 (1-F_gate)^2 % + time_weight x t_gate on the gauge-invariant average gate fidelity."""
    keys = ("avg_fidelity", "f11", "cz_phase_fidelity", "avg_gate_fidelity")
    return float(compute_cost_batch({k: np.atleast_1d(metrics.get(k, np.nan)) for k in keys},
                                    np.atleast_1d(gate_time_us), time_weight, cost)[0])


def compute_cost_batch(metrics: Dict[str, np.ndarray], gate_time_us: np.ndarray,
                       time_weight: float = 0.01, cost: str = "reference") -> np.ndarray:
    """compute_cost over arrays (one entry per candidate).

    ``cost="reference"`` (default) is the reference's cost, whose noisy avg F and phase
    fidelity come from the eigenvector-phase penalty and so depend on the eigensolver's
    gauge (RYD_STATUS_GAUGE_UNSTABLE); ``cost="process_fidelity"`` uses the average gate
    fidelity to CZ up to local Z phases (noise_models.gate_fidelity), a continuous
    function of the gate's map."""
    t = time_weight * np.asarray(gate_time_us, dtype=float)
    if cost == "process_fidelity":
        fg = np.asarray(metrics["avg_gate_fidelity"], dtype=float)
        c = 10.0 * ((1.0 - fg) * 100.0) ** 2 + t
        return np.where(np.isnan(fg) | (fg < 0.50), FAIL_COST, c)
    if cost != "reference":
        raise ValueError(f"Unknown cost {cost!r}: use one of {COST_KINDS}")
    f = np.asarray(metrics["avg_fidelity"], dtype=float)
    f11 = np.asarray(metrics["f11"], dtype=float)
    p = np.asarray(metrics["cz_phase_fidelity"], dtype=float)
    c = (10.0 * ((1.0 - f) * 100.0) ** 2 + 5.0 * ((1.0 - f11) * 100.0) ** 2
         + 2.0 * ((1.0 - p) * 100.0) ** 2 + t)
    bad = np.isnan(f) | np.isnan(f11) | np.isnan(p) | (f < 0.50)
    return np.where(bad, FAIL_COST, c)


METRIC_KEYS = ("controlled_phase_deg", "phase_error_deg", "cz_phase_fidelity", "f00", "f01", "f10",
               "f11", "avg_fidelity", "gate_time_us", "V_over_Omega", "Omega_MHz")
# carried when the evaluator provides them (the GPU evaluator does): the gauge-invariant
# fidelities and the gauge flag of the reference penalty (1.0 = flagged)
EXTRA_METRIC_KEYS = ("process_fidelity", "avg_gate_fidelity", "gauge_unstable")


def extract_metrics(result) -> Dict[str, float]:
    """Optimisation metrics of one SimulationResult (:434-451)."""
    pi, fid = result.phase_info, result.fidelities
    return {"controlled_phase_deg": pi.get("controlled_phase_deg", np.nan),
            "phase_error_deg": pi.get("phase_error_from_pi_deg", np.nan),
            "cz_phase_fidelity": pi.get("cz_phase_fidelity", np.nan),
            "f00": fid.get("00", np.nan), "f01": fid.get("01", np.nan),
            "f10": fid.get("10", np.nan), "f11": fid.get("11", np.nan),
            "avg_fidelity": result.avg_fidelity, "gate_time_us": result.tau_total * 1e6,
            "V_over_Omega": result.V_over_Omega, "Omega_MHz": result.Omega / (2 * np.pi * 1e6)}


def extract_metrics_batch(br) -> Dict[str, np.ndarray]:
    """extract_metrics for every row of a simulation.BatchResult."""
    c = br.batch.cols
    cp = br.controlled_phase
    err = np.minimum(np.abs(cp - np.pi), np.abs(cp + np.pi))
    nan = np.full(br.n, np.nan)
    return {"controlled_phase_deg": np.degrees(cp), "phase_error_deg": np.degrees(err),
            "cz_phase_fidelity": br.cz_phase_fidelity.copy(),
            "f00": br.fidelities[:, 0].copy(), "f01": br.fidelities[:, 1].copy(),
            "f10": br.fidelities[:, 2].copy(), "f11": br.fidelities[:, 3].copy(),
            "avg_fidelity": br.avg_fidelity.copy(), "gate_time_us": c["tau_total"] * 1e6,
            "V_over_Omega": c["V_over_Omega"].copy(), "Omega_MHz": c["Omega"] / (2 * np.pi * 1e6),
            "process_fidelity": nan.copy() if br.process_fidelity is None else br.process_fidelity.copy(),
            "avg_gate_fidelity": nan.copy() if br.avg_gate_fidelity is None else br.avg_gate_fidelity.copy(),
            "gauge_unstable": br.gauge_unstable.astype(float)}


# ---------------------------------------------------------------------------
# parameterisations (:458-643)
# ---------------------------------------------------------------------------

def _build_lp_inputs(params, excitation, noise) -> LPSimulationInputs:
    return LPSimulationInputs(excitation=excitation, noise=noise, delta_over_omega=float(params[0]),
                              omega_tau=float(params[1]), pulse_shape="square")


def _bangbang_times(omega_tau, fracs):
    """Fractional switching positions -> sorted absolute dimensionless times (:501-508)."""
    return np.sort(np.asarray(fracs, dtype=float), axis=-1) * np.asarray(omega_tau, dtype=float)[..., None]


def _build_jp_bangbang_inputs(params, excitation, noise, n_segments: int = 5,
                              spacing_factor_idx: Optional[int] = None) -> JPSimulationInputs:
    ns = n_segments - 1
    ot = float(params[0])
    times = _bangbang_times(np.array(ot), np.asarray(params[1:1 + ns], dtype=float))
    return JPSimulationInputs(excitation=excitation, noise=noise, omega_tau=ot,
                              switching_times=[float(t) for t in times],
                              phases=[float(p) for p in params[1 + ns:1 + ns + n_segments]])


def _build_smooth_jp_inputs(params, excitation, noise) -> SmoothJPSimulationInputs:
    return SmoothJPSimulationInputs(excitation=excitation, noise=noise, omega_tau=float(params[0]),
                                    A=float(params[1]), omega_mod_ratio=float(params[2]),
                                    phi_offset=float(params[3]), delta_over_omega=float(params[4]))


def _get_lp_bounds_and_x0() -> Tuple[list, np.ndarray]:
    return [(0.20, 0.50), (3.5, 5.5)], np.array([PR.LP_DELTA_OVER_OMEGA_DEFAULT, PR.LP_OMEGA_TAU_DEFAULT])


def _get_jp_bangbang_bounds_and_x0(n_segments: int = 5) -> Tuple[list, np.ndarray]:
    if n_segments == 5:
        ot0, times, phases, ot_b = JP_OMEGA_TAU_VALIDATED, JP_SWITCHING_TIMES_VALIDATED, JP_PHASES_VALIDATED, (5.0, 40.0)
    elif n_segments == 7:
        ot0, times, phases, ot_b = 7.0, JP_SWITCHING_TIMES_DEFAULT, JP_PHASES_DEFAULT, (3.0, 30.0)
    else:
        raise ValueError(f"Unsupported n_segments: {n_segments}. Use 5 or 7.")
    bounds = [ot_b] + [(0.01, 0.99)] * (n_segments - 1) + [(-np.pi, np.pi)] * n_segments
    x0 = np.array([ot0] + [t / ot0 for t in times] + list(phases))
    return bounds, x0


def _get_smooth_jp_bounds_and_x0() -> Tuple[list, np.ndarray]:
    d = PR.SMOOTH_JP_DEFAULTS
    bounds = [(5.0, 25.0), (0.05 * np.pi, 1.0 * np.pi), (0.5, 3.0), (0.0, 2 * np.pi), (0.001, 0.10)]
    return bounds, np.array([d["omega_tau"], d["A"], d["omega_mod_ratio"], d["phi_offset"],
                             abs(d["delta_over_omega"])])


def warm_start_bounds(opt_result: "OptimizationResult", frac: float = 0.20,
                      original_bounds: Optional[list] = None) -> Tuple[list, np.ndarray]:
    """Tight bounds around a previous optimum (:646-704): phases +-frac*pi, switching
    fractions +-frac inside [0.01, 0.99], others x(1 +- frac) (at least +-0.01),
    clamped to ``original_bounds``."""
    x0 = np.array(opt_result.best_params, dtype=float).copy()
    out = []
    for i, (name, v) in enumerate(zip(opt_result.param_names, x0)):
        if "phi" in name:
            lo, hi = v - frac * np.pi, v + frac * np.pi
        elif "frac" in name:
            lo, hi = max(0.01, v - frac), min(0.99, v + frac)
        else:
            d = max(abs(v) * frac, 0.01)
            lo, hi = v - d, v + d
        if original_bounds is not None and i < len(original_bounds):
            lo, hi = max(lo, original_bounds[i][0]), min(hi, original_bounds[i][1])
        if lo >= hi:
            lo = hi - 0.01
        out.append((lo, hi))
    return out, x0


@dataclass
class _Param:
    """One protocol's search space: names, default bounds/x0, the cache protocol
    tag, and the map from a population (S, d) to simulate_CZ_gate_batch inputs."""
    kind: str                  # lp | jp_bangbang | smooth_jp
    names: List[str]
    bounds: list
    x0: np.ndarray
    cache_protocol: str
    n_segments: Optional[int] = None

    def inputs(self, X: np.ndarray, excitation, noise):
        """-> (simulation_inputs template, per-point overrides)."""
        if self.kind == "lp":
            return (LPSimulationInputs(excitation=excitation, noise=noise, pulse_shape="square"),
                    dict(delta_over_omega=X[:, 0], omega_tau=X[:, 1]))
        if self.kind == "smooth_jp":
            return (SmoothJPSimulationInputs(excitation=excitation, noise=noise),
                    dict(omega_tau=X[:, 0], A=X[:, 1], omega_mod_ratio=X[:, 2], phi_offset=X[:, 3],
                         delta_over_omega=X[:, 4]))
        ns = self.n_segments - 1
        return (JPSimulationInputs(excitation=excitation, noise=noise),
                dict(omega_tau=X[:, 0], switching_times=_bangbang_times(X[:, 0], X[:, 1:1 + ns]),
                     phases=X[:, 1 + ns:1 + ns + self.n_segments]))


def _param_space(protocol_norm: str, n_segments: Optional[int] = None) -> _Param:
    if protocol_norm in ("lp", "levine_pichler"):
        b, x0 = _get_lp_bounds_and_x0()
        return _Param("lp", ["delta_over_omega", "omega_tau"], b, x0, "lp")
    if protocol_norm in ("jp_bangbang", "jp", "jandura_pupillo"):
        ns = n_segments if n_segments is not None else 5
        b, x0 = _get_jp_bangbang_bounds_and_x0(ns)
        names = ["omega_tau"] + [f"frac{i + 1}" for i in range(ns - 1)] + [f"phi{i}" for i in range(ns)]
        return _Param("jp_bangbang", names, b, x0, f"jp_bangbang_{ns}seg", ns)
    if protocol_norm in ("smooth_jp", "dark_state"):
        b, x0 = _get_smooth_jp_bounds_and_x0()
        return _Param("smooth_jp", ["omega_tau", "A", "omega_mod_ratio", "phi_offset", "delta_over_omega"],
                      b, x0, "smooth_jp")
    raise ValueError(f"Unknown protocol: {protocol_norm}. Use 'lp', 'jp_bangbang', or 'smooth_jp'.")


def _noise_hash(noise: NoiseSourceConfig) -> str:
    """8-hex md5 of the noise flags (:1067-1079)."""
    s = (f"se{int(noise.include_spontaneous_emission)}is{int(noise.include_intermediate_scattering)}"
         f"md{int(noise.include_motional_dephasing)}dd{int(noise.include_doppler_dephasing)}"
         f"in{int(noise.include_intensity_noise)}ld{int(noise.include_laser_dephasing)}"
         f"mg{int(noise.include_magnetic_dephasing)}")
    if noise.include_intensity_noise and noise.intensity_noise_frac:
        s += f"_inf{noise.intensity_noise_frac:.4f}"
    return hashlib.md5(s.encode()).hexdigest()[:8]


# ---------------------------------------------------------------------------
# batched evaluation
# ---------------------------------------------------------------------------

def default_batch_evaluator(simulation_inputs, n: int, include_noise: bool, overrides: Dict[str, Any],
                            *, process_fidelity: bool = False, gauge_copies: int = OPT_GAUGE_COPIES,
                            **apparatus) -> Tuple[Dict[str, np.ndarray], np.ndarray]:
    """One GPU pass over n candidates -> (metrics arrays, ok mask).  The metrics
    dict also carries the derived batch under "_batch" (noise breakdowns).
    ``process_fidelity``: also the gauge-invariant fidelities (one more engine pass for
    the qubit coherences of noisy points); the gauge check of the reference penalty is
    then skipped (the cost does not read it).  ``gauge_copies``: its probes otherwise."""
    from .simulation import simulate_CZ_gate_batch
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        br = simulate_CZ_gate_batch(simulation_inputs, n, include_noise=include_noise,
                                    overrides=overrides, process_fidelity=process_fidelity,
                                    gauge_check=not process_fidelity and gauge_copies > 0,
                                    gauge_copies=gauge_copies, **apparatus)
    m = extract_metrics_batch(br)
    m["_batch"] = br.batch
    return m, br.ok


def _check_evaluator_accepts(evaluator, ev_kw: Dict[str, Any]) -> None:
    """Raise TypeError if ``evaluator`` takes neither the keywords of ``ev_kw`` nor **kwargs
    (e.g. cost='process_fidelity' with an evaluator that cannot supply avg_gate_fidelity)."""
    try:
        sig = inspect.signature(evaluator)
    except (TypeError, ValueError):          # builtins / C callables: nothing to check
        return
    params = sig.parameters.values()
    if any(p.kind is inspect.Parameter.VAR_KEYWORD for p in params):
        return
    names = {p.name for p in params if p.kind in (inspect.Parameter.POSITIONAL_OR_KEYWORD,
                                                  inspect.Parameter.KEYWORD_ONLY)}
    missing = sorted(k for k in ev_kw if k not in names)
    if missing:
        raise TypeError(f"batch evaluator {getattr(evaluator, '__name__', evaluator)!r} does not accept "
                        f"{missing}: the requested cost needs an evaluator that supplies them")


def _evaluate_rows(evaluator, si, X_over: Dict[str, Any], n: int, include_noise: bool, apparatus_rows,
                   **ev_kw):
    """Evaluate a population; if the whole batch raises (the reference's per-call
    exception path), fall back to one candidate at a time so only the failing
    candidates get the failure cost.  ``ev_kw`` (e.g. process_fidelity=True) goes to
    the evaluator only when given, so evaluators without those keywords still work -- and an
    evaluator that cannot take them is refused up front (a TypeError caught below would
    otherwise give every candidate the failure cost silently)."""
    if ev_kw:
        _check_evaluator_accepts(evaluator, ev_kw)
    try:
        return evaluator(si, n, include_noise, X_over, **ev_kw, **apparatus_rows)
    except Exception:
        mets = {k: np.full(n, np.nan) for k in METRIC_KEYS + EXTRA_METRIC_KEYS}
        ok = np.zeros(n, bool)
        for i in range(n):
            sub = {k: (v[i:i + 1] if np.ndim(v) > 0 else v) for k, v in X_over.items()}
            app = {k: (v[i:i + 1] if np.ndim(v) > 0 else v) for k, v in apparatus_rows.items()}
            try:
                m, o = evaluator(si, 1, include_noise, sub, **ev_kw, **app)
            except Exception:
                continue
            for k in METRIC_KEYS:
                mets[k][i] = m[k][0]
            for k in EXTRA_METRIC_KEYS:
                if k in m:
                    mets[k][i] = m[k][0]
            ok[i] = o[0]
        return mets, ok


# ---------------------------------------------------------------------------
# result
# ---------------------------------------------------------------------------

@dataclass
class OptimizationResult:
    """Same fields as RG/optimize_cz_gate.py:712-751."""
    success: bool
    protocol: str
    best_params: np.ndarray
    param_names: List[str]
    best_cost: float
    best_metrics: Dict[str, float]
    n_evaluations: int
    runtime_s: float
    discrete_variant: str = ""
    all_variants: Dict[str, Any] = field(default_factory=dict)
    cache_hits: int = 0
    n_batches: int = 0          # engine passes (new: one per DE generation / polish step)
    cost: str = "reference"     # the cost minimised (COST_KINDS)
    n_simulated: int = 0        # candidates evaluated by the engine (cache misses)
    gauge_flagged: int = 0      # of those, noisy points whose reference penalty was gauge-flagged

    @property
    def gauge_flagged_fraction(self) -> float:
        """Fraction of simulated candidates whose reference phase penalty (and so the
        reference cost) depends on the eigensolver's gauge; a lower bound (4 probes)."""
        return self.gauge_flagged / self.n_simulated if self.n_simulated else 0.0

    def __repr__(self) -> str:
        m = self.best_metrics
        rows = [("Success", f"{self.success}"), ("Variant", self.discrete_variant),
                ("Cost", f"{self.best_cost:.4f}"),
                ("Avg fidelity", f"{m.get('avg_fidelity', 0):.6f}  ({(1 - m.get('avg_fidelity', 0)) * 100:.4f}% error)"),
                ("F(|11>)", f"{m.get('f11', 0):.6f}"), ("CZ phase fid", f"{m.get('cz_phase_fidelity', 0):.6f}"),
                ("Phase error", f"{m.get('phase_error_deg', 999):.2f} deg"),
                ("Controlled phase", f"{m.get('controlled_phase_deg', 0):.2f} deg"),
                ("Gate time", f"{m.get('gate_time_us', 0):.3f} us"), ("V/Omega", f"{m.get('V_over_Omega', 0):.1f}"),
                ("Omega/2pi", f"{m.get('Omega_MHz', 0):.3f} MHz"), ("Evaluations", f"{self.n_evaluations}"),
                ("Engine batches", f"{self.n_batches}"), ("Runtime", f"{self.runtime_s:.1f} s"),
                ("Cache hits", f"{self.cache_hits}"), ("Cost", self.cost),
                ("Gauge-flagged", f"{self.gauge_flagged} of {self.n_simulated} simulated")]
        out = ["=" * 70, f"  CZ Gate Optimisation Result -- {self.protocol}", "=" * 70]
        out += [f"  {k + ':':18s}{v}" for k, v in rows]
        out += ["-" * 70, "  Optimal parameters:"]
        out += [f"    {n:25s} = {v:.6f}" for n, v in zip(self.param_names, self.best_params)]
        out.append("=" * 70)
        return "\n".join(out)


# ---------------------------------------------------------------------------
# optimiser
# ---------------------------------------------------------------------------

def _normalise(protocol: str) -> str:
    p = protocol.lower().replace("-", "_").replace(" ", "_")
    if p not in {"lp", "levine_pichler", "jp_bangbang", "jp", "jandura_pupillo", "smooth_jp", "dark_state"}:
        raise ValueError(f"Unknown protocol: {protocol}. Use 'lp', 'jp_bangbang', or 'smooth_jp'.")
    return p


def optimize_cz_gate(protocol: str, apparatus: ApparatusConstraints, include_noise: bool = False,
                     noise_config: Optional[NoiseSourceConfig] = None, time_weight: float = 0.01,
                     optimize_spacing: bool = False, spacing_bounds: Optional[Tuple[float, float]] = None,
                     maxiter: int = 80, popsize: int = 15, tol: float = 1e-6, seed: int = 42,
                     bounds: Optional[list] = None, x0: Optional[np.ndarray] = None,
                     cache: Optional[SimulationCache] = None, cache_path: Optional[str] = None,
                     strategy: str = "standard", variant: Optional[str] = None, verbose: bool = True,
                     vectorized: bool = True, evaluator: Optional[Callable] = None,
                     cost: str = "reference") -> OptimizationResult:
    """Differential-evolution search of the protocol parameters (RG/optimize_cz_gate.py:786-990).

    Extra keywords: ``vectorized`` (default True: one engine pass per DE generation,
    scipy's deferred updating; False: one candidate per call, the reference's
    immediate updating), ``evaluator`` (the batched metrics function, default
    the GPU engine; tests inject the CPU oracle) and ``cost`` ("reference", the
    default, or "process_fidelity": the gauge-invariant average gate fidelity, see
    compute_cost_batch).  The result reports how many simulated candidates had a
    gauge-flagged reference penalty (``gauge_flagged``)."""
    pn = _normalise(protocol)
    if cost not in COST_KINDS:
        raise ValueError(f"Unknown cost {cost!r}: use one of {COST_KINDS}")
    is_bb = pn in ("jp_bangbang", "jp", "jandura_pupillo")
    excitation = apparatus.make_excitation_config(pol_purity=0.99 if include_noise else 1.0)
    noise = noise_config if noise_config is not None else (
        apparatus.make_full_noise() if include_noise else apparatus.make_noiseless())
    cache = _global_cache if cache is None else cache
    if cache_path:
        cache.load(cache_path)
    if is_bb:
        allowed = {"5-segment": 5, "7-segment": 7}
        if variant is not None and variant not in allowed:
            raise ValueError(f"Unknown variant '{variant}'. Use '5-segment' or '7-segment'.")
        variants = {variant: allowed[variant]} if variant else dict(allowed)
    else:
        variants = {"default": None}
    if verbose:
        print("=" * 70)
        print(f"  CZ Gate Optimisation -- {protocol}  ({apparatus.species}, n={apparatus.n_rydberg}, "
              f"noise {'ON' if include_noise else 'OFF'}, {'batched' if vectorized else 'per-point'})")
        print("=" * 70)
    results = {}
    for name, nseg in variants.items():
        r = _optimize_single_variant(pn, nseg, excitation, noise, apparatus, include_noise, time_weight,
                                     maxiter, popsize, tol, seed, bounds, x0, cache, strategy, verbose,
                                     optimize_spacing, spacing_bounds, vectorized,
                                     evaluator or default_batch_evaluator, cost)
        r.discrete_variant = name
        results[name] = r
        if verbose:
            print(f"    -> {name}: cost={r.best_cost:.4f}, F={r.best_metrics.get('avg_fidelity', 0):.6f}, "
                  f"phase_err={r.best_metrics.get('phase_error_deg', 999):.2f} deg")
    best_name = min(results, key=lambda k: results[k].best_cost)
    best = results[best_name]
    best.all_variants = {k: {"cost": v.best_cost, "avg_fidelity": v.best_metrics.get("avg_fidelity", 0),
                             "phase_error_deg": v.best_metrics.get("phase_error_deg", 999),
                             "params": np.asarray(v.best_params).tolist()} for k, v in results.items()}
    if cache_path:
        cache.save(cache_path)
    if verbose:
        print(f"\n  Best variant: {best_name}")
        print(best)
    return best


class _Objective:
    """The DE objective over a population: cache lookups per member with the
    reference's keys, ONE batched evaluation of the misses, cost per member."""

    def __init__(self, space: _Param, excitation, noise, apparatus: ApparatusConstraints,
                 include_noise: bool, time_weight: float, cache: SimulationCache, optimize_spacing: bool,
                 evaluator: Callable, verbose: bool, cost: str = "reference"):
        self.space, self.excitation, self.noise = space, excitation, noise
        self.apparatus, self.include_noise, self.time_weight = apparatus, include_noise, time_weight
        self.cache, self.optimize_spacing, self.evaluator, self.verbose = cache, optimize_spacing, evaluator, verbose
        self.app_hash = apparatus.fingerprint()
        self.noise_hash = _noise_hash(noise)
        self.n_eval = 0
        self.n_hits = 0
        self.n_batches = 0
        self.n_sim = 0
        self.n_flagged = 0
        self.cost = cost
        self.best = np.inf
        self.d = len(space.names)

    def split(self, X: np.ndarray):
        if self.optimize_spacing:
            return X[:, :self.d], X[:, self.d]
        return X, np.full(X.shape[0], self.apparatus.spacing_factor)

    def key(self, prot: np.ndarray, sf: float) -> str:
        h = self.app_hash if not self.optimize_spacing else f"{self.app_hash}_sf{sf:.6f}"
        # the reference cost keeps the reference's key; another cost must not share entries
        tag = "" if self.cost == "reference" else f"_{self.cost}"
        return self.cache.make_key(self.space.cache_protocol, prot.tolist(), f"{h}_n{self.noise_hash}{tag}")

    def evaluate(self, X: np.ndarray) -> Tuple[np.ndarray, List[Optional[Dict]]]:
        """X (S, D) -> (costs (S,), metrics dict or None per member)."""
        X = np.atleast_2d(X)
        S = X.shape[0]
        prot, sf = self.split(X)
        keys = [self.key(prot[i], sf[i]) for i in range(S)]
        costs = np.empty(S)
        mets: List[Optional[Dict]] = [None] * S
        miss = []
        for i, k in enumerate(keys):
            self.n_eval += 1
            if k in self.cache:
                self.n_hits += 1
                costs[i], mets[i] = self.cache[k]
            else:
                self.cache.misses += 1
                miss.append(i)
        if miss:
            idx = np.array(miss)
            si, over = self.space.inputs(prot[idx], self.excitation, self.noise)
            app = self.apparatus.simulate_kwargs(spacing_factor=sf[idx] if self.optimize_spacing else None)
            ev_kw = {"process_fidelity": True} if self.cost == "process_fidelity" else {}
            m, ok = _evaluate_rows(self.evaluator, si, over, idx.size, self.include_noise, app, **ev_kw)
            self.n_batches += 1
            self.n_sim += idx.size
            if "gauge_unstable" in m:
                self.n_flagged += int(np.nansum(np.asarray(m["gauge_unstable"], dtype=float)[ok] > 0))
            c = compute_cost_batch(m, m["gate_time_us"], self.time_weight, self.cost)
            c = np.where(ok, c, FAIL_COST)
            for j, i in enumerate(miss):
                costs[i] = c[j]
                if ok[j]:
                    mets[i] = {k: float(m[k][j]) for k in METRIC_KEYS}
                    mets[i].update({k: float(m[k][j]) for k in EXTRA_METRIC_KEYS if k in m})
                    self.cache[keys[i]] = (float(c[j]), mets[i])
                if c[j] < self.best:
                    self.best = c[j]
                    if self.verbose and mets[i] is not None:
                        mm = mets[i]
                        print(f"    [{self.n_eval - S + i + 1:5d}] cost={c[j]:10.4f}  F={mm['avg_fidelity']:.6f}  "
                              f"F11={mm['f11']:.6f}  CZphi={mm['cz_phase_fidelity']:.4f}  "
                              f"phi_err={mm['phase_error_deg']:.2f}  t={mm['gate_time_us']:.3f}us")
        return costs, mets

    def vec(self, x: np.ndarray) -> np.ndarray:      # scipy vectorized: x (D, S)
        return self.evaluate(np.asarray(x).T)[0]

    def scalar(self, x: np.ndarray) -> float:
        return float(self.evaluate(np.asarray(x)[None, :])[0][0])


def _run_de(obj: _Objective, bounds, x0, maxiter, popsize, tol, seed, vectorized, **kw):
    fn = obj.vec if vectorized else obj.scalar
    extra = dict(vectorized=True, updating="deferred") if vectorized else {}
    extra.update(kw)
    return differential_evolution(fn, bounds=bounds, x0=x0, maxiter=maxiter, popsize=popsize, tol=tol,
                                  seed=seed, polish=True, disp=False, **extra)


def _optimize_single_variant(pn, n_segments, excitation, noise, apparatus, include_noise, time_weight,
                             maxiter, popsize, tol, seed, bounds, x0, cache, strategy, verbose,
                             optimize_spacing, spacing_bounds, vectorized, evaluator,
                             cost: str = "reference") -> OptimizationResult:
    """DE for one discrete variant (:993-1324)."""
    space = _param_space(pn, n_segments)
    names = list(space.names)
    bounds = list(space.bounds if bounds is None else bounds)
    x0 = np.array(space.x0 if x0 is None else x0, dtype=float)
    if optimize_spacing:
        bounds = bounds + [spacing_bounds or (1.5, 5.0)]
        x0 = np.append(x0, apparatus.spacing_factor)
        names.append("spacing_factor")
    obj = _Objective(space, excitation, noise, apparatus, include_noise, time_weight, cache,
                     optimize_spacing, evaluator, verbose, cost)
    t0 = time.time()
    if strategy == "two_phase" and space.kind == "smooth_jp":
        # phase 1: omega_tau (and spacing) only, the other shape parameters at x0 (:1184-1241)
        fixed = x0.copy()
        sub = [0] + ([len(bounds) - 1] if optimize_spacing else [])

        def expand(Y):
            Y = np.atleast_2d(Y)
            full = np.repeat(fixed[None, :], Y.shape[0], axis=0)
            full[:, sub] = Y
            return full

        p1 = _Objective(space, excitation, noise, apparatus, include_noise, time_weight, cache,
                        optimize_spacing, evaluator, verbose, cost)
        fn = (lambda y: p1.evaluate(expand(np.asarray(y).T))[0]) if vectorized else \
             (lambda y: float(p1.evaluate(expand(np.asarray(y)))[0][0]))
        extra = dict(vectorized=True, updating="deferred") if vectorized else {}
        r1 = differential_evolution(fn, bounds=[bounds[i] for i in sub], x0=x0[sub], maxiter=max(20, maxiter // 4),
                                    popsize=10, tol=tol, seed=seed, polish=True, disp=False, **extra)
        obj.n_eval += p1.n_eval
        obj.n_hits += p1.n_hits
        obj.n_batches += p1.n_batches
        obj.n_sim += p1.n_sim
        obj.n_flagged += p1.n_flagged
        x0 = expand(r1.x)[0]
        ot = r1.x[0]
        bounds = [(max(bounds[0][0], ot * 0.7), min(bounds[0][1], ot * 1.3))] + bounds[1:]
        if verbose:
            print(f"    Phase 1 best Omega*tau = {ot:.3f}, cost = {r1.fun:.4f}")
    de = _run_de(obj, bounds, x0, maxiter, popsize, tol, seed, vectorized)
    runtime = time.time() - t0
    # final metrics: from the cache (the reference's path, :1274-1306), else one re-evaluation
    xf = np.asarray(de.x)[None, :]
    prot, sf = obj.split(xf)
    fkey = obj.key(prot[0], sf[0])
    if fkey in cache:
        final = cache[fkey][1]
    else:
        n_eval = obj.n_eval
        final = obj.evaluate(xf)[1][0]
        obj.n_eval = n_eval
    final = final or {"avg_fidelity": 0, "phase_error_deg": 999, "f11": 0}
    success = (final.get("avg_fidelity", 0) >= 0.99 and final.get("cz_phase_fidelity", 0) >= 0.99
               and final.get("phase_error_deg", 999) < 10.0)
    return OptimizationResult(success=success, protocol=pn, best_params=np.asarray(de.x), param_names=names,
                              best_cost=float(de.fun), best_metrics=final, n_evaluations=obj.n_eval,
                              runtime_s=runtime, cache_hits=obj.n_hits, n_batches=obj.n_batches, cost=cost,
                              n_simulated=obj.n_sim, gauge_flagged=obj.n_flagged)


def run_baseline(protocol: str, apparatus: ApparatusConstraints, include_noise: bool = False,
                 verbose: bool = True, evaluator: Optional[Callable] = None) -> Dict[str, float]:
    """Default protocol parameters, no optimisation (:1331-1407)."""
    pn = _normalise(protocol)
    excitation = apparatus.make_excitation_config(pol_purity=0.99 if include_noise else 1.0)
    noise = apparatus.make_full_noise() if include_noise else apparatus.make_noiseless()
    if pn in ("lp", "levine_pichler"):
        si = LPSimulationInputs(excitation=excitation, noise=noise)
    elif pn in ("jp_bangbang", "jp", "jandura_pupillo"):
        si = JPSimulationInputs(excitation=excitation, noise=noise)
    else:
        si = SmoothJPSimulationInputs(excitation=excitation, noise=noise)
    m, ok = (evaluator or default_batch_evaluator)(si, 1, include_noise, {}, **apparatus.simulate_kwargs())
    if not ok[0]:
        raise RuntimeError("engine reported a failure for the baseline point")
    metrics = {k: float(m[k][0]) for k in METRIC_KEYS}
    if verbose:
        print(f"\n  Baseline -- {protocol}")
        for k in ("avg_fidelity", "f11", "cz_phase_fidelity", "phase_error_deg", "controlled_phase_deg",
                  "gate_time_us", "V_over_Omega", "Omega_MHz"):
            print(f"  {k:22s} {metrics[k]:.6f}")
        print(f"  cost (ref)             {compute_cost(metrics, metrics['gate_time_us']):.4f}")
    return metrics


__all__ = ["ApparatusConstraints", "SimulationCache", "compute_cost", "compute_cost_batch", "COST_KINDS",
           "extract_metrics", "extract_metrics_batch", "warm_start_bounds", "OptimizationResult",
           "optimize_cz_gate", "run_baseline", "default_batch_evaluator"]
