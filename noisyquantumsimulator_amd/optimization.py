"""Hardware-parameter inverse problem and Pareto exploration, a whole DE
population per GPU launch.

Drop-in for RG/optimization.py (RG = src/qpu_simulator/micro_physics/
neutral_atoms/rydberg_gates): ``HardwareOptimizationResult`` (:92-123),
``EvaluatedPoint`` / ``ExplorationResult`` (:131-273), ``optimize_CZ_parameters``
(:280-739), ``explore_parameter_space`` (:746-980), ``combine_explorations``
(:983-1000) -- same arguments, objectives, penalties and reference quirks
(fixed 50 um laser waists and sigma+ default polarisation in the inverse
problem; 1 um / 10 um waists and bang-bang ``JPSimulationInputs`` for non-LP
exploration; ``protocol == "two_pulse"`` builds JP inputs; Delta_e in Hz).

``explore_parameter_space`` runs DE with ``updating='deferred'`` in the
reference too, so the batched objective (one engine pass per generation)
follows the reference's DE trajectory exactly.  ``optimize_CZ_parameters`` uses
``'immediate'`` updating with ``workers=1`` in the reference; ``vectorized=False``
reproduces that, the default (True) batches each generation.

Persistence: ``ExplorationResult.save/load`` write JSON here (the reference
pickles; pickles are never loaded by this package).
"""
from __future__ import annotations

import json
import time
import warnings
from dataclasses import asdict, dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

import numpy as np
from scipy.optimize import differential_evolution

from .configurations import (JPSimulationInputs, LaserParameters, LPSimulationInputs,
                             NoiseSourceConfig, TwoPhotonExcitationConfig)
from .optimize_cz_gate import COST_KINDS, default_batch_evaluator


@dataclass
class HardwareOptimizationResult:
    success: bool
    target_fidelity: float
    target_gate_time_ns: float
    achieved_fidelity: float
    achieved_gate_time_ns: float
    fidelity_error_pct: float
    gate_time_error_pct: float
    optimal_parameters: Dict[str, float]
    V_over_Omega: float
    noise_breakdown: Dict[str, float]
    n_evaluations: int
    final_cost: float
    message: str

    def __repr__(self):
        return (f"HardwareOptimizationResult(\n"
                f"  Target:   F={self.target_fidelity:.4f}, t={self.target_gate_time_ns:.1f} ns\n"
                f"  Achieved: F={self.achieved_fidelity:.4f}, t={self.achieved_gate_time_ns:.1f} ns\n"
                f"  Errors:   dF={self.fidelity_error_pct:+.2f}%, dt={self.gate_time_error_pct:+.2f}%\n"
                f"  V/Omega={self.V_over_Omega:.1f}, Evals={self.n_evaluations}, Cost={self.final_cost:.2e}\n"
                f"  Success: {self.success}\n)")


@dataclass
class EvaluatedPoint:
    Omega_MHz: float
    laser_linewidth_kHz: float
    V_over_Omega: float
    fidelity: float
    gate_time_ns: float
    infidelity: float
    noise_breakdown: Dict[str, float] = field(default_factory=dict)
    protocol: str = ""
    species: str = "Rb87"


@dataclass
class ExplorationResult:
    protocol: str
    species: str
    points: List[EvaluatedPoint] = field(default_factory=list)
    pareto_front: List[EvaluatedPoint] = field(default_factory=list)
    n_evaluations: int = 0
    runtime_seconds: float = 0.0
    optimizer_settings: Dict[str, Any] = field(default_factory=dict)

    def add_point(self, point: EvaluatedPoint):
        self.points.append(point)
        self.n_evaluations += 1

    def compute_pareto_front(self):
        """Points with better fidelity than every faster point (:174-198); Python's
        stable sort keeps the reference's tie order."""
        if not self.points:
            return
        front, best = [], -1.0
        for p in sorted(self.points, key=lambda q: q.gate_time_ns):
            if p.fidelity > best:
                front.append(p)
                best = p.fidelity
        self.pareto_front = front

    def get_points_above_fidelity(self, min_fidelity: float) -> List[EvaluatedPoint]:
        return [p for p in self.points if p.fidelity >= min_fidelity]

    def get_points_below_time(self, max_time_ns: float) -> List[EvaluatedPoint]:
        return [p for p in self.points if p.gate_time_ns <= max_time_ns]

    def get_best_for_target(self, target_fidelity: float = None,
                            target_time_ns: float = None) -> Optional[EvaluatedPoint]:
        if target_fidelity is not None:
            c = self.get_points_above_fidelity(target_fidelity)
            return min(c, key=lambda p: p.gate_time_ns) if c else None
        if target_time_ns is not None:
            c = self.get_points_below_time(target_time_ns)
            return max(c, key=lambda p: p.fidelity) if c else None
        return None

    def summary(self) -> str:
        if not self.points:
            return "No points evaluated."
        F = [p.fidelity for p in self.points]
        T = [p.gate_time_ns for p in self.points]
        out = ["=" * 60, f"EXPLORATION RESULTS: {self.protocol.upper()}", "=" * 60,
               f"Total evaluations: {self.n_evaluations}",
               f"Runtime: {self.runtime_seconds:.1f}s ({self.runtime_seconds / 60:.1f} min)", "",
               f"Fidelity range: {min(F) * 100:.2f}% - {max(F) * 100:.2f}%",
               f"Gate time range: {min(T):.1f} - {max(T):.1f} ns", "",
               f"Pareto front: {len(self.pareto_front)} points"]
        if self.pareto_front:
            out += ["", "Key Pareto points:"]
            out += [f"  F={p.fidelity * 100:.2f}% @ {p.gate_time_ns:.1f}ns (V/Omega={p.V_over_Omega:.1f})"
                    for p in self.pareto_front[:5]]
            if len(self.pareto_front) > 5:
                out.append(f"  ... and {len(self.pareto_front) - 5} more")
        return "\n".join(out)

    def save(self, filepath: str):
        d = asdict(self)
        with open(filepath, "w") as f:
            json.dump(d, f, default=float)
        print(f"Saved {self.n_evaluations} points to {filepath}")

    @staticmethod
    def load(filepath: str) -> "ExplorationResult":
        with open(filepath) as f:
            d = json.load(f)
        mk = lambda L: [EvaluatedPoint(**p) for p in L]
        return ExplorationResult(protocol=d["protocol"], species=d["species"], points=mk(d["points"]),
                                 pareto_front=mk(d["pareto_front"]), n_evaluations=d["n_evaluations"],
                                 runtime_seconds=d["runtime_seconds"],
                                 optimizer_settings=d.get("optimizer_settings", {}))


def _breakdown(m: Dict[str, Any], j: int) -> Dict[str, float]:
    b = m.get("_batch")
    if b is None:
        return {}
    from .simulation import noise_breakdown_row
    return noise_breakdown_row(b, j)


def _is_lp(protocol: str) -> bool:
    return protocol.lower() in ("levine_pichler", "lp", "two_pulse")


# ---------------------------------------------------------------------------
# inverse problem
# ---------------------------------------------------------------------------

_DEFAULTS = dict(rydberg_power_1=50e-6, rydberg_power_2=500e-3, n_rydberg=70, temperature=5e-6,
                 spacing_factor=3.0, tweezer_power=50e-3, tweezer_waist=1e-6, Delta_e=5e9)


def optimize_CZ_parameters(
        target_fidelity: float = 0.99, target_gate_time_ns: float = 300.0, protocol: str = "levine_pichler",
        weight_fidelity: float = 1.0, weight_time: float = 0.5, constraint_penalty: float = 100.0,
        species: str = "Rb87", background_loss_rate_hz: float = 10.0, include_noise: bool = True,
        include_motional_dephasing: bool = True,
        bounds_rydberg_power_2=(0.5, 50.0), bounds_rydberg_power_1=(0.1e-3, 20e-3),
        bounds_temperature=(0.1e-6, 20e-6), bounds_spacing_factor=(1.8, 6.0), bounds_n_rydberg=(40, 100),
        bounds_tweezer_power=(5e-3, 200e-3), bounds_tweezer_waist=(0.4e-6, 3.0e-6),
        bounds_Delta_e=(0.5e9, 15e9), bounds_laser_linewidth=(100.0, 50e3),
        bounds_delta_over_omega=(0.30, 0.45), bounds_omega_tau_lp=(3.8, 5.0), bounds_omega_tau_jp=(5.5, 8.5),
        optimize_protocol_params: bool = True, couple_powers: bool = False, power_ratio_780_480: float = 0.001,
        maxiter: int = 100, tol: float = 1e-5, seed: Optional[int] = 42, polish: bool = True, workers: int = 1,
        popsize: int = 15, fixed_params: Optional[Dict[str, float]] = None,
        callback: Optional[Callable[[int, float, Dict], None]] = None, verbose: bool = True,
        vectorized: bool = True, evaluator: Optional[Callable] = None,
        cost: str = "reference") -> HardwareOptimizationResult:
    """Find hardware parameters reaching a target fidelity and gate time
    (RG/optimization.py:280-739).  Objective per candidate:
    w_F (1 - F/F_t)^2 + w_t ((t - t_t)/t_t)^2 + c * penalties (V/Omega < 10,
    spacing_factor*tweezer_waist < 2 tweezer_waist, T < 50 nK); failures cost 1e6.
    ``cost="process_fidelity"``: F is the gauge-invariant average gate fidelity to CZ
    (optimize_cz_gate.compute_cost_batch) instead of the reference's avg F."""
    if cost not in COST_KINDS:
        raise ValueError(f"Unknown cost {cost!r}: use one of {COST_KINDS}")
    ev_kw = {"process_fidelity": True} if cost == "process_fidelity" else {}
    fixed_params = dict(fixed_params or {})
    is_lp = _is_lp(protocol)
    is_jp = protocol.lower() in ("jandura_pupillo", "jp", "smooth_jp", "single_pulse", "time_optimal")
    if not is_lp and not is_jp:
        raise ValueError(f"Unknown protocol '{protocol}'. Use 'levine_pichler' (or 'lp') "
                         f"or 'jandura_pupillo' / 'smooth_jp' (or 'jp').")
    cfg = {"total_power": bounds_rydberg_power_2} if couple_powers else {
        "rydberg_power_2": bounds_rydberg_power_2, "rydberg_power_1": bounds_rydberg_power_1}
    cfg.update(temperature=bounds_temperature, spacing_factor=bounds_spacing_factor, n_rydberg=bounds_n_rydberg,
               tweezer_power=bounds_tweezer_power, tweezer_waist=bounds_tweezer_waist,
               laser_linewidth=bounds_laser_linewidth, Delta_e=bounds_Delta_e)
    if optimize_protocol_params:
        if is_lp:
            cfg.update(delta_over_omega=bounds_delta_over_omega, omega_tau=bounds_omega_tau_lp)
        else:
            cfg["omega_tau"] = bounds_omega_tau_jp
    names = [k for k in cfg if k not in fixed_params]
    bounds = [cfg[k] for k in names]
    evaluator = evaluator or default_batch_evaluator
    builds_lp = protocol in ("levine_pichler", "lp")       # the reference's inputs switch (:517)
    state = dict(n=0, best=np.inf, best_params=None)

    def columns(X: np.ndarray) -> Dict[str, np.ndarray]:
        S = X.shape[0]
        P = {k: X[:, i] for i, k in enumerate(names)}
        P.update({k: np.full(S, float(v)) for k, v in fixed_params.items()})
        if couple_powers and "total_power" in P:
            P["rydberg_power_2"] = P.pop("total_power")
            P["rydberg_power_1"] = P["rydberg_power_2"] * power_ratio_780_480
        if "n_rydberg" in P:
            P["n_rydberg"] = np.round(P["n_rydberg"]).astype(int).astype(float)
        return P

    def objective(X: np.ndarray) -> np.ndarray:
        X = np.atleast_2d(X)
        S = X.shape[0]
        P = columns(X)
        g = lambda k: P.get(k, np.full(S, _DEFAULTS.get(k, np.nan)))
        lw = P.get("laser_linewidth", np.full(S, 1000.0))
        over = dict(laser_1_power=g("rydberg_power_1"), laser_2_power=g("rydberg_power_2"),
                    laser_1_linewidth_hz=lw, laser_2_linewidth_hz=lw, Delta_e=2 * np.pi * g("Delta_e"))
        if "omega_tau" in P:
            over["omega_tau"] = P["omega_tau"]
        if builds_lp and "delta_over_omega" in P:
            over["delta_over_omega"] = P["delta_over_omega"]
        exc = TwoPhotonExcitationConfig(laser_1=LaserParameters(power=50e-6, waist=50e-6),
                                        laser_2=LaserParameters(power=500e-3, waist=50e-6))
        noise = NoiseSourceConfig(include_motional_dephasing=include_motional_dephasing)
        si = (LPSimulationInputs(excitation=exc, noise=noise) if builds_lp
              else JPSimulationInputs(excitation=exc, noise=noise))
        app = dict(species=species, n_rydberg=g("n_rydberg"), temperature=g("temperature"),
                   spacing_factor=g("spacing_factor"), tweezer_power=g("tweezer_power"),
                   tweezer_waist=g("tweezer_waist"), background_loss_rate_hz=background_loss_rate_hz)
        from .optimize_cz_gate import _evaluate_rows
        m, ok = _evaluate_rows(evaluator, si, over, S, include_noise, app, **ev_kw)
        F = m["avg_gate_fidelity"] if cost == "process_fidelity" else m["avg_fidelity"]
        t_ns, vo = m["gate_time_us"] * 1e3, m["V_over_Omega"]
        sf, w, T = g("spacing_factor"), g("tweezer_waist"), g("temperature")
        pen = (np.where(vo < 10, (10 - vo) ** 2, 0.0)
               + np.where(sf * w < 2 * w, ((2 * w - sf * w) / w) ** 2, 0.0)
               + np.where(T < 0.05e-6, ((0.05e-6 - T) / 1e-6) ** 2, 0.0))
        obj = (weight_fidelity * (1 - F / target_fidelity) ** 2
                + weight_time * ((t_ns - target_gate_time_ns) / target_gate_time_ns) ** 2
                + constraint_penalty * pen)
        obj = np.where(ok & np.isfinite(obj), obj, 1e6)
        for j in range(S):                     # sequential bookkeeping, as the scalar objective
            state["n"] += 1
            if not ok[j]:
                continue
            params = {k: float(v[j]) for k, v in P.items() if k != "laser_linewidth"}
            if "n_rydberg" in params:
                params["n_rydberg"] = int(params["n_rydberg"])
            if obj[j] < state["best"]:
                state["best"] = float(obj[j])
                bp = dict(params)
                bp.update(laser_linewidth=float(lw[j]), _fidelity=float(F[j]), _gate_time_ns=float(t_ns[j]),
                          _V_over_Omega=float(vo[j]), _noise=_breakdown(m, j))
                state["best_params"] = bp
            if callback is not None:
                callback(state["n"], float(obj[j]), params)
            if verbose and state["n"] % 20 == 0:
                print(f"  [Eval {state['n']:4d}] F={F[j]:.4f}, t={t_ns[j]:.1f}ns, V/Omega={vo[j]:.1f}, "
                      f"cost={obj[j]:.2e}")
        return obj

    if verbose:
        print(f"CZ hardware optimisation: {protocol}, target F={target_fidelity:.4f}, "
              f"t={target_gate_time_ns:.1f} ns, {len(names)} parameters, "
              f"{'batched' if vectorized else 'per-point'} objective")
    vec = vectorized and workers == 1
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        if vec:
            res = differential_evolution(lambda x: objective(np.asarray(x).T), bounds=bounds, maxiter=maxiter,
                                         tol=tol, seed=seed, polish=polish, popsize=popsize, disp=False,
                                         vectorized=True, updating="deferred")
        else:
            res = differential_evolution(lambda x: float(objective(np.asarray(x)[None, :])[0]), bounds=bounds,
                                         maxiter=maxiter, tol=tol, seed=seed, polish=polish, popsize=popsize,
                                         disp=False, updating="deferred" if workers > 1 else "immediate")
    bp = state["best_params"]
    if bp is None:                                      # nothing succeeded: report the DE point
        objective(np.asarray(res.x)[None, :])
        bp = state["best_params"] or {"_fidelity": 0.0, "_gate_time_ns": np.inf, "_V_over_Omega": 0.0,
                                      "_noise": {}}
    final = {k: v for k, v in bp.items() if not k.startswith("_")}
    F, t_ns, vo = bp["_fidelity"], bp["_gate_time_ns"], bp["_V_over_Omega"]
    dF = (F / target_fidelity - 1) * 100
    dt = (t_ns / target_gate_time_ns - 1) * 100
    tolF = 2.0 if target_fidelity > 0.995 else 5.0
    success = abs(dF) < tolF and abs(dt) < 30.0 and vo >= 8
    if success:
        msg = "Optimization converged successfully"
    else:
        issues = []
        if abs(dF) >= tolF:
            issues.append(f"fidelity error {dF:+.1f}%")
        if abs(dt) >= 30.0:
            issues.append(f"time error {dt:+.1f}%")
        if vo < 8:
            issues.append(f"V/Ω={vo:.1f} < 8")
        msg = f"Optimization incomplete: {', '.join(issues)}"
    if verbose:
        print(f"  Achieved: F={F:.4f}, t={t_ns:.1f} ns (dF={dF:+.2f}%, dt={dt:+.2f}%), V/Omega={vo:.1f}; {msg}")
    return HardwareOptimizationResult(success=success, target_fidelity=target_fidelity,
                                      target_gate_time_ns=target_gate_time_ns, achieved_fidelity=F,
                                      achieved_gate_time_ns=t_ns, fidelity_error_pct=dF, gate_time_error_pct=dt,
                                      optimal_parameters=final, V_over_Omega=vo, noise_breakdown=bp["_noise"],
                                      n_evaluations=state["n"], final_cost=state["best"], message=msg)


# ---------------------------------------------------------------------------
# Pareto exploration
# ---------------------------------------------------------------------------

def explore_parameter_space(
        protocol: str = "levine_pichler", species: str = "Rb87", n_runs: int = 1, maxiter: int = 30,
        popsize: int = 10, seeds: List[int] = None, verbose: bool = True,
        bounds_rydberg_power_2=(0.5, 30.0), bounds_rydberg_power_1=(0.5e-3, 10e-3),
        bounds_temperature=(1e-6, 15e-6), bounds_spacing_factor=(2.0, 5.0), bounds_n_rydberg=(50, 90),
        bounds_tweezer_power=(10e-3, 100e-3), bounds_tweezer_waist=(0.5e-6, 2.0e-6),
        bounds_laser_linewidth=(100.0, 10e3), bounds_delta_over_omega=(0.32, 0.42),
        bounds_omega_tau=(3.9, 4.8), evaluator: Optional[Callable] = None,
        cost: str = "reference") -> ExplorationResult:
    """Every DE evaluation recorded, Pareto front post hoc (RG/optimization.py:746-980).
    One engine pass per DE generation (the reference's DE already uses deferred
    updating, so the candidate sequence is the reference's).  ``cost="process_fidelity"``
    records and minimises the gauge-invariant average gate fidelity instead of the
    reference's avg F; ``optimizer_settings["gauge_flagged"]`` counts the evaluated points
    whose reference penalty was gauge-flagged."""
    if cost not in COST_KINDS:
        raise ValueError(f"Unknown cost {cost!r}: use one of {COST_KINDS}")
    ev_kw = {"process_fidelity": True} if cost == "process_fidelity" else {}
    seeds = seeds if seeds is not None else [42 + 111 * i for i in range(n_runs)]
    result = ExplorationResult(protocol=protocol, species=species,
                               optimizer_settings=dict(n_runs=n_runs, maxiter=maxiter, popsize=popsize,
                                                       seeds=seeds, cost=cost, gauge_flagged=0))
    t0 = time.time()
    is_lp = _is_lp(protocol)
    names = ["rydberg_power_2", "rydberg_power_1", "temperature", "spacing_factor", "n_rydberg",
             "tweezer_power", "tweezer_waist", "laser_linewidth"]
    bounds = [bounds_rydberg_power_2, bounds_rydberg_power_1, bounds_temperature, bounds_spacing_factor,
              bounds_n_rydberg, bounds_tweezer_power, bounds_tweezer_waist, bounds_laser_linewidth]
    if is_lp:
        names += ["delta_over_omega", "omega_tau"]
        bounds += [bounds_delta_over_omega, bounds_omega_tau]
    evaluator = evaluator or default_batch_evaluator
    best = dict(F=0.0, t=np.inf)
    from .optimize_cz_gate import _evaluate_rows

    def objective(X: np.ndarray) -> np.ndarray:
        X = np.atleast_2d(X)
        S = X.shape[0]
        P = {k: X[:, i] for i, k in enumerate(names)}
        lw = P["laser_linewidth"]
        exc = TwoPhotonExcitationConfig(laser_1=LaserParameters(power=1e-3, waist=1.0e-6),
                                        laser_2=LaserParameters(power=1e-3, waist=10e-6))
        noise = NoiseSourceConfig(include_motional_dephasing=True, include_doppler_dephasing=True,
                                  include_intensity_noise=True, intensity_noise_frac=0.01)
        over = dict(laser_1_power=P["rydberg_power_1"], laser_2_power=P["rydberg_power_2"],
                    laser_1_linewidth_hz=lw, laser_2_linewidth_hz=lw)
        if is_lp:
            over.update(delta_over_omega=P["delta_over_omega"], omega_tau=P["omega_tau"])
            si = LPSimulationInputs(excitation=exc, noise=noise)
        else:
            si = JPSimulationInputs(excitation=exc, noise=noise)
        app = dict(species=species, n_rydberg=np.round(P["n_rydberg"]), temperature=P["temperature"],
                   spacing_factor=P["spacing_factor"], tweezer_power=P["tweezer_power"],
                   tweezer_waist=P["tweezer_waist"])
        m, ok = _evaluate_rows(evaluator, si, over, S, True, app, **ev_kw)
        F = m["avg_gate_fidelity"] if cost == "process_fidelity" else m["avg_fidelity"]
        t_ns = m["gate_time_us"] * 1e3
        if "gauge_unstable" in m:
            result.optimizer_settings["gauge_flagged"] += int((np.asarray(m["gauge_unstable"])[ok] > 0).sum())
        out = np.where(ok, (1 - F) + 0.001 * (t_ns / 1000), 1.0)
        for j in range(S):
            if not ok[j]:
                continue
            result.add_point(EvaluatedPoint(
                Omega_MHz=float(m["Omega_MHz"][j]), laser_linewidth_kHz=float(lw[j]) / 1e3,
                V_over_Omega=float(m["V_over_Omega"][j]), fidelity=float(F[j]), gate_time_ns=float(t_ns[j]),
                infidelity=float(1 - F[j]), noise_breakdown=_breakdown(m, j), protocol=protocol, species=species))
            best["F"] = max(best["F"], float(F[j]))
            if F[j] > 0.95:
                best["t"] = min(best["t"], float(t_ns[j]))
            if verbose and result.n_evaluations % 25 == 0:
                print(f"  [{result.n_evaluations:4d}] best F={best['F'] * 100:.2f}%, "
                      f"fastest (F>95%)={best['t']:.0f}ns")
        return out

    for k, seed in enumerate(seeds):
        if verbose:
            print(f"\nRun {k + 1}/{n_runs} (seed={seed}) -- batched DE")
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            differential_evolution(lambda x: objective(np.asarray(x).T), bounds=bounds, maxiter=maxiter,
                                   popsize=popsize, seed=seed, disp=False, vectorized=True,
                                   updating="deferred", mutation=(0.5, 1.0), recombination=0.7)
    result.compute_pareto_front()
    result.runtime_seconds = time.time() - t0
    if verbose:
        print("\n" + result.summary())
    return result


def combine_explorations(*results: ExplorationResult) -> ExplorationResult:
    if not results:
        raise ValueError("No results to combine")
    out = ExplorationResult(protocol=results[0].protocol, species=results[0].species)
    for r in results:
        out.points.extend(r.points)
        out.runtime_seconds += r.runtime_seconds
    out.n_evaluations = len(out.points)
    out.compute_pareto_front()
    return out


__all__ = ["HardwareOptimizationResult", "optimize_CZ_parameters", "EvaluatedPoint", "ExplorationResult",
           "explore_parameter_space", "combine_explorations"]
