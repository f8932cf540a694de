"""MI355X-native batched Lindblad engine for the two-atom Rydberg CZ gate.

Drop-in for the public API of the reference package
``qpu_simulator.micro_physics.neutral_atoms.rydberg_gates`` (its ``__all__``,
RG/__init__.py:243-321) on the path this build replaces: ``simulate_CZ_gate`` and
its inputs and result record, the fidelity functions, the optimiser entry points,
the protocol tables, the sweep driver of examples/research_parameter_sweeps.py
and the physical constants.  Importing needs no GPU; the first engine call
loads the in-tree HIP library (``libryd_engine.so``) and raises if it or a GPU
is missing -- there is no CPU fallback.
"""
from .constants import A0, C, E_CHARGE, EPS0, HBAR, KB, MU_B, RY_JOULES
from .configurations import (AtomicConfiguration, JPSimulationInputs, LaserParameters,
                             LPSimulationInputs, NoiseSourceConfig, SmoothJPSimulationInputs,
                             TwoPhotonExcitationConfig)
from .protocols import (JP_BANGBANG_OMEGA_TAU, JP_BANGBANG_PHASES, JP_BANGBANG_SWITCHING_TIMES,
                        LP_DELTA_OVER_OMEGA_DEFAULT, LP_OMEGA_TAU_DEFAULT, LP_XI_DEFAULT,
                        SMOOTH_JP_DEFAULTS as SMOOTH_JP_PARAMS, compute_phase_shift_xi)
from .simulation import (BatchResult, SimulationResult, compute_CZ_fidelity, compute_state_fidelity,
                         evolve_state, evolve_state_batch, mixed_phase_penalty, simulate_CZ_gate,
                         simulate_CZ_gate_batch)
from .optimize_cz_gate import (JP_PHASES_DEFAULT, JP_SWITCHING_TIMES_DEFAULT, ApparatusConstraints,
                               OptimizationResult, SimulationCache, compute_cost, extract_metrics,
                               optimize_cz_gate, run_baseline)
from .optimization import (EvaluatedPoint, ExplorationResult, HardwareOptimizationResult,
                           combine_explorations, explore_parameter_space, optimize_CZ_parameters)
from .engine import Engine, DeviceBatch
from .noise_models import gate_process_maps
from .calibration import calibrate_cz, load_calibration, write_calibration

__all__ = [
    # simulate / analyse (RG/simulation.py)
    "simulate_CZ_gate", "simulate_CZ_gate_batch", "SimulationResult", "BatchResult",
    "compute_CZ_fidelity", "compute_state_fidelity", "mixed_phase_penalty", "evolve_state", "evolve_state_batch",
    # inputs (RG/configurations.py)
    "TwoPhotonExcitationConfig", "NoiseSourceConfig", "LPSimulationInputs", "JPSimulationInputs",
    "SmoothJPSimulationInputs", "LaserParameters", "AtomicConfiguration",
    # protocol parameters (RG/protocols.py)
    "LP_OMEGA_TAU_DEFAULT", "LP_DELTA_OVER_OMEGA_DEFAULT", "LP_XI_DEFAULT", "SMOOTH_JP_PARAMS",
    "JP_SWITCHING_TIMES_DEFAULT", "JP_PHASES_DEFAULT", "JP_BANGBANG_OMEGA_TAU",
    "JP_BANGBANG_SWITCHING_TIMES", "JP_BANGBANG_PHASES", "compute_phase_shift_xi",
    # optimisation (RG/optimize_cz_gate.py, RG/optimization.py)
    "ApparatusConstraints", "optimize_cz_gate", "run_baseline", "compute_cost", "extract_metrics",
    "SimulationCache", "OptimizationResult", "HardwareOptimizationResult", "optimize_CZ_parameters",
    "EvaluatedPoint", "ExplorationResult", "explore_parameter_space", "combine_explorations",
    # constants (RG/constants.py)
    "HBAR", "EPS0", "C", "E_CHARGE", "A0", "KB", "MU_B", "RY_JOULES",
    # engine, process maps, calibration files (beyond the reference)
    "Engine", "DeviceBatch", "gate_process_maps", "calibrate_cz", "write_calibration", "load_calibration",
]
