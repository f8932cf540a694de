"""Input dataclasses of the simulate_CZ_gate contract.

Same field names, defaults and meaning as the reference (RG/configurations.py:
LaserParameters :77, TwoPhotonExcitationConfig :178, NoiseSourceConfig :219,
LPSimulationInputs :263, JPSimulationInputs :317, SmoothJPSimulationInputs :379,
AtomicConfiguration :640), so callers can switch imports unchanged.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

from . import species as _sp
from .constants import C, EPS0


@dataclass
class LaserParameters:
    power: float = 1e-3
    waist: float = 50e-6
    polarization: str = "sigma+"
    polarization_purity: float = 0.99
    linewidth_hz: float = 100.0

    def peak_intensity(self) -> float:
        return 2 * self.power / (np.pi * self.waist ** 2)

    def peak_electric_field(self) -> float:
        return float(np.sqrt(2 * self.peak_intensity() / (EPS0 * C)))


@dataclass
class TwoPhotonExcitationConfig:
    laser_1: LaserParameters = field(default_factory=lambda: LaserParameters(
        power=50e-6, waist=50e-6, polarization="pi", linewidth_hz=1000))
    laser_2: LaserParameters = field(default_factory=lambda: LaserParameters(
        power=500e-3, waist=50e-6, polarization="sigma+", linewidth_hz=1000))
    Delta_e: float = 2 * np.pi * 1e9
    counter_propagating: bool = True


@dataclass
class NoiseSourceConfig:
    # The four flags marked (*) are read but have no effect in the reference
    # either (RG/simulation.py:2804-2811); their noise is always on when
    # include_noise=True.
    include_spontaneous_emission: bool = True      # (*)
    include_intermediate_scattering: bool = True   # (*)
    include_motional_dephasing: bool = True
    include_doppler_dephasing: bool = True
    include_intensity_noise: bool = True
    intensity_noise_frac: float = 0.01
    include_laser_dephasing: bool = True           # (*)
    include_magnetic_dephasing: bool = True        # (*)


@dataclass
class LPSimulationInputs:
    excitation: TwoPhotonExcitationConfig = field(default_factory=TwoPhotonExcitationConfig)
    noise: NoiseSourceConfig = field(default_factory=NoiseSourceConfig)
    delta_over_omega: Optional[float] = None
    omega_tau: Optional[float] = None
    pulse_shape: str = "square"
    drag_lambda: float = 1.0

    @property
    def protocol_name(self) -> str:
        return "levine_pichler"

    @property
    def n_pulses(self) -> int:
        return 2


@dataclass
class JPSimulationInputs:
    excitation: TwoPhotonExcitationConfig = field(default_factory=TwoPhotonExcitationConfig)
    noise: NoiseSourceConfig = field(default_factory=NoiseSourceConfig)
    omega_tau: Optional[float] = None
    switching_times: Optional[List[float]] = None
    phases: Optional[List[float]] = None

    @property
    def protocol_name(self) -> str:
        return "jandura_pupillo"

    @property
    def pulse_shape(self) -> str:
        return "bangbang"

    @property
    def n_pulses(self) -> int:
        return 1


@dataclass
class SmoothJPSimulationInputs:
    excitation: TwoPhotonExcitationConfig = field(default_factory=TwoPhotonExcitationConfig)
    noise: NoiseSourceConfig = field(default_factory=NoiseSourceConfig)
    omega_tau: Optional[float] = None
    A: Optional[float] = None
    omega_mod_ratio: Optional[float] = None
    phi_offset: Optional[float] = None
    delta_over_omega: Optional[float] = None

    @property
    def protocol_name(self) -> str:
        return "smooth_jp"

    @property
    def pulse_shape(self) -> str:
        return "smooth_sinusoidal"

    @property
    def n_pulses(self) -> int:
        return 1


@dataclass
class AtomicConfiguration:
    species: str = "Rb87"
    n_rydberg: int = 70
    L_rydberg: str = "S"
    qubit_0: Tuple[int, int] = (1, 0)
    qubit_1: Tuple[int, int] = (2, 0)
    intermediate_state: Optional[str] = None

    def __post_init__(self):
        sp = _sp.get(self.species)
        if self.intermediate_state is None:
            self.intermediate_state = sp.intermediate

    @property
    def is_clock_transition(self) -> bool:
        return self.qubit_0[1] == 0 and self.qubit_1[1] == 0

    @property
    def C6(self) -> float:
        return float(_sp.C6(_sp.get(self.species), self.n_rydberg))

    @property
    def rydberg_lifetime_300K(self) -> float:
        return float(_sp.rydberg_lifetime(_sp.get(self.species), self.n_rydberg, 300.0))

    @property
    def excitation_wavelength_1_nm(self) -> float:
        return float(_sp.excitation_wavelengths_nm(_sp.get(self.species), self.n_rydberg)[0])

    @property
    def excitation_wavelength_2_nm(self) -> float:
        return float(_sp.excitation_wavelengths_nm(_sp.get(self.species), self.n_rydberg)[1])
