"""Turn a golden-fixture config dict into this package's inputs (shared by tests)."""
import numpy as np

from noisyquantumsimulator_amd import configurations as CF
from noisyquantumsimulator_amd import physics as PH


def simulation_inputs(cfg):
    L1 = CF.LaserParameters(power=cfg["l1p"], waist=cfg["l1w"], polarization="pi",
                            polarization_purity=cfg.get("purity", 1.0),
                            linewidth_hz=cfg.get("lw1", 100.0))
    L2 = CF.LaserParameters(power=cfg["l2p"], waist=cfg["l2w"], polarization="sigma+",
                            polarization_purity=cfg.get("purity", 1.0),
                            linewidth_hz=cfg.get("lw2", 100.0))
    exc = CF.TwoPhotonExcitationConfig(laser_1=L1, laser_2=L2,
                                       Delta_e=cfg.get("Delta_e", 2 * np.pi * 1e9),
                                       counter_propagating=cfg.get("counter", True))
    noise = CF.NoiseSourceConfig(**cfg.get("noise_cfg", {}))
    p = cfg["protocol"]
    if p == "levine_pichler":
        return CF.LPSimulationInputs(excitation=exc, noise=noise,
                                     delta_over_omega=cfg.get("delta_over_omega"),
                                     omega_tau=cfg.get("omega_tau"),
                                     pulse_shape=cfg.get("pulse_shape", "square"))
    if p == "smooth_jp":
        return CF.SmoothJPSimulationInputs(excitation=exc, noise=noise, omega_tau=cfg.get("omega_tau"),
                                           A=cfg.get("A"), omega_mod_ratio=cfg.get("omega_mod_ratio"),
                                           phi_offset=cfg.get("phi_offset"),
                                           delta_over_omega=cfg.get("delta_over_omega"))
    return CF.JPSimulationInputs(excitation=exc, noise=noise, omega_tau=cfg.get("omega_tau"),
                                 switching_times=cfg.get("switching_times"), phases=cfg.get("phases"))


def simulate_kwargs(cfg):
    return dict(species=cfg.get("species", "Rb87"), n_rydberg=cfg["n"],
                qubit_0=tuple(cfg.get("qubit_0", (1, 0))), qubit_1=tuple(cfg.get("qubit_1", (2, 0))),
                hilbert_space_dim=cfg.get("dim", 3), tweezer_power=cfg["Ptw"],
                tweezer_waist=cfg["wtw"], tweezer_wavelength_nm=cfg.get("wl_nm"),
                temperature=cfg["T"], B_field=cfg.get("B", 1e-4), NA=cfg.get("NA", 0.5),
                spacing_factor=cfg["sf"], include_noise=cfg.get("include_noise", True),
                background_loss_rate_hz=cfg.get("bg"), trap_laser_on=cfg.get("trap_on", True))


def derive(cfg):
    return PH.derive_batch(simulation_inputs(cfg), **simulate_kwargs(cfg))
