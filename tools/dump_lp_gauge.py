"""Dump the 11-point LP-square states of test_stable_penalty_matches_oracle_through_engine
and their gauge flags for the library named by RYD_ENGINE_LIB (A/B of kernel variants).
    RYD_ENGINE_LIB=... python tools/dump_lp_gauge.py OUT.npz"""
import sys
import warnings

import numpy as np

from noisyquantumsimulator_amd import _native as N
from noisyquantumsimulator_amd import engine as E
from noisyquantumsimulator_amd import sweeps as SW
from noisyquantumsimulator_amd.protocols import compute_phase_shift_xi

warnings.simplefilter("ignore")
P = N.P
batch = SW.pareto_tgate_grid(omega_slice=slice(0, 1000, 111))
p = SW.c3_four_op_params(batch)[:, ::97].copy()
p[P["TAU"]] = 4.29268 / p[P["OMEGA"]]
p[P["DELTA"]] = 0.377371 * p[P["OMEGA"]]
xi = np.asarray(compute_phase_shift_xi(p[P["DELTA"]], p[P["OMEGA"]], p[P["TAU"]]))
p[P["XI_RE"]], p[P["XI_IM"]] = xi.real, xi.imag
p = np.ascontiguousarray(p)
eng = E.Engine()
r = eng.run(p, "lp_square", "lindblad")
ph, flags = E.mixed_phase(r.state, r.n, 3, copies=64)
print("flags", (flags & N.STATUS_GAUGE_UNSTABLE) != 0)
np.savez(sys.argv[1], state=r.state, flags=flags, ph=ph)
