import warnings, numpy as np
from noisyquantumsimulator_amd import engine as E, sweeps as SW
warnings.simplefilter("ignore")
p = SW.c3_four_op_params(SW.pareto_tgate_grid(n_omega=100, n_tau=100))[:, :8].copy()
r = E.Engine().run(p, "smooth_jp", "lindblad", n_steps=300)
print("status", r.status)
