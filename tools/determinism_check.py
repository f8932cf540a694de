"""Run-to-run determinism of the resident-batch launches: the same C2 / C3
batch launched repeatedly must give bit-identical states, summaries and status (guards
the LDS ordering assumptions of the sym16 kernel: zero words, weight table, transposes).
    python tools/determinism_check.py [repeats]"""
import hashlib
import sys
import warnings

import numpy as np

from noisyquantumsimulator_amd import engine as E
from noisyquantumsimulator_amd import sweeps as SW

warnings.simplefilter("ignore")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
eng = E.Engine()
cases = [("c2", E.pack_params(SW.omega_delta_grid(100, 100)), "lp_square", None),
         ("c3", SW.c3_four_op_params(SW.pareto_tgate_grid(n_omega=100, n_tau=40)), "smooth_jp", 300)]
for name, p, proto, ns in cases:
    db = E.DeviceBatch(eng, p, proto, "lindblad", n_steps=ns)
    digests = set()
    for _ in range(reps):
        db.launch()
        r = db.fetch()
        h = hashlib.sha256()
        for a in (r.state, r.summary, r.status):
            h.update(np.ascontiguousarray(a).tobytes())
        digests.add(h.hexdigest())
    print(name, "points", p.shape[1], "repeats", reps, "distinct results", len(digests))
    assert len(digests) == 1, name
print("deterministic")
