#!/bin/bash
# Round 3: the exact-jump-time C5 kernel (traj3e_kernel, ladder_levels = 0) -- parity tests,
# then C5 bench exact vs ladder 16, then the rocprof kernel stats of the exact run.
set -o pipefail
mkdir -p gpurun_out/c5eig
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_trajectories.py -k "exact_jump_times or zero_rates or multi_segment" \
  > gpurun_out/c5eig/pytest.log 2>&1 || { tail -40 gpurun_out/c5eig/pytest.log; exit 1; }
tail -3 gpurun_out/c5eig/pytest.log
timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 2 --ladder 0 --no-cpu-baseline \
  > gpurun_out/c5eig/bench_exact.json 2> gpurun_out/c5eig/bench_exact.err || { tail -20 gpurun_out/c5eig/bench_exact.err; exit 1; }
timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/c5eig/bench_l16.json 2> gpurun_out/c5eig/bench_l16.err || { tail -20 gpurun_out/c5eig/bench_l16.err; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/c5eig/prof -o run -- \
  python3 bench.py --workload c5 --steps 5 --warmup 2 --ladder 0 --no-cpu-baseline > gpurun_out/c5eig/bench_exact_prof.json 2>&1
python3 - <<'PY'
import json
for f in ("bench_exact", "bench_l16"):
    d = json.load(open(f"gpurun_out/c5eig/{f}.json"))
    print(f, d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"].get("kernel"))
PY
