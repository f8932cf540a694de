#!/bin/bash
# exact-time C5 kernel, several points per wave: trajectory tests (both modes), bench, phases
set -o pipefail
O=gpurun_out/c5eig3
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_trajectories.py \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python bench.py --workload c5 --steps 10 --warmup 2 --ladder 0 --no-cpu-baseline > $O/bench_exact.json 2> $O/bench_exact.err || exit 1
RYD_ENGINE_LIB=$PWD/build/libryd_tprof.so timeout -k 10 200 python -u tools/traj_prof.py 0 > $O/phase.log 2>&1 || exit 1
cat $O/phase.log
python3 -c "
import json
d = json.load(open('$O/bench_exact.json')); r = d['roofline']
print('exact', d['value'], r['kernel_ms'], r['frac'], r['exec_over_useful'])"
