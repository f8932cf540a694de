#!/bin/bash
# exact-time C5 kernel: parity tests, bench (2 and 1 waves/SIMD), phase profiles
set -o pipefail
O=gpurun_out/c5eig2
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_trajectories.py -k "exact_jump_times or zero_rates or multi_segment" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 2 --ladder 0 --no-cpu-baseline > $O/bench_exact.json 2> $O/bench_exact.err || exit 1
RYD_ENGINE_LIB=$PWD/build/libryd_eigw1.so timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 2 --ladder 0 --no-cpu-baseline > $O/bench_exact_w1.json 2> $O/bench_exact_w1.err || exit 1
RYD_ENGINE_LIB=$PWD/build/libryd_tprof.so timeout -k 10 200 python -u tools/traj_prof.py 0 > $O/phase_w2.log 2>&1 || exit 1
RYD_ENGINE_LIB=$PWD/build/libryd_eigw1p.so timeout -k 10 200 python -u tools/traj_prof.py 0 > $O/phase_w1.log 2>&1 || exit 1
cat $O/phase_w2.log $O/phase_w1.log
python3 -c "
import json
for f in ('bench_exact', 'bench_exact_w1'):
    d = json.load(open('$O/' + f + '.json')); r = d['roofline']
    print(f, d['value'], r['kernel_ms'], r['frac'], r['exec_over_useful'])"
