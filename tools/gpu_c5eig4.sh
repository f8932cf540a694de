#!/bin/bash
# exact-time C5 kernel: trajectory tests, bench at 4 (default), 2 and 8 points per wave, phases
set -o pipefail
O=gpurun_out/c5eig4
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_trajectories.py \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="bench.py --workload c5 --steps 10 --warmup 2 --ladder 0 --no-cpu-baseline"
timeout -k 10 200 python $B > $O/bench_p4.json 2> $O/bench_p4.err || exit 1
RYD_ENGINE_LIB=$PWD/build/libryd_eigp2.so timeout -k 10 200 python $B > $O/bench_p2.json 2> $O/bench_p2.err || exit 1
RYD_ENGINE_LIB=$PWD/build/libryd_eigp8.so timeout -k 10 200 python $B > $O/bench_p8.json 2> $O/bench_p8.err || exit 1
RYD_ENGINE_LIB=$PWD/build/libryd_tprof.so timeout -k 10 200 python -u tools/traj_prof.py 0 > $O/phase.log 2>&1 || exit 1
cat $O/phase.log
python3 -c "
import json
for f in ('p4', 'p2', 'p8'):
    d = json.load(open('$O/bench_' + f + '.json')); r = d['roofline']
    print(f, d['value'], r['kernel_ms'], r['frac'], r['exec_over_useful'])"
