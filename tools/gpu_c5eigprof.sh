#!/bin/bash
# exact-time C5 kernel: phase profile (2 waves and 1 wave per SIMD) and the 1-wave bench
set -o pipefail
O=gpurun_out/c5eigprof
mkdir -p $O
export PYTHONPATH=$PWD
RYD_ENGINE_LIB=$PWD/build/libryd_tprof.so timeout -k 10 200 python -u tools/traj_prof.py 0 > $O/phase_w2.log 2>&1 || exit 1
RYD_ENGINE_LIB=$PWD/build/libryd_eigw1p.so timeout -k 10 200 python -u tools/traj_prof.py 0 > $O/phase_w1.log 2>&1 || exit 1
RYD_ENGINE_LIB=$PWD/build/libryd_tprof.so timeout -k 10 200 python -u tools/traj_prof.py 16 > $O/phase_l16.log 2>&1 || exit 1
RYD_ENGINE_LIB=$PWD/build/libryd_eigw1.so timeout -k 10 200 python -u bench.py --workload c5 --steps 5 --warmup 2 --ladder 0 --no-cpu-baseline > $O/bench_w1.json 2> $O/bench_w1.err || exit 1
cat $O/phase_w2.log $O/phase_w1.log $O/phase_l16.log
python3 -c "import json; d=json.load(open('$O/bench_w1.json')); print('w1', d['value'], d['roofline']['kernel_ms'])"
