#!/bin/bash
# C5 A/B: the default build against the variants named in $1 (build/libryd_<v>.so)
set -o pipefail
O=gpurun_out/${2:-c5ab}
mkdir -p $O
export PYTHONPATH=$PWD
B="bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline"
timeout -k 10 200 python $B > $O/bench_default.json 2> $O/bench_default.err || exit 1
for v in $1; do
  RYD_ENGINE_LIB=$PWD/build/libryd_$v.so timeout -k 10 200 python $B > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
done
for f in $O/bench_*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', d['value'], r['kernel_ms'], r['exec_over_useful'])"; done
