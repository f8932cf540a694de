# C5: trajectory tests on the default build, then the C5 bench line for it and for the
# A/B variants in build/ (libryd_<name>.so)
# Usage: gpurun --timeout 900 -- bash tools/gpu_c5ab.sh TAG "name ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD
TAG=${1:-c5ab}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_trajectories.py -x -v --timeout 200 --timeout-method thread > $O/pytest_traj.log 2>&1; rc=$?
tail -3 $O/pytest_traj.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
for v in $2; do
  RYD_ENGINE_LIB=$PWD/build/libryd_$v.so timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5_$v.json 2> $O/bench_c5_$v.err || exit 1
done
for f in $O/bench_c5*.json; do python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', d['value'], r['kernel_ms'], r['frac'], r.get('exec_over_useful'), r.get('mean_jumps'))"; done
