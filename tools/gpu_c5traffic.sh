# C5: trajectory tests, the C5 line for the default build and A/B variants in build/, and
# the FETCH/WRITE PMC passes of the default build (spill traffic).
# Usage: gpurun --timeout 900 -- bash tools/gpu_c5traffic.sh TAG "variant ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$PWD
TAG=${1:-c5t}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_trajectories.py -x -v --timeout 200 --timeout-method thread > $O/pytest_traj.log 2>&1; rc=$?
tail -2 $O/pytest_traj.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
for v in $2; do
  RYD_ENGINE_LIB=$PWD/build/libryd_$v.so timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5_$v.json 2> $O/bench_c5_$v.err || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c5 -o run -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/fetch_c5.log 2>&1 || { echo "fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c5 -o run -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/write_c5.log 2>&1 || { echo "write failed"; exit 1; }
for f in $O/bench_c5*.json; do python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', d['value'], r['kernel_ms'], r['frac'])"; done
