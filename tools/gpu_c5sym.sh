# C5 adapted-basis kernel: trajectory tests, phase profile, bench (default and variants)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD
TAG=${1:-c5sym}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_trajectories.py -x -v --timeout 300 --timeout-method thread > $O/pytest_traj.log 2>&1; rc=$?
tail -3 $O/pytest_traj.log
[ $rc -eq 0 ] || exit $rc
RYD_ENGINE_LIB=$PWD/build/libryd_tprof.so timeout -k 10 200 python -u tools/traj_prof.py 16 > $O/phase_new.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
for v in $2; do
  RYD_ENGINE_LIB=$PWD/build/libryd_$v.so timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5_$v.json 2> $O/bench_c5_$v.err || exit 1
done
RYD_T_SYM=0 timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5_old.json 2> $O/bench_c5_old.err || exit 1
cat $O/phase_new.log
for f in $O/bench_c5*.json; do python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f', r['kernel_ms'], r['frac'], d.get('exec_over_useful'))"; done
