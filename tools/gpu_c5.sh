# C5: trajectory GPU tests, then the bench with the paired kernel (RYD_T_PAIR=1) and the
# one-point-per-wave kernel (RYD_T_PAIR=0) at several ladder depths, in one box session.
# Usage: gpurun -- bash tools/gpu_c5.sh TAG [notest]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-c5}
mkdir -p $O
if [ "$2" != notest ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_trajectories.py -x -q --timeout 300 --timeout-method thread > $O/pytest_traj.log 2>&1 || { echo "traj tests failed"; tail -30 $O/pytest_traj.log; exit 1; }
  tail -2 $O/pytest_traj.log
fi
for P in 1 0; do
  for L in ${LADDERS:-24 16 12}; do
    RYD_T_PAIR=$P timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline --ladder $L > $O/c5_pair${P}_L$L.json 2> $O/c5_pair${P}_L$L.err || { echo "bench pair=$P L=$L failed"; tail -5 $O/c5_pair${P}_L$L.err; exit 1; }
    python -c "import json; d=json.load(open('$O/c5_pair${P}_L$L.json')); r=d['roofline']; print('pair=$P L=$L', round(d['value']), round(r['kernel_ms'],4), round(r['frac'],4), round(r['exec_over_useful'],3))"
  done
done
echo done
