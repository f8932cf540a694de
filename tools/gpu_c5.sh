# C5 iteration loop: trajectory GPU tests + C5 bench line (no CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-c5}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_trajectories.py -x -v --timeout 240 --timeout-method thread > $O/pytest_traj.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err
echo "exit=$?"
