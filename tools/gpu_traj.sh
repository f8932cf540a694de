# C5 trajectory kernel: GPU parity tests, then a short C5 timing probe
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/traj
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_trajectories.py -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
echo "exit=$?"
timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err
echo "bench exit=$?"
