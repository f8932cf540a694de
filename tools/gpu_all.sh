# full GPU check: trajectory tests first (newest), all gpu tests, smoke, C2 + C5 bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/all
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_trajectories.py -x -v --timeout 240 --timeout-method thread > $O/pytest_traj.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench_c2.json 2> $O/bench_c2.err && \
timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 2 > $O/bench_c5.json 2> $O/bench_c5.err
echo "exit=$?"
