# Round check on one MI355X: smoke -> gpu tests -> benches (C2 metric line, C3, C4, C5)
# -> rocprof kernel stats (C2, C3, C5) -> PMC traffic passes for C2 (one counter per pass).
# Usage (from this container): gpurun --timeout 1200 -- bash tools/gpu_round.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-round}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench_c2.json 2> $O/bench_c2.err && \
timeout -k 10 300 python -u bench.py --workload c3 --steps 5 --warmup 1 > $O/bench_c3.json 2> $O/bench_c3.err && \
timeout -k 10 300 python -u bench.py --workload c4 --steps 5 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err && \
timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 2 > $O/bench_c5.json 2> $O/bench_c5.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/rocprof_c2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline > $O/rocprof_c3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/rocprof_c5.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_c2 -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_fetch_c2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_c2 -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_write_c2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_c5 -o run -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_fetch_c5.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_c5 -o run -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_write_c5.log 2>&1
echo "exit=$?"
