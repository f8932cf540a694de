# Round check on one MI355X: smoke -> gpu tests -> benches -> rocprof stats -> PMC traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/round
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench_c2.json 2> $O/bench_c2.err && \
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --method cheb_vector --no-cpu-baseline > $O/bench_c2_vector.json 2>&1 && \
timeout -k 10 300 python bench.py --workload c3 --steps 5 --warmup 1 > $O/bench_c3.json 2>&1 && \
timeout -k 10 300 python bench.py --workload c3 --steps 2 --warmup 1 --method cheb_vector > $O/bench_c3_vector.json 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/rocprof_c2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_c2 -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_fetch_c2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_c2 -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_write_c2.log 2>&1
echo "exit=$?"
