# C5 kernel profile: rocprofv3 kernel stats, then HBM traffic (one counter per pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-prof_c5}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python bench.py --workload c5 --steps 10 --warmup 2 > $O/rocprof_c5.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/rocprof_c2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_c5 -o run -- python bench.py --workload c5 --steps 2 --warmup 1 > $O/pmc_fetch_c5.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_c5 -o run -- python bench.py --workload c5 --steps 2 --warmup 1 > $O/pmc_write_c5.log 2>&1
echo "exit=$?"
