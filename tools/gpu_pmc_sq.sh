# SQ stall/issue counters for the C2 propagator kernel and the C5 trajectory kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_sq}
mkdir -p $O
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/c2 -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/c2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/c5 -o run -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5.log 2>&1
echo "exit=$?"
