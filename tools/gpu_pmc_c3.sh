# SQ stall/issue counters and kernel stats for the C3 smooth-JP propagator kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_c3}
mkdir -p $O
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline > $O/c3_stats.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/sq -o run -- python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > $O/c3_sq.log 2>&1
echo "exit=$?"
