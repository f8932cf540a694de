# Kernel stats (C2, C3 split) + extra SQ instruction-mix counters for the C2 propagator kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-prof_final}
mkdir -p $O
C="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2_stats -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/c2_stats.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3_stats -o run -- python bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline > $O/c3_stats.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/c2_mix -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/c2_mix.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/c3_mix -o run -- python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > $O/c3_mix.log 2>&1
echo "exit=$?"
