# tuning variants (X_BASE, squaring unroll) + PMC passes on the default build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tune
timeout -k 10 60 rocprofv3 -L > gpurun_out/tune/counters.txt 2>&1 || true
for v in xb1p5 xb3 xb6 xb3u5 xb6u5; do
  RYD_ENGINE_LIB=$PWD/build_var/lib_$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/tune/bench_$v.json 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/tune/pmc_fetch -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/tune/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/tune/pmc_write -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/tune/pmc_write.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d gpurun_out/tune/pmc_sq1 -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/tune/pmc_sq1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --output-format csv -d gpurun_out/tune/pmc_sq2 -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/tune/pmc_sq2.log 2>&1
echo "exit=$?"
