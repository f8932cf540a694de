# Round-3 measurement pass: C2 metric line (host_path with the pooled staging), the
# secondary kernels, the published optimiser workloads, rocprof summaries of each.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_r03_bench.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r03b}
O=gpurun_out/$TAG
mkdir -p $O
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline"
$B --steps 20 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err && \
$B --workload shaped --steps 5 --warmup 1 > $O/bench_shaped.json 2> $O/bench_shaped.err && \
$B --workload dim4 --steps 5 --warmup 1 > $O/bench_dim4.json 2> $O/bench_dim4.err && \
$B --workload ket --steps 5 --warmup 1 > $O/bench_ket.json 2> $O/bench_ket.err && \
$B --workload ket_cheb --steps 5 --warmup 1 > $O/bench_ket_cheb.json 2> $O/bench_ket_cheb.err && \
$B --workload coherence --steps 5 --warmup 1 > $O/bench_coherence.json 2> $O/bench_coherence.err && \
$B --workload opt_lp > $O/bench_opt_lp.json 2> $O/bench_opt_lp.err && \
$B --workload opt_smooth > $O/bench_opt_smooth.json 2> $O/bench_opt_smooth.err && \
for w in shaped dim4 ket ket_cheb coherence; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline > $O/rocprof_$w.log 2>&1 || exit 1
done && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_opt_lp -o run -- python bench.py --workload opt_lp --no-cpu-baseline > $O/rocprof_opt_lp.log 2>&1
echo "exit=$?"
