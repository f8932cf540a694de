# bench.py --gpus N self-launch on the 1-GPU lease (both ranks on device 0: functional
# check, not scaling) + the C2 single-rank line for comparison.
# Usage: gpurun --timeout 600 -- bash tools/gpu_launch.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-launch}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2_n1.json 2> $O/bench_c2_n1.err && \
timeout -k 10 240 python -u bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_c2_n2.json 2> $O/bench_c2_n2.err && \
timeout -k 10 240 python -u bench.py --workload c4 --gpus 2 --steps 3 --warmup 1 > $O/bench_c4_n2.json 2> $O/bench_c4_n2.err && \
timeout -k 10 240 python -u bench.py --workload c5 --gpus 2 --steps 3 --warmup 1 > $O/bench_c5_n2.json 2> $O/bench_c5_n2.err
echo "exit=$?"
