# C2 / C3 bench lines: default library vs build_var/lib_occ4.so (identical-atom propagator kernel at 3 waves/SIMD)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-occ}
mkdir -p $O
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/c2_base.json 2>&1 && \
RYD_ENGINE_LIB=$PWD/build_var/lib_occ4.so timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/c2_occ4.json 2>&1 && \
timeout -k 10 120 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_base.json 2>&1 && \
RYD_ENGINE_LIB=$PWD/build_var/lib_occ4.so timeout -k 10 120 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_occ4.json 2>&1
echo "exit=$?"
