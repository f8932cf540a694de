# X_BASE variants of the propagator kernel (build_var/lib_xb*.so) on the C2 and C3 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tune2
for v in 2 3 4 6; do
  RYD_ENGINE_LIB=$PWD/build_var/lib_xb$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/tune2/c2_xb$v.json 2>&1 || exit 1
  RYD_ENGINE_LIB=$PWD/build_var/lib_xb$v.so timeout -k 10 120 python bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/tune2/c3_xb$v.json 2>&1 || exit 1
done
echo done
