# X_BASE variants of the propagator kernel (build_var/lib_xb*.so) on the C2 and C3 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-tune3}
mkdir -p $O
for v in ${XB_LIST:-1 1.5 2 3}; do
  RYD_ENGINE_LIB=$PWD/build_var/lib_xb$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/c2_xb$v.json 2>&1 || exit 1
  RYD_ENGINE_LIB=$PWD/build_var/lib_xb$v.so timeout -k 10 120 python bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline > $O/c3_xb$v.json 2>&1 || exit 1
done
echo done
