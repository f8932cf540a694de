// Probe: FP64 matrix-core rate on gfx950 and whether it overlaps FP64 VALU work.
//   MODE 0: 8 independent v_mfma_f64_16x16x4f64 accumulator chains per iteration
//   MODE 1: 32 v_fmac_f64 per iteration (16 independent chains, 2 each)
//   MODE 2: both streams interleaved in one wave (8 MFMA + 32 FMA per iteration)
// One wave per SIMD (1024 workgroups of 64) or W waves per SIMD; wall time by events.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe/mfma_f64 tools/probe/mfma_f64.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(64) void k(double* out, int iters) {
  const double a = 1.0 + 1e-9 * threadIdx.x, b = 0.999999;
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0, c6 = c0, c7 = c0;
  double f[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) f[j] = 1e-3 * (j + threadIdx.x);
  for (int i = 0; i < iters; ++i) {
    if (MODE == 0 || MODE == 2) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
      c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c4, 0, 0, 0);
      c5 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c5, 0, 0, 0);
      c6 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c6, 0, 0, 0);
      c7 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c7, 0, 0, 0);
    }
    if (MODE == 1 || MODE == 2) {
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int j = 0; j < 16; ++j) asm volatile("v_fmac_f64_e32 %0, %1, %2" : "+v"(f[j]) : "v"(a), "v"(b));
    }
  }
  double s = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) s += f[j];
  d4 t = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
  out[blockIdx.x * 64 + threadIdx.x] = s + t.x + t.y + t.z + t.w;
}

template <int MODE>
float run(double* out, int blocks, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), 0, 0, out, iters);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return ms;
}

int main() {
  double* out;
  hipMalloc(&out, 64 * 8192 * sizeof(double));
  const int iters = 4000;
  for (int w = 1; w <= 4; w *= 2) {
    const int blocks = 1024 * w;                // w waves per SIMD
    const float m0 = run<0>(out, blocks, iters), m1 = run<1>(out, blocks, iters), m2 = run<2>(out, blocks, iters);
    const double mf = 8.0 * iters * blocks, vf = 32.0 * iters * blocks;   // instructions
    printf("waves/SIMD %d: MFMA-only %.3f ms (%.1f cyc/MFMA/SIMD at 2.4 GHz, %.1f TF)  VALU-only %.3f ms "
           "(%.2f cyc/FMA/SIMD, %.1f TF)  both %.3f ms (sum %.3f, max %.3f)\n",
           w, m0, m0 * 1e-3 * 2.4e9 / (mf / 1024), mf * 2048 / (m0 * 1e-3) / 1e12, m1,
           m1 * 1e-3 * 2.4e9 / (vf / 1024), vf * 128 / (m1 * 1e-3) / 1e12, m2, m0 + m1, m0 > m1 ? m0 : m1);
  }
  hipFree(out);
  return 0;
}
