// Probe: issue cost of v_fmac_f64 (plain) vs v_fmac_f64_dpp row_newbcast, one wave per
// SIMD and 3 waves per SIMD, via wall-clock events over many iterations.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int MODE>
__global__ __launch_bounds__(64) void k(double* out, int iters) {
  double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  double c0 = 1e-9 * threadIdx.x, c1 = c0 * 0.5, w = 0.999;
  for (int i = 0; i < iters; ++i) {
    if (MODE == 0) {
      asm volatile(
          "v_fmac_f64_e32 %0, %8, %9\n\tv_fmac_f64_e32 %1, %8, %9\n\tv_fmac_f64_e32 %2, %8, %9\n\tv_fmac_f64_e32 %3, %8, %9\n\t"
          "v_fmac_f64_e32 %4, %10, %9\n\tv_fmac_f64_e32 %5, %10, %9\n\tv_fmac_f64_e32 %6, %10, %9\n\tv_fmac_f64_e32 %7, %10, %9"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "v"(c0), "v"(w), "v"(c1));
    } else if (MODE == 1) {
      asm volatile(
          "v_fmac_f64_dpp %0, %8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_fmac_f64_dpp %1, %8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
          "v_fmac_f64_dpp %2, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
          "v_fmac_f64_dpp %3, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
          "v_fmac_f64_dpp %4, %10, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
          "v_fmac_f64_dpp %5, %10, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
          "v_fmac_f64_dpp %6, %10, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
          "v_fmac_f64_dpp %7, %10, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "v"(c0), "v"(w), "v"(c1));
    } else {
      asm volatile(
          "v_mov_b64_dpp %0, %8 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b64_dpp %1, %8 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b64_dpp %2, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b64_dpp %3, %8 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b64_dpp %4, %10 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b64_dpp %5, %10 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b64_dpp %6, %10 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b64_dpp %7, %10 row_newbcast:8 row_mask:0xf bank_mask:0xf"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "v"(c0), "v"(w), "v"(c1));
    }
  }
  out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

int main() {
  double* out;
  hipMalloc(&out, sizeof(double) * 64 * 8192);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  const char* names[3] = {"v_fmac_f64_e32", "v_fmac_f64_dpp", "v_mov_b64_dpp"};
  for (int mode = 0; mode < 3; ++mode)
    for (int wps : {1, 2, 3, 4}) {
      const int blocks = 1024 * wps;   // 256 CUs x 4 SIMDs x wps
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0, 0);
        if (mode == 0) k<0><<<blocks, 64>>>(out, iters);
        if (mode == 1) k<1><<<blocks, 64>>>(out, iters);
        if (mode == 2) k<2><<<blocks, 64>>>(out, iters);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep == 1) {
          const double instr = 8.0 * iters;   // per wave
          const double cyc = ms * 1e-3 * 2.4e9;
          printf("%-16s waves/SIMD %d: %.3f ms, %.2f cycles per instruction per SIMD\n", names[mode], wps, ms,
                 cyc / (instr * wps));
        }
      }
    }
  return 0;
}
