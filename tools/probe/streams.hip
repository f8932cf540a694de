// Probe: do two non-blocking streams on one device overlap (kernel | kernel,
// kernel | pinned H2D)?  Prints event timestamps relative to the first event.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void spin(double* out, long iters) {
  double x = threadIdx.x;
  for (long i = 0; i < iters; ++i) x = x * 0.999999 + 1e-7;
  if (x == 12345.0) out[threadIdx.x] = x;   // keep the loop
}

#define CK(e) do { hipError_t r = (e); if (r != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(r), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  long iters = argc > 1 ? atol(argv[1]) : 200000;
  size_t bytes = 2 << 20;
  hipStream_t s[2];
  for (int k = 0; k < 2; ++k) CK(hipStreamCreateWithFlags(&s[k], hipStreamNonBlocking));
  double *d0, *d1, *hp;
  CK(hipMalloc(&d0, bytes));
  CK(hipMalloc(&d1, bytes));
  CK(hipHostMalloc((void**)&hp, bytes, hipHostMallocPortable));
  hipEvent_t e[8];
  for (int k = 0; k < 8; ++k) CK(hipEventCreate(&e[k]));
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipDeviceSynchronize());
      // stream 0: kernel (few blocks, long)
      CK(hipEventRecord(e[0], s[0]));
      spin<<<64, 64, 0, s[0]>>>(d0, iters);
      CK(hipEventRecord(e[1], s[0]));
      // stream 1: H2D (mode 0/2) then kernel (mode 1/2)
      CK(hipEventRecord(e[2], s[1]));
      if (mode != 1) CK(hipMemcpyAsync(d1, hp, bytes, hipMemcpyHostToDevice, s[1]));
      CK(hipEventRecord(e[3], s[1]));
      if (mode != 0) spin<<<64, 64, 0, s[1]>>>(d1, iters);
      CK(hipEventRecord(e[4], s[1]));
      CK(hipDeviceSynchronize());
      float t[5];
      for (int k = 0; k < 5; ++k) CK(hipEventElapsedTime(&t[k], e[0], e[k]));
      printf("mode %d rep %d: s0 kernel [%.3f, %.3f]  s1 start %.3f  after-h2d %.3f  after-kernel %.3f\n",
             mode, rep, t[0], t[1], t[2], t[3], t[4]);
    }
  }
  return 0;
}
