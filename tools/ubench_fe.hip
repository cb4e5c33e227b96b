// Field-multiply throughput microbenchmark (gfx950): independent chains of
// fd_fe_mul / fd_fe_sq per lane, full occupancy, measured with HIP events.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "fd_ed25519_gpu_fe.h"

#define ITERS 256
template<int CH, int SQ>
__global__ void __launch_bounds__(256) k_mul(fd_gpu_fe_t *out, int seed) {
  fd_gpu_fe_t x[CH], y;
  for (int c = 0; c < CH; c++) for (int k = 0; k < 10; k++) x[c].v[k] = (int)((threadIdx.x * 7919u + c * 104729u + k * 31u + seed) & 0x1ffffff) - (1 << 24);
  for (int k = 0; k < 10; k++) y.v[k] = (int)((threadIdx.x * 13u + k * 17u + seed) & 0xffffff);
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int c = 0; c < CH; c++) { if (SQ) fd_fe_sq(x[c], x[c]); else fd_fe_mul(x[c], x[c], y); }
  }
  fd_gpu_fe_t r = x[0];
  for (int c = 1; c < CH; c++) for (int k = 0; k < 10; k++) r.v[k] ^= x[c].v[k];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template<int CH, int SQ> void run(const char *name, fd_gpu_fe_t *out, int blocks) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((k_mul<CH,SQ>), dim3(blocks), dim3(256), 0, 0, out, 1);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 3; r++) hipLaunchKernelGGL((k_mul<CH,SQ>), dim3(blocks), dim3(256), 0, 0, out, 2 + r);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double muls = 3.0 * blocks * 256.0 * ITERS * CH;
  printf("%-14s chains=%d  %.3f ms  %.3f G fmul/s  (%.1f lane-cycles/fmul @2.4GHz, 1024 SIMD x 32 lanes)\n", name, CH, ms, muls / (ms * 1e-3) / 1e9,
         (ms * 1e-3 * 2.4e9 * 1024 * 32) / muls);
}

int main() {
  int blocks = 256 * 8;
  fd_gpu_fe_t *out; hipMalloc(&out, (size_t)blocks * 256 * sizeof(fd_gpu_fe_t));
  run<1,0>("mul", out, blocks); run<2,0>("mul", out, blocks); run<4,0>("mul", out, blocks);
  run<1,1>("sq", out, blocks); run<2,1>("sq", out, blocks); run<4,1>("sq", out, blocks);
  return 0;
}
