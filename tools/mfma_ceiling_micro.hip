// Microbenchmark: the fp32 MFMA ceiling on this part with no memory traffic at all: every wave
// issues v_mfma_f32_32x32x2_f32 back to back on NACC independent accumulators (register
// operands), at W waves per SIMD. Prints TFLOP/s against the 157.3 TF nominal (2.4 GHz) peak.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(256) void k_pure(float* out, int iters, float a0, float b0) {
  f32x16 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  float a = a0 + threadIdx.x * 1e-7f, b = b0 - threadIdx.x * 1e-7f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[i][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int NACC>
void run(int wgs_per_cu, float* out, int iters = 2000) {
  const int wgs = 256 * wgs_per_cu;
  k_pure<NACC><<<wgs, 256>>>(out, 10, 1.f, 1.f);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  k_pure<NACC><<<wgs, 256>>>(out, iters, 1.f, 1.f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double flop = 2.0 * 32 * 32 * 2 * 8.0 * NACC * iters * (wgs * 4.0);  // per wave-instruction x waves
  printf("NACC %d  %d waves/SIMD, %6d iters: %9.1f us  %6.1f TF/s  (%.0f%% of 157.3)\n", NACC, wgs_per_cu, iters, ms * 1e3,
         flop / (ms * 1e-3) / 1e12, 100.0 * flop / (ms * 1e-3) / 1e12 / 157.3);
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 8 * 256 * 4);
  for (int rep = 0; rep < 2; ++rep) {
    run<2>(1, out);
    run<4>(1, out);
    run<2>(2, out);
    run<2>(5, out);
    run<4>(5, out);
  }
  // sustained: the same instruction stream for longer (clock under a full-chip MFMA load)
  for (int iters : {2000, 8000, 32000}) run<2>(5, out, iters);
  for (int iters : {500, 2000, 8000}) run<4>(5, out, iters);
  // accumulators per wave x waves per SIMD
  for (int w : {1, 2, 3, 4, 5}) {
    run<1>(w, out, 2000);
    run<2>(w, out, 1000);
    run<4>(w, out, 500);
    run<8>(w, out, 250);
  }
  return 0;
}
