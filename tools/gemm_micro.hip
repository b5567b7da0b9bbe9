// Microbenchmark of the fp32 MFMA GEMM core (gemm_core.h) over tile configurations, on the
// shapes the STGCN-LSTM path runs: NT (C = A.B^T, both k-contiguous: gate / GCN GEMMs) and
// NN (C = A.B, B n-contiguous: BPTT / dX). Prints TFLOP/s per variant (HIP events, 10 reps).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "gemm_core.h"
#include "loaders.h"
using namespace smaml;

template <class C, bool NN>
__global__ __launch_bounds__(C::NTH) void k_bench(const float* A, const float* B, float* O, int M, int N, int K) {
  __shared__ float smem[C::SMEM_FLOATS];
  const int m0 = blockIdx.x * C::BM, n0 = blockIdx.y * C::BN;
  Acc<C> acc;
  acc.zero();
  RowMajorKC la{A, M, K};
  if (NN) {
    RowMajorMC lb{B, K, N};
    gemm_mainloop<C>(la, lb, m0, n0, 0, K, acc, smem);
  } else {
    RowMajorKC lb{B, N, K};
    gemm_mainloop<C>(la, lb, m0, n0, 0, K, acc, smem);
  }
#pragma unroll
  for (int i = 0; i < C::WTM; ++i)
#pragma unroll
    for (int j = 0; j < C::WTN; ++j) {
      const int c = n0 + acc_col<C>(j);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + acc_row<C>(i, r);
        if (m < M && c < N) O[(int64_t)m * N + c] = acc.v[i][j][r];
      }
    }
}

template <class C, bool NN>
void run(const char* name, const float* A, const float* B, float* O, int M, int N, int K) {
  dim3 grid((M + C::BM - 1) / C::BM, (N + C::BN - 1) / C::BN);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k_bench<C, NN><<<grid, C::NTH>>>(A, B, O, M, N, K);
  hipEventRecord(a);
  const int reps = 10;
  for (int i = 0; i < reps; ++i) k_bench<C, NN><<<grid, C::NTH>>>(A, B, O, M, N, K);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  ms /= reps;
  printf("%-34s M=%d N=%d K=%d  %8.3f ms  %6.1f TF/s  (lds %d B)\n", name, M, N, K, ms,
         2.0 * M * N * K / (ms * 1e-3) / 1e12, (int)(C::SMEM_FLOATS * 4));
}

int main() {
  const int M = 211680;
  size_t big = (size_t)M * 512;
  float *A, *B, *O;
  hipMalloc(&A, big * 4);
  hipMalloc(&B, 512 * 512 * 4);
  hipMalloc(&O, big * 4);
  std::vector<float> h(big);
  for (size_t i = 0; i < big; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  hipMemcpy(A, h.data(), big * 4, hipMemcpyHostToDevice);
  hipMemcpy(B, h.data(), 512 * 512 * 4, hipMemcpyHostToDevice);
  for (int K : {256, 384}) {
    run<GemmCfg<128, 128, 4, 1, true, true>, false>("NT 128x128 w4x1", A, B, O, M, 512, K);
    run<GemmCfg<128, 128, 2, 2, true, true>, false>("NT 128x128 w2x2", A, B, O, M, 512, K);
    run<GemmCfg<256, 128, 4, 2, true, true>, false>("NT 256x128 w4x2 (8 waves)", A, B, O, M, 512, K);
    run<GemmCfg<128, 256, 2, 4, true, true>, false>("NT 128x256 w2x4 (8 waves)", A, B, O, M, 512, K);
    run<GemmCfg<256, 256, 4, 2, true, true>, false>("NT 256x256 w4x2 (8 waves)", A, B, O, M, 512, K);
    run<GemmCfg<64, 128, 2, 2, true, true>, false>("NT 64x128 w2x2", A, B, O, M, 512, K);
    run<GemmCfg<128, 64, 2, 2, true, true>, false>("NT 128x64 w2x2", A, B, O, M, 512, K);
  }
  run<GemmCfg<128, 128, 4, 1, true, false>, true>("NN 128x128 w4x1", A, B, O, M, 128, 512);
  run<GemmCfg<128, 128, 2, 2, true, false>, true>("NN 128x128 w2x2", A, B, O, M, 128, 512);
  run<GemmCfg<64, 128, 2, 2, true, false>, true>("NN 64x128 w2x2", A, B, O, M, 128, 512);
  run<GemmCfg<128, 64, 2, 2, true, false>, true>("NN 128x64 w2x2", A, B, O, M, 128, 512);
  run<GemmCfg<256, 128, 4, 2, true, false>, true>("NN 256x128 w4x2 (8 waves)", A, B, O, M, 128, 512);
  run<GemmCfg<128, 128, 4, 1, true, false>, true>("NN 128x128 w4x1 K=128", A, B, O, M, 128, 128);
  return 0;
}
