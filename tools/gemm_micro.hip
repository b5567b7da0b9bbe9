// Microbenchmark of the fp32 MFMA GEMM core (gemm_core.h): tile / BK variants on the STGCN-LSTM
// shapes, and the LSTM forward-step epilogue cost (GEMM + cell update + 6 stores per element)
// against the bare GEMM. Prints TFLOP/s per variant (HIP events, 10 reps).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "gemm_core.h"
#include "loaders.h"
using namespace smaml;

template <class C, bool NN, int EPI>
__global__ __launch_bounds__(C::NTH) void k_bench(const float* A, const float* B, float* O, float* O2, int M, int N,
                                                  int K) {
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
  if (EPI == 0) {
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
  } else {  // LSTM cell epilogue (C::WTN == 4 gates per wave, H = 128)
    constexpr int H = 128;
    const int wn = (threadIdx.x >> 6) % C::WAVES_N;
    const int j = (blockIdx.y * C::WAVES_N + wn) * 32 + (threadIdx.x & 31);
    const int rb = m0 + acc_row<C>(0, 0);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = rb + racc(r);
      if (m >= M) continue;
      const uint32_t oh = (uint32_t)m * H + j, og = (uint32_t)m * 4 * H + j;
      const float gi = sigmoidf_(acc.v[0][0][r]), gf = sigmoidf_(acc.v[0][1][r]);
      const float gg = tanhf_(acc.v[0][2][r]), go = sigmoidf_(acc.v[0][3][r]);
      const float cp = ldb(O2, 4u * oh);
      const float c = gf * cp + gi * gg;
      stb(O, 4u * og, gi);
      stb(O, 4u * (og + H), gf);
      stb(O, 4u * (og + 2 * H), gg);
      stb(O, 4u * (og + 3 * H), go);
      stb(O2, 4u * oh + 4u * M * H, c);
      stb(O2, 4u * oh + 8u * M * H, go * tanhf_(c));
    }
  }
}

template <class C, bool NN, int EPI = 0>
void run(const char* name, const float* A, const float* B, float* O, float* O2, int M, int N, int K) {
  dim3 grid((M + C::BM - 1) / C::BM, (N + C::BN - 1) / C::BN);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k_bench<C, NN, EPI><<<grid, C::NTH>>>(A, B, O, O2, M, N, K);
  hipEventRecord(a);
  const int reps = 10;
  for (int i = 0; i < reps; ++i) k_bench<C, NN, EPI><<<grid, C::NTH>>>(A, B, O, O2, M, N, K);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  ms /= reps;
  printf("%-40s M=%d N=%d K=%d  %8.3f ms  %6.1f TF/s  (lds %d B)\n", name, M, N, K, ms,
         2.0 * M * N * K / (ms * 1e-3) / 1e12, (int)(C::SMEM_FLOATS * 4));
}

int main() {
  const int M = 211680;
  size_t big = (size_t)M * 768;
  float *A, *B, *O, *O2;
  hipMalloc(&A, big * 4);
  hipMalloc(&B, 768 * 512 * 4);
  hipMalloc(&O, (size_t)M * 512 * 4);
  hipMalloc(&O2, (size_t)M * 128 * 4 * 3);
  std::vector<float> h(big);
  for (size_t i = 0; i < big; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  hipMemcpy(A, h.data(), big * 4, hipMemcpyHostToDevice);
  hipMemcpy(B, h.data(), 768 * 512 * 4, hipMemcpyHostToDevice);
  hipMemset(O2, 0, (size_t)M * 128 * 4 * 3);
  for (int K : {256, 384, 768}) {
    run<GemmCfg<128, 128, 4, 1, true, true>, false>("NT 128x128 w4x1 BK32", A, B, O, O2, M, 512, K);
    run<GemmCfg<128, 128, 4, 1, true, true, 64>, false>("NT 128x128 w4x1 BK64", A, B, O, O2, M, 512, K);
    run<GemmCfg<128, 128, 4, 1, true, true, 16>, false>("NT 128x128 w4x1 BK16", A, B, O, O2, M, 512, K);
    run<GemmCfg<128, 128, 4, 1, true, true>, false, 1>("NT 128x128 w4x1 BK32 +cell epi", A, B, O, O2, M, 512, K);
    run<GemmCfg<128, 128, 4, 1, true, true, 64>, false, 1>("NT 128x128 w4x1 BK64 +cell epi", A, B, O, O2, M, 512, K);
    run<GemmCfg<128, 256, 2, 4, true, true>, false>("NT 128x256 w2x4 BK32", A, B, O, O2, M, 512, K);
    run<GemmCfg<128, 128, 4, 1, true, true, 16>, false, 1>("NT 128x128 w4x1 BK16 +cell epi", A, B, O, O2, M, 512, K);
    run<GemmCfg<128, 256, 4, 2, true, true>, false, 1>("NT 128x256 w4x2 BK32 +cell epi", A, B, O, O2, M, 512, K);
    run<GemmCfg<128, 256, 4, 2, true, true, 16>, false, 1>("NT 128x256 w4x2 BK16 +cell epi", A, B, O, O2, M, 512, K);
    run<GemmCfg<64, 128, 2, 2, true, true, 16>, false, 0>("NT 64x128 w2x2 BK16", A, B, O, O2, M, 512, K);
  }
  run<GemmCfg<64, 128, 2, 2, true, false>, true>("NN 64x128 w2x2 BK32", A, B, O, O2, M, 128, 512);
  run<GemmCfg<64, 128, 2, 2, true, false, 16>, true>("NN 64x128 w2x2 BK16", A, B, O, O2, M, 128, 512);
  run<GemmCfg<128, 128, 4, 1, true, false, 16>, true>("NN 128x128 w4x1 BK16", A, B, O, O2, M, 128, 512);
  run<GemmCfg<64, 128, 2, 2, true, false, 64>, true>("NN 64x128 w2x2 BK64", A, B, O, O2, M, 128, 512);
  run<GemmCfg<128, 128, 2, 2, true, false, 64>, true>("NN 128x128 w2x2 BK64", A, B, O, O2, M, 128, 512);
  return 0;
}
