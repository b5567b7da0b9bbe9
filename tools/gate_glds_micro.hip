// Microbenchmark for the LSTM gate GEMM shape (C[M x 512] = A[M x K] . B[512 x K]^T, both operands
// k-contiguous, K = 384): the library's 128 x 128 register-staged tile (4 waves, 4 workgroups per
// CU) against a 256 x 256 tile with 8 waves of 64 x 128 and direct-to-LDS loads into a 3-stage
// ring (one workgroup per CU; k-contiguous 16-float rows stored unpadded, 16-B chunks XOR-swizzled
// by (row >> 1) & 3 through the source address). GEMM only. Prints TFLOP/s and checks the glds
// result against the register-staged one.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
#include "kernels.h"
#include "loaders.h"
using namespace smaml;

typedef __attribute__((address_space(3))) void lds_void_g;
typedef __attribute__((address_space(1))) const void gbl_void_g;
__device__ __forceinline__ void glds16g(const float* g, float* l) {
  __builtin_amdgcn_global_load_lds((gbl_void_g*)g, (lds_void_g*)l, 16, 0, 0);
}

constexpr int N = 512, K = 384;
using CfgR = GemmCfg<128, 128, 4, 1, true, true, 16>;

__global__ __launch_bounds__(256) void k_reg(const float* A, const float* B, float* O, int M) {
  __shared__ float smem[CfgR::SMEM_FLOATS];
  const int m0 = blockIdx.x * 128, n0 = blockIdx.y * 128;
  Acc<CfgR> acc;
  acc.zero();
  RowMajorKC la{A, M, K};
  RowMajorKC lb{B, N, K};
  gemm_mainloop<CfgR>(la, lb, m0, n0, 0, K, acc, smem);
#pragma unroll
  for (int j = 0; j < CfgR::WTN; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      O[(int64_t)(m0 + acc_row<CfgR>(0, r)) * N + n0 + acc_col<CfgR>(j)] = acc.v[0][j][r];
}

// 256 x 256 tile, 8 waves as 4 (rows) x 2 (cols), each 64 x 128 (2 x 4 MFMA blocks)
struct CfgB {
  static constexpr int BM = 256, BN = 256, WAVES_M = 4, WAVES_N = 2, WTM = 2, WTN = 4, NTH = 512;
};
constexpr int TS = 256 * 16;  // floats per operand tile per stage

__device__ __forceinline__ void issue(const float* A, const float* B, int m0, int n0, int k0, float* As, float* Bs) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // 16 instructions per operand tile: wave w -> row blocks 2w, 2w+1
    const int rb = 2 * w + i;
    const int row = 16 * rb + (lane >> 2), pc = lane & 3, lc = pc ^ ((row >> 1) & 3);
    glds16g(A + (int64_t)(m0 + row) * K + k0 + 4 * lc, As + rb * 256);
    glds16g(B + (int64_t)(n0 + row) * K + k0 + 4 * lc, Bs + rb * 256);
  }
}

__device__ __forceinline__ float4 fragkc(const float* s, int row, int c) {
  const int pc = c ^ ((row >> 1) & 3);
  return *reinterpret_cast<const float4*>(s + row * 16 + 4 * pc);
}

__global__ __launch_bounds__(512) void k_glds(const float* A, const float* B, float* O, int M) {
  __shared__ float smem[3 * 2 * TS];
  float* As = smem;
  float* Bs = smem + 3 * TS;
  const int m0 = blockIdx.x * 256, n0 = blockIdx.y * 256;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / CfgB::WAVES_N, wn = wave % CfgB::WAVES_N;
  const int arow = wm * 64 + (lane & 31), brow = wn * 128 + (lane & 31), h = lane >> 5;
  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  constexpr int nkt = K / 16;
  issue(A, B, m0, n0, 0, As, Bs);
  issue(A, B, m0, n0, 16, As + TS, Bs + TS);
  for (int kt = 0; kt < nkt; ++kt) {
    if (kt + 1 < nkt)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    const int st = kt % 3;
    if (kt + 2 < nkt) {
      const int s2 = (kt + 2) % 3;
      issue(A, B, m0, n0, (kt + 2) * 16, As + s2 * TS, Bs + s2 * TS);
    }
    const float* as = As + st * TS;
    const float* bs = Bs + st * TS;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float4 a[2], b[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = fragkc(as, arow + 32 * i, 2 * h + q);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = fragkc(bs, brow + 32 * j, 2 * h + q);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(a[i], e), f4get(b[j], e), acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int col = n0 + wn * 128 + 32 * j + (lane & 31);
        O[(int64_t)row * N + col] = acc[i][j][r];
      }
}

template <class Kern>
float timeit(Kern kern, dim3 grid, int nth, const float* A, const float* B, float* O, int M) {
  kern<<<grid, nth>>>(A, B, O, M);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int i = 0; i < 10; ++i) kern<<<grid, nth>>>(A, B, O, M);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 10;
}

int main() {
  const int M = 256 * 280;  // 71680 rows (5 tasks x 14112 rounded to whole 256-row tiles)
  float *A, *B, *O1, *O2;
  if (hipMalloc(&A, (size_t)M * K * 4) || hipMalloc(&B, (size_t)N * K * 4) || hipMalloc(&O1, (size_t)M * N * 4) ||
      hipMalloc(&O2, (size_t)M * N * 4))
    return 1;
  std::vector<float> h((size_t)M * K);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  hipMemcpy(A, h.data(), (size_t)M * K * 4, hipMemcpyHostToDevice);
  hipMemcpy(B, h.data() + 777, (size_t)N * K * 4, hipMemcpyHostToDevice);
  const double fl = 2.0 * M * N * K;
  for (int rep = 0; rep < 3; ++rep) {
    const float tr = timeit(k_reg, dim3(M / 128, N / 128), 256, A, B, O1, M);
    const float tg = timeit(k_glds, dim3(M / 256, N / 256), 512, A, B, O2, M);
    printf("reg 128x128 %8.1f us %6.1f TF/s | glds 256x256 %8.1f us %6.1f TF/s\n", tr * 1e3, fl / (tr * 1e-3) / 1e12,
           tg * 1e3, fl / (tg * 1e-3) / 1e12);
  }
  std::vector<float> o1((size_t)M * N), o2(o1.size());
  hipMemcpy(o1.data(), O1, o1.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(o2.data(), O2, o2.size() * 4, hipMemcpyDeviceToHost);
  double md = 0;
  for (size_t i = 0; i < o1.size(); ++i) md = fmax(md, fabs((double)o1[i] - o2[i]));
  printf("glds vs reg: max |diff| %.3g\n", md);
  return 0;
}
