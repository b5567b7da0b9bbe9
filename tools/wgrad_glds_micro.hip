// Microbenchmark for the weight-gradient GEMM (k_wgrad's shape: C[512 x 128] += A^T B over a long
// K slice, A = dG rows [K][512], B = [x | h] rows [K][128], both k-major) on the fp32 MFMA core:
//   reg   -- the library's mainloop (global -> VGPR -> ds_write, 2 LDS stages, one barrier/K-tile)
//   glds  -- direct-to-LDS loads (global_load_lds_dwordx4), 3 LDS stages, a counted vmcnt that
//            leaves the next tile in flight across the raw barrier, no staging VGPRs.
// Also checks the glds result against the reg result. Prints TFLOP/s (HIP events).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
#include "kernels.h"
#include "loaders.h"
using namespace smaml;

using CfgR = GemmCfg<512, 128, 8, 1, false, false, 16>;
struct CfgG : CfgR {  // unpadded B rows (a glds wave-instruction writes 2 rows of 128 floats)
  static constexpr int LDB = 128;
  static constexpr int B_STAGE = 16 * 128;
};
struct CfgG4 : CfgG {  // unpadded A rows too (the 4-stage ring needs all 160 KB)
  static constexpr int LDA = 512;
  static constexpr int A_STAGE = 16 * 512;
};
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_void;

#ifndef KCH_
#define KCH_ 3328
#endif
#ifndef SLICES_
#define SLICES_ 64
#endif
constexpr int KCH = KCH_;  // K rows per workgroup (a k_wgrad split)
constexpr int SLICES = SLICES_;  // distinct K slices (1536 = every workgroup its own, as in k_wgrad)

__device__ __forceinline__ void glds16(const float* g, float* l) {
  __builtin_amdgcn_global_load_lds((gbl_void*)g, (lds_void*)l, 16, 0, 0);
}

// tile kt of this workgroup's slice into stage st: 5 glds per wave (4 x A half-rows, 1 x B 2 rows)
template <int LDA_ = CfgG::LDA>
__device__ __forceinline__ void issue_tile(const float* A, const float* B, int k0, float* As, float* Bs) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int row = 2 * w + r;
      glds16(A + (int64_t)(k0 + row) * 512 + half * 256 + 4 * lane, As + row * LDA_ + half * 256);
    }
  const int brow = 2 * w + (lane >> 5);
  glds16(B + (int64_t)(k0 + brow) * 128 + 4 * (lane & 31), Bs + 2 * w * 128);
}

__global__ __launch_bounds__(512) void k_glds(const float* A0, const float* B0, float* O) {
  __shared__ float smem[3 * (CfgG::A_STAGE + CfgG::B_STAGE)];
  float* As = smem;
  float* Bs = smem + 3 * CfgG::A_STAGE;
  const int sl = blockIdx.x % SLICES;
  const float* A = A0 + (int64_t)sl * KCH * 512;
  const float* B = B0 + (int64_t)sl * KCH * 128;
  Acc<CfgG> acc;
  acc.zero();
  NoHook hook;
  constexpr int nkt = KCH / 16;
  issue_tile(A, B, 0, As, Bs);
  issue_tile(A, B, 16, As + CfgG::A_STAGE, Bs + CfgG::B_STAGE);
  for (int kt = 0; kt < nkt; ++kt) {
    if (kt + 1 < nkt)
      asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int st = kt % 3;
    if (kt + 2 < nkt) {
      const int s2 = (kt + 2) % 3;
      issue_tile(A, B, (kt + 2) * 16, As + s2 * CfgG::A_STAGE, Bs + s2 * CfgG::B_STAGE);
    }
    __builtin_amdgcn_s_setprio(1);
    mma_tile<CfgG>(As + st * CfgG::A_STAGE, Bs + st * CfgG::B_STAGE, acc, hook);
    __builtin_amdgcn_s_setprio(0);
  }
#pragma unroll
  for (int i = 0; i < CfgG::WTM; ++i)
#pragma unroll
    for (int j = 0; j < CfgG::WTN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        O[((int64_t)blockIdx.x * 512 + acc_row<CfgG>(i, r)) * 128 + acc_col<CfgG>(j)] = acc.v[i][j][r];
}

// 4-stage ring (160 KB: the whole LDS), three tiles in flight
__global__ __launch_bounds__(512) void k_glds4(const float* A0, const float* B0, float* O) {
  __shared__ float smem[4 * (CfgG4::A_STAGE + CfgG4::B_STAGE)];
  float* As = smem;
  float* Bs = smem + 4 * CfgG4::A_STAGE;
  const int sl = blockIdx.x % SLICES;
  const float* A = A0 + (int64_t)sl * KCH * 512;
  const float* B = B0 + (int64_t)sl * KCH * 128;
  Acc<CfgG4> acc;
  acc.zero();
  NoHook hook;
  constexpr int nkt = KCH / 16;
  issue_tile<512>(A, B, 0, As, Bs);
  issue_tile<512>(A, B, 16, As + CfgG4::A_STAGE, Bs + CfgG4::B_STAGE);
  issue_tile<512>(A, B, 32, As + 2 * CfgG4::A_STAGE, Bs + 2 * CfgG4::B_STAGE);
  for (int kt = 0; kt < nkt; ++kt) {
    if (kt + 2 < nkt)
      asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else if (kt + 1 < nkt)
      asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int st = kt & 3;
    if (kt + 3 < nkt) {
      const int s3 = (kt + 3) & 3;
      issue_tile<512>(A, B, (kt + 3) * 16, As + s3 * CfgG4::A_STAGE, Bs + s3 * CfgG4::B_STAGE);
    }
    __builtin_amdgcn_s_setprio(1);
    mma_tile<CfgG4>(As + st * CfgG4::A_STAGE, Bs + st * CfgG4::B_STAGE, acc, hook);
    __builtin_amdgcn_s_setprio(0);
  }
#pragma unroll
  for (int i = 0; i < CfgG4::WTM; ++i)
#pragma unroll
    for (int j = 0; j < CfgG4::WTN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        O[((int64_t)blockIdx.x * 512 + acc_row<CfgG4>(i, r)) * 128 + acc_col<CfgG4>(j)] = acc.v[i][j][r];
}

__global__ __launch_bounds__(512) void k_reg(const float* A0, const float* B0, float* O) {
  __shared__ float smem[CfgR::SMEM_FLOATS];
  const int sl = blockIdx.x % SLICES;
  RowMajorMC la{A0 + (int64_t)sl * KCH * 512, KCH, 512};
  RowMajorMC lb{B0 + (int64_t)sl * KCH * 128, KCH, 128};
  Acc<CfgR> acc;
  acc.zero();
  gemm_mainloop<CfgR>(la, lb, 0, 0, 0, KCH, acc, smem);
#pragma unroll
  for (int i = 0; i < CfgR::WTM; ++i)
#pragma unroll
    for (int j = 0; j < CfgR::WTN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        O[((int64_t)blockIdx.x * 512 + acc_row<CfgR>(i, r)) * 128 + acc_col<CfgR>(j)] = acc.v[i][j][r];
}

__global__ void k_fill(float* p, size_t n, size_t off) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (float)(((i + off) * 2654435761u) % 1000) / 1000.f - 0.5f;
}

template <class K>
float timeit(K kern, int wgs, const float* A, const float* B, float* O) {
  kern<<<wgs, 512>>>(A, B, O);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int i = 0; i < 5; ++i) kern<<<wgs, 512>>>(A, B, O);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  const size_t na = (size_t)SLICES * KCH * 512, nb = (size_t)SLICES * KCH * 128;
  float *A, *B, *O1, *O2;
  if (hipMalloc(&A, na * 4) || hipMalloc(&B, nb * 4)) return 1;
  const int wgs = 256 * 6;
  if (hipMalloc(&O1, (size_t)wgs * 512 * 128 * 4) || hipMalloc(&O2, (size_t)wgs * 512 * 128 * 4)) return 1;
  k_fill<<<4096, 256>>>(A, na, 0);
  k_fill<<<4096, 256>>>(B, nb, 12345);
  const double fl = 2.0 * 512 * 128 * KCH * wgs;
  for (int rep = 0; rep < 3; ++rep) {
    const float tr = timeit(k_reg, wgs, A, B, O1);
    const float tg = timeit(k_glds, wgs, A, B, O2);
    const float t4 = timeit(k_glds4, wgs, A, B, O1);
    printf("glds4 %8.1f us %6.1f TF/s\n", t4 * 1e3, fl / (t4 * 1e-3) / 1e12);
    printf("reg  %8.1f us %6.1f TF/s | glds %8.1f us %6.1f TF/s\n", tr * 1e3, fl / (tr * 1e-3) / 1e12, tg * 1e3,
           fl / (tg * 1e-3) / 1e12);
  }
  std::vector<float> o1((size_t)4 * 512 * 128), o2(o1.size());
  hipMemcpy(o1.data(), O1, o1.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(o2.data(), O2, o2.size() * 4, hipMemcpyDeviceToHost);
  double maxd = 0, maxv = 0;
  for (size_t i = 0; i < o1.size(); ++i) {
    maxd = fmax(maxd, fabs((double)o1[i] - o2[i]));
    maxv = fmax(maxv, fabs((double)o1[i]));
  }
  printf("glds vs reg: max |diff| %.3g (max |value| %.3g)\n", maxd, maxv);
  return hipGetLastError() != hipSuccess;
}
