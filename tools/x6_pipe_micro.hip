// Microbenchmark for the staged bf16x6 mainloop on the weight-gradient shape (k_wgrad: C[BM x 128] +=
// A^T B over a long K slice; A = dG rows [K][BM], B = [x | h] rows [K][128], both n-contiguous):
//   lib    -- gemm_mainloop (gemm_core.h staged split, 2 LDS stages, one barrier per K-tile): the tile
//             loads of K-tile k+1 are issued before tile k's MFMAs and split + stored after them;
//   noload -- the same loop fed by a loader that reads no memory (split + MFMA + LDS only);
//   pipe2  -- two register sets: tile k+2's loads are issued at the top of iteration k, and tile k+1
//             (loaded one iteration earlier) is split and stored INTO the MFMA phase of tile k
//             (sched_group_barrier interleave), so neither the load latency nor the split VALU sits
//             between two MFMA phases.
// Prints TFLOP/s of f32 work (HIP events) and checks pipe2 against lib bitwise.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "kernels.h"
#include "loaders.h"
using namespace smaml;

#ifndef MICRO_BM
#define MICRO_BM 512
#endif
#ifndef MICRO_KCH
#define MICRO_KCH 3072
#endif
#ifndef MICRO_SLICES
#define MICRO_SLICES 96
#endif
#ifndef ILV_VALU
#define ILV_VALU 3  // split VALU per MFMA in the pipe2 interleave
#endif
#ifndef MICRO_BN
#define MICRO_BN 128
#endif
#ifndef MICRO_WN
#define MICRO_WN 1
#endif
constexpr int BMc = MICRO_BM, BNc = MICRO_BN;
#ifndef MICRO_WM
#define MICRO_WM (MICRO_BM / 64)  // waves along M (MICRO_BM / 128: one wave per SIMD with 128 x 128 wave tiles)
#endif
constexpr int WM = MICRO_WM;
using C = GemmCfg<BMc, BNc, WM, MICRO_WN, false, false, 16, 2, 2>;
constexpr int NTH = C::NTH;
constexpr int KCH = MICRO_KCH;
constexpr int SLICES = MICRO_SLICES;

struct NoMem {  // [K][cols] values from the indices (no memory traffic)
  int cols;
  __device__ __forceinline__ float4 operator()(int64_t k, int c) const {
    const float b = (float)((k * 131 + c) & 1023) * (1.f / 1024.f) - 0.5f;
    return make_float4(b, b + 0.001f, b - 0.002f, b + 0.003f);
  }
};

// mma_tile_x6s with a filler: after MFMA number q (of WTM * WTN * 6 per 16-k step) fill(q) runs, fenced
// by sched_barriers so the compiler keeps it there (fine-grained VALU / DS-write interleave).
template <class F>
__device__ __forceinline__ void mma_fill(const char* as, const char* bs, Acc<C>& acc, F&& fill) {
  const int wave = threadIdx.x >> 6;
  const int wm = wave / C::WAVES_N, wn = wave % C::WAVES_N;
  Split3 a[C::WTM];
#pragma unroll
  for (int i = 0; i < C::WTM; ++i) a[i] = frag_x6<C::BM, C::A_KC, C::BK>(as, wm * (C::WTM * 32) + 32 * i, 0);
  int q = 0;
#pragma unroll
  for (int j = 0; j < C::WTN; ++j) {
    const Split3 b = frag_x6<C::BN, C::B_KC, C::BK>(bs, wn * (C::WTN * 32) + 32 * j, 0);
#pragma unroll
    for (int i = 0; i < C::WTM; ++i) {
      f32x16 c = acc.v[i][j];
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i].p2, b.p0, c, 0, 0, 0);
      fill(q++);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i].p1, b.p1, c, 0, 0, 0);
      fill(q++);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i].p0, b.p2, c, 0, 0, 0);
      fill(q++);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i].p1, b.p0, c, 0, 0, 0);
      fill(q++);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i].p0, b.p1, c, 0, 0, 0);
      fill(q++);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i].p0, b.p0, c, 0, 0, 0);
      fill(q++);
      acc.v[i][j] = c;
    }
  }
}

// One float4 of a staged operand tile split into its image (store_tile_x6 for element i only).
template <int ROWS, int F4, bool KC>
__device__ __forceinline__ void store_one_x6(char* img, const float4& v, int i) {
  using I = X6Img<ROWS, KC, C::BK>;
  const int f = (int)threadIdx.x + C::NTH * i;
  int off;
  if (KC) {
    const int rr = f / (C::BK / 4), qq = f % (C::BK / 4);
    off = rr * I::RS + 16 * ((qq >> 1) ^ I::swz(rr)) + 8 * (qq & 1);
  } else {
    const int kk = f / (ROWS / 4), qq = f % (ROWS / 4);
    off = I::mc(kk, 8 * qq);
  }
  uint2 p0, p1, p2;
  split4(v, p0, p1, p2);
  *reinterpret_cast<uint2*>(img + off) = p0;
  *reinterpret_cast<uint2*>(img + I::PLANE + off) = p1;
  *reinterpret_cast<uint2*>(img + 2 * I::PLANE + off) = p2;
}

template <class LA, class LB>
__device__ __forceinline__ void pipe2(const LA& la, const LB& lb, int kbeg, int kend, Acc<C>& acc, float* smem) {
  constexpr int SA = C::AImg::BYTES;
  char* st0 = reinterpret_cast<char*>(smem);
  const int nkt = (kend - kbeg) / C::BK;
  float4 ra0[C::A_F4], rb0[C::B_F4], ra1[C::A_F4], rb1[C::B_F4];
  auto fetch = [&](float4(&ra)[C::A_F4], float4(&rb)[C::B_F4], int k0) {
    fetch_tile<C::BM, C::A_F4, C::NTH, C::A_KC, C::BK>(la, 0, k0, ra);
    fetch_tile<C::BN, C::B_F4, C::NTH, C::B_KC, C::BK>(lb, 0, k0, rb);
  };
  auto store = [&](char* st, const float4(&ra)[C::A_F4], const float4(&rb)[C::B_F4]) {
    store_tile_x6<C::BM, C::A_F4, C::NTH, C::A_KC, C::BK>(st, ra);
    store_tile_x6<C::BN, C::B_F4, C::NTH, C::B_KC, C::BK>(st + SA, rb);
  };
  fetch(ra0, rb0, kbeg);
  fetch(ra1, rb1, kbeg + C::BK);
  store(st0, ra0, rb0);
  __syncthreads();
  // body<P>: MFMAs of the tile in stage P; split + store of the next tile (register set P^1) into
  // stage P^1; the tile after that into register set P.
  auto body = [&](auto par, int kt) {
    constexpr int P = decltype(par)::value;
    float4(&rn)[C::A_F4] = P ? ra0 : ra1;  // next tile (kt + 1)
    float4(&rbn)[C::B_F4] = P ? rb0 : rb1;
    float4(&rf)[C::A_F4] = P ? ra1 : ra0;  // free set: tile kt + 2
    float4(&rbf)[C::B_F4] = P ? rb1 : rb0;
    if (kt + 2 < nkt) fetch(rf, rbf, kbeg + (kt + 2) * C::BK);
    const char* st = st0 + P * C::X6S_STAGE;
    __builtin_amdgcn_s_setprio(1);
    char* nx = st0 + (P ^ 1) * C::X6S_STAGE;
#if ILV_VALU > 0
    // unconditional (one basic block with the MFMAs): after the last tile it rewrites the idle stage
    constexpr int NQ = C::WTM * C::WTN * 6, NF = C::A_F4 + C::B_F4, GAP = NQ / (NF + 1);
    mma_fill(st, st + SA, acc, [&](int q) {
      if (q % GAP == GAP - 1 && q / GAP < NF) {
        const int f = q / GAP;
        if (f < C::A_F4)
          store_one_x6<C::BM, C::A_F4, C::A_KC>(nx, rn[f], f);
        else
          store_one_x6<C::BN, C::B_F4, C::B_KC>(nx + SA, rbn[f - C::A_F4], f - C::A_F4);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
#else
    mma_tile_x6s<C, -1>(st, st + SA, acc);
    store(nx, rn, rbn);
#endif
    __builtin_amdgcn_s_setprio(0);
    __syncthreads();
  };
  for (int kt = 0; kt < nkt; kt += 2) {
    body(std::integral_constant<int, 0>{}, kt);
    if (kt + 1 < nkt) body(std::integral_constant<int, 1>{}, kt + 1);
  }
}

#ifndef MICRO_WPE
#define MICRO_WPE (64 * MICRO_WM * MICRO_WN >= 512 ? 2 : MICRO_BM / MICRO_WM >= 128 ? 1 : 2)  // waves per SIMD
#endif
template <int MODE>
__global__ __attribute__((amdgpu_waves_per_eu(MICRO_WPE))) __launch_bounds__(NTH) void k_micro(const float* A0, const float* B0, float* O) {
  __shared__ float smem[C::SMEM_FLOATS];
  const int sl = blockIdx.x % SLICES;
  RowMajorMC la{A0 + (int64_t)sl * KCH * BMc, KCH, BMc};
  RowMajorMC lb{B0 + (int64_t)sl * KCH * BNc, KCH, BNc};
  Acc<C> acc;
  acc.zero();
  if (MODE == 0) gemm_mainloop<C, -1>(la, lb, 0, 0, 0, KCH, acc, smem);
  if (MODE == 1) gemm_mainloop<C, -1>(NoMem{BMc}, NoMem{BNc}, 0, 0, 0, KCH, acc, smem);
  if (MODE == 2) pipe2(la, lb, 0, KCH, acc, smem);
#pragma unroll
  for (int i = 0; i < C::WTM; ++i)
#pragma unroll
    for (int j = 0; j < C::WTN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        O[((int64_t)blockIdx.x * BMc + acc_row<C>(i, r)) * BNc + acc_col<C>(j)] = acc.v[i][j][r];
}

__global__ void k_fill(float* p, size_t n, size_t off) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (float)(((i + off) * 2654435761u) % 1000) / 1000.f - 0.5f;
}

template <class K>
float timeit(K kern, int wgs, const float* A, const float* B, float* O) {
  kern<<<wgs, NTH>>>(A, B, O);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int i = 0; i < 5; ++i) kern<<<wgs, NTH>>>(A, B, O);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  const size_t na = (size_t)SLICES * KCH * BMc, nb = (size_t)SLICES * KCH * BNc;
  float *A, *B, *O1, *O2;
  if (hipMalloc(&A, na * 4) || hipMalloc(&B, nb * 4)) return 1;
  const int wgs = 256 * 6 * (512 * 128 / (BMc * BNc));
  if (hipMalloc(&O1, (size_t)wgs * BMc * BNc * 4) || hipMalloc(&O2, (size_t)wgs * BMc * BNc * 4)) return 1;
  k_fill<<<4096, 256>>>(A, na, 0);
  k_fill<<<4096, 256>>>(B, nb, 12345);
  const double fl = 2.0 * BMc * BNc * KCH * wgs;
  printf("BM %d BN %d, %d threads, %d workgroups, K %d per workgroup, LDS %d B\n", BMc, BNc, NTH, wgs, KCH, C::SMEM_FLOATS * 4);
  for (int rep = 0; rep < 3; ++rep) {
    const float t0 = timeit(k_micro<0>, wgs, A, B, O1);
    const float t1 = timeit(k_micro<1>, wgs, A, B, O2);
    const float t2 = timeit(k_micro<2>, wgs, A, B, O2);
    printf("lib %8.1f us %6.1f TF/s | noload %8.1f us %6.1f TF/s | pipe2 %8.1f us %6.1f TF/s\n", t0 * 1e3,
           fl / (t0 * 1e-3) / 1e12, t1 * 1e3, fl / (t1 * 1e-3) / 1e12, t2 * 1e3, fl / (t2 * 1e-3) / 1e12);
  }
  std::vector<float> o1((size_t)wgs * BMc * BNc), o2(o1.size());
  hipMemcpy(o1.data(), O1, o1.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(o2.data(), O2, o2.size() * 4, hipMemcpyDeviceToHost);
  size_t nd = 0;
  for (size_t i = 0; i < o1.size(); ++i) nd += o1[i] != o2[i];
  printf("pipe2 vs lib: %zu of %zu outputs differ\n", nd, o1.size());
  return hipGetLastError() != hipSuccess;
}
