// Microbenchmark: the BPTT GEMM shape (M = 221 x 64 rows x 15 tasks, N = H = 128, K = 8H = 1024)
// on the fp32 MFMA core with the B operand (the weights) k-major ("MC", read with 4 ds_read_b32 per
// fragment: the kernels' current layout) vs row-major k-contiguous ("KC", one ds_read_b128 per
// fragment; padded LDS rows). GEMM only, result stored once. Prints TFLOP/s (HIP events).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "kernels.h"
#include "loaders.h"
using namespace smaml;

// Variant core: all LDS fragments of the K-tile first, then the K-tile's MFMAs (one wait).
template <class C>
__device__ __forceinline__ void mma_tile_all(const float* as, const float* bs, Acc<C>& acc) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / C::WAVES_N, wn = wave % C::WAVES_N;
  const int arow = wm * (C::WTM * 32) + (lane & 31);
  const int brow = wn * (C::WTN * 32) + (lane & 31);
  const int h = lane >> 5;
  constexpr int Q = C::BK / 8;
  float4 a[Q][C::WTM], b[Q][C::WTN];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
#pragma unroll
    for (int i = 0; i < C::WTM; ++i) a[q][i] = frag4<C::A_KC, C::LDA, C::BK>(as, arow + 32 * i, h, q);
#pragma unroll
    for (int j = 0; j < C::WTN; ++j) b[q][j] = frag4<C::B_KC, C::LDB, C::BK>(bs, brow + 32 * j, h, q);
  }
#pragma unroll
  for (int q = 0; q < Q; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int i = 0; i < C::WTM; ++i)
#pragma unroll
        for (int j = 0; j < C::WTN; ++j)
          acc.v[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(a[q][i], e), f4get(b[q][j], e), acc.v[i][j], 0, 0, 0);
}
template <class C, class LA, class LB>
__device__ __forceinline__ void mainloop_all(const LA& la, const LB& lb, int m0, int n0, int K, Acc<C>& acc, float* smem) {
  float* As = smem;
  float* Bs = smem + 2 * C::A_STAGE;
  const int nkt = K / C::BK;
  float4 ra[C::A_F4], rb[C::B_F4];
  fetch_tile<C::BM, C::A_F4, C::NTH, C::A_KC, C::BK>(la, m0, 0, ra);
  fetch_tile<C::BN, C::B_F4, C::NTH, C::B_KC, C::BK>(lb, n0, 0, rb);
  store_tile<C::BM, C::LDA, C::A_F4, C::NTH, C::A_KC, C::BK>(As, ra);
  store_tile<C::BN, C::LDB, C::B_F4, C::NTH, C::B_KC, C::BK>(Bs, rb);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nkt;
    if (more) {
      fetch_tile<C::BM, C::A_F4, C::NTH, C::A_KC, C::BK>(la, m0, (kt + 1) * C::BK, ra);
      fetch_tile<C::BN, C::B_F4, C::NTH, C::B_KC, C::BK>(lb, n0, (kt + 1) * C::BK, rb);
    }
    __builtin_amdgcn_s_setprio(1);
    mma_tile_all<C>(As + cur * C::A_STAGE, Bs + cur * C::B_STAGE, acc);
    __builtin_amdgcn_s_setprio(0);
    if (more) {
      store_tile<C::BM, C::LDA, C::A_F4, C::NTH, C::A_KC, C::BK>(As + (cur ^ 1) * C::A_STAGE, ra);
      store_tile<C::BN, C::LDB, C::B_F4, C::NTH, C::B_KC, C::BK>(Bs + (cur ^ 1) * C::B_STAGE, rb);
    }
    __syncthreads();
  }
}
// Variant core: 3-stage LDS ring. Tile k+1 is in LDS one barrier before tile k's MFMAs start, so
// its fragments are read into a second register set under tile k's MFMAs; the global loads of
// tile k+3 are in flight under them as well. One barrier per K-tile.
template <class C>
struct Frags {
  float4 a[C::BK / 8][C::WTM], b[C::BK / 8][C::WTN];
};
template <class C>
__device__ __forceinline__ void read_frags(const float* as, const float* bs, Frags<C>& f) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / C::WAVES_N, wn = wave % C::WAVES_N;
  const int arow = wm * (C::WTM * 32) + (lane & 31);
  const int brow = wn * (C::WTN * 32) + (lane & 31);
  const int h = lane >> 5;
#pragma unroll
  for (int q = 0; q < C::BK / 8; ++q) {
#pragma unroll
    for (int i = 0; i < C::WTM; ++i) f.a[q][i] = frag4<C::A_KC, C::LDA, C::BK>(as, arow + 32 * i, h, q);
#pragma unroll
    for (int j = 0; j < C::WTN; ++j) f.b[q][j] = frag4<C::B_KC, C::LDB, C::BK>(bs, brow + 32 * j, h, q);
  }
}
template <class C>
__device__ __forceinline__ void mma_frags(const Frags<C>& f, Acc<C>& acc) {
#pragma unroll
  for (int q = 0; q < C::BK / 8; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int i = 0; i < C::WTM; ++i)
#pragma unroll
        for (int j = 0; j < C::WTN; ++j)
          acc.v[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(f.a[q][i], e), f4get(f.b[q][j], e), acc.v[i][j], 0, 0, 0);
}
template <class C, class LA, class LB>
__device__ __forceinline__ void mainloop_ring3(const LA& la, const LB& lb, int m0, int n0, int K, Acc<C>& acc,
                                               float* smem) {
  float* As = smem;
  float* Bs = smem + 3 * C::A_STAGE;
  const int nkt = K / C::BK;
  float4 ra[C::A_F4], rb[C::B_F4];
  auto fetch = [&](int kt) {
    fetch_tile<C::BM, C::A_F4, C::NTH, C::A_KC, C::BK>(la, m0, kt * C::BK, ra);
    fetch_tile<C::BN, C::B_F4, C::NTH, C::B_KC, C::BK>(lb, n0, kt * C::BK, rb);
  };
  auto store = [&](int st) {
    store_tile<C::BM, C::LDA, C::A_F4, C::NTH, C::A_KC, C::BK>(As + st * C::A_STAGE, ra);
    store_tile<C::BN, C::LDB, C::B_F4, C::NTH, C::B_KC, C::BK>(Bs + st * C::B_STAGE, rb);
  };
  fetch(0);
  store(0);
  if (nkt > 1) {
    fetch(1);
    store(1);
  }
  __syncthreads();
  Frags<C> f0, f1;
  read_frags<C>(As, Bs, f0);
  if (nkt > 2) fetch(2);
  for (int kt = 0; kt < nkt; kt += 2) {
    // even step: MFMAs on f0 (tile kt), fragments of tile kt+1 into f1
    if (kt + 1 < nkt) read_frags<C>(As + ((kt + 1) % 3) * C::A_STAGE, Bs + ((kt + 1) % 3) * C::B_STAGE, f1);
    __builtin_amdgcn_s_setprio(1);
    mma_frags<C>(f0, acc);
    __builtin_amdgcn_s_setprio(0);
    if (kt + 2 < nkt) {
      store((kt + 2) % 3);
      if (kt + 3 < nkt) fetch(kt + 3);
    }
    __syncthreads();
    if (kt + 1 >= nkt) break;
    // odd step: MFMAs on f1 (tile kt+1), fragments of tile kt+2 into f0
    if (kt + 2 < nkt) read_frags<C>(As + ((kt + 2) % 3) * C::A_STAGE, Bs + ((kt + 2) % 3) * C::B_STAGE, f0);
    __builtin_amdgcn_s_setprio(1);
    mma_frags<C>(f1, acc);
    __builtin_amdgcn_s_setprio(0);
    if (kt + 3 < nkt) {
      store((kt + 3) % 3);
      if (kt + 4 < nkt) fetch(kt + 4);
    }
    __syncthreads();
  }
}
template <class C>
__global__ __launch_bounds__(C::NTH) void k_ring(const float* A, const float* B, float* O, int M, int N, int K) {
  __shared__ float smem[3 * (C::A_STAGE + C::B_STAGE)];
  const int m0 = blockIdx.x * C::BM, n0 = blockIdx.y * C::BN;
  Acc<C> acc;
  acc.zero();
  RowMajorKC la{A, M, K};
  RowMajorMC lb{B, K, N};
  mainloop_ring3<C>(la, lb, m0, n0, K, acc, smem);
  const int c = n0 + acc_col<C>(0);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < C::WTM; ++i)
#pragma unroll
    for (int j = 0; j < C::WTN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) s += acc.v[i][j][r];
  O[(int64_t)blockIdx.x * C::NTH + threadIdx.x] = s + c;
}
template <class C>
void run_ring(const char* name, const float* A, const float* B, float* O, int M, int N, int K) {
  dim3 grid(M / C::BM, N / C::BN);
  for (int i = 0; i < 3; ++i) k_ring<C><<<grid, C::NTH>>>(A, B, O, M, N, K);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) k_ring<C><<<grid, C::NTH>>>(A, B, O, M, N, K);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  const double tf = 2.0 * M * N * K * reps / (ms * 1e-3) / 1e12;
  printf("%-36s %8.1f us  %6.1f TF/s\n", name, ms * 1e3 / reps, tf);
}

// Variant core: direct-to-LDS loads (global_load_lds_dwordx4) into a 3-stage ring with a counted
// vmcnt across raw barriers, for the 64 x 128 BPTT tile (4 waves). A (k-contiguous rows of 16
// floats) is stored unpadded with the 16-B chunks XOR-swizzled by (row >> 1) & 3 through the
// SOURCE address (a glds wave-instruction writes lane-linear LDS); B rows (128 floats) unpadded.
typedef __attribute__((address_space(3))) void lds_void_m;
typedef __attribute__((address_space(1))) const void gbl_void_m;
__device__ __forceinline__ void glds16m(const float* g, float* l) {
  __builtin_amdgcn_global_load_lds((gbl_void_m*)g, (lds_void_m*)l, 16, 0, 0);
}
__device__ __forceinline__ void bptt_issue(const float* A, const float* B, int lda, int ldb, int m0, int n0, int k0,
                                           float* As, float* Bs) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  {  // A: wave w -> rows 16w .. 16w+15 (lane: row 16w + lane/4, LDS chunk lane%4)
    const int row = 16 * w + (lane >> 2), pc = lane & 3, lc = pc ^ ((row >> 1) & 3);
    glds16m(A + (int64_t)(m0 + row) * lda + k0 + 4 * lc, As + 16 * w * 16);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // B: wave w -> k-rows 4w + 2i, +1
    const int kr = 4 * w + 2 * i + (lane >> 5);
    glds16m(B + (int64_t)(k0 + kr) * ldb + n0 + 4 * (lane & 31), Bs + (4 * w + 2 * i) * 128);
  }
}
template <class C>
__device__ __forceinline__ void bptt_mma(const float* as, const float* bs, Acc<C>& acc) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / C::WAVES_N, wn = wave % C::WAVES_N;
  const int arow = wm * (C::WTM * 32) + (lane & 31);
  const int brow = wn * (C::WTN * 32) + (lane & 31);
  const int h = lane >> 5;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    float4 a[C::WTM], b[C::WTN];
#pragma unroll
    for (int i = 0; i < C::WTM; ++i) {
      const int row = arow + 32 * i, pc = (2 * h + q) ^ ((row >> 1) & 3);
      a[i] = *reinterpret_cast<const float4*>(as + row * 16 + 4 * pc);
    }
#pragma unroll
    for (int j = 0; j < C::WTN; ++j) {
      const float* p = bs + (8 * h + 4 * q) * 128 + brow + 32 * j;
      b[j] = make_float4(p[0], p[128], p[256], p[384]);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int i = 0; i < C::WTM; ++i)
#pragma unroll
        for (int j = 0; j < C::WTN; ++j)
          acc.v[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(a[i], e), f4get(b[j], e), acc.v[i][j], 0, 0, 0);
  }
}
template <class C>
__global__ __launch_bounds__(C::NTH) void k_gldsb(const float* A, const float* B, float* O, int M, int N, int K) {
  static_assert(C::BM == 64 && C::BN == 128 && C::NTH == 256 && C::BK == 16, "BPTT tile");
  __shared__ float smem[3 * (64 * 16 + 16 * 128)];
  float* As = smem;
  float* Bs = smem + 3 * 64 * 16;
  const int m0 = blockIdx.x * C::BM, n0 = blockIdx.y * C::BN;
  Acc<C> acc;
  acc.zero();
  const int nkt = K / 16;
  bptt_issue(A, B, K, N, m0, n0, 0, As, Bs);
  bptt_issue(A, B, K, N, m0, n0, 16, As + 1024, Bs + 2048);
  for (int kt = 0; kt < nkt; ++kt) {
    if (kt + 1 < nkt)
      asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    const int st = kt % 3;
    if (kt + 2 < nkt) {
      const int s2 = (kt + 2) % 3;
      bptt_issue(A, B, K, N, m0, n0, (kt + 2) * 16, As + s2 * 1024, Bs + s2 * 2048);
    }
    __builtin_amdgcn_s_setprio(1);
    bptt_mma<C>(As + st * 1024, Bs + st * 2048, acc);
    __builtin_amdgcn_s_setprio(0);
  }
  const int c = n0 + acc_col<C>(0);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < C::WTM; ++i)
#pragma unroll
    for (int j = 0; j < C::WTN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) s += acc.v[i][j][r];
  O[(int64_t)blockIdx.x * C::NTH + threadIdx.x] = s + c;
}
template <class C>
void run_gldsb(const char* name, const float* A, const float* B, float* O, int M, int N, int K) {
  dim3 grid(M / C::BM, N / C::BN);
  for (int i = 0; i < 3; ++i) k_gldsb<C><<<grid, C::NTH>>>(A, B, O, M, N, K);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) k_gldsb<C><<<grid, C::NTH>>>(A, B, O, M, N, K);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  const double tf = 2.0 * M * N * K * reps / (ms * 1e-3) / 1e12;
  printf("%-36s %8.1f us  %6.1f TF/s\n", name, ms * 1e3 / reps, tf);
}

// 256 x 128 tile, 8 waves of 32 x 128 (8 x 1), direct-to-LDS 3-stage ring (72 KB: two
// workgroups per CU): A rows swizzled as in k_gldsb, B rows unpadded.
__device__ __forceinline__ void bptt_issue256(const float* A, const float* B, int lda, int ldb, int m0, int n0, int k0,
                                              float* As, float* Bs) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // A: 16 instructions of 16 rows; wave w -> row blocks 2w, 2w+1
    const int rb = 2 * w + i;
    const int row = 16 * rb + (lane >> 2), pc = lane & 3, lc = pc ^ ((row >> 1) & 3);
    glds16m(A + (int64_t)(m0 + row) * lda + k0 + 4 * lc, As + rb * 256);
  }
  const int kr = 2 * w + (lane >> 5);  // B: 8 instructions of 2 rows; wave w -> rows 2w, 2w+1
  glds16m(B + (int64_t)(k0 + kr) * ldb + n0 + 4 * (lane & 31), Bs + 2 * w * 128);
}
__global__ __launch_bounds__(512) void k_gldsb256(const float* A, const float* B, float* O, int M, int N, int K) {
  using C = GemmCfg<256, 128, 8, 1, true, false, 16>;
  __shared__ float smem[3 * (256 * 16 + 16 * 128)];
  float* As = smem;
  float* Bs = smem + 3 * 256 * 16;
  const int m0 = blockIdx.x * 256, n0 = blockIdx.y * 128;
  Acc<C> acc;
  acc.zero();
  const int nkt = K / 16;
  bptt_issue256(A, B, K, N, m0, n0, 0, As, Bs);
  bptt_issue256(A, B, K, N, m0, n0, 16, As + 4096, Bs + 2048);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int arow = wave * 32 + (lane & 31), h = lane >> 5;
  for (int kt = 0; kt < nkt; ++kt) {
    if (kt + 1 < nkt)
      asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    const int st = kt % 3;
    if (kt + 2 < nkt) {
      const int s2 = (kt + 2) % 3;
      bptt_issue256(A, B, K, N, m0, n0, (kt + 2) * 16, As + s2 * 4096, Bs + s2 * 2048);
    }
    const float* as = As + st * 4096;
    const float* bs = Bs + st * 2048;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int pc = (2 * h + q) ^ ((arow >> 1) & 3);
      const float4 a = *reinterpret_cast<const float4*>(as + arow * 16 + 4 * pc);
      float4 b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float* p = bs + (8 * h + 4 * q) * 128 + 32 * j + (lane & 31);
        b[j] = make_float4(p[0], p[128], p[256], p[384]);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc.v[0][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(a, e), f4get(b[j], e), acc.v[0][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  }
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) sum += acc.v[0][j][r];
  O[(int64_t)blockIdx.x * 512 + threadIdx.x] = sum;
}
void run_gldsb256(const char* name, const float* A, const float* B, float* O, int M, int N, int K) {
  dim3 grid(M / 256, N / 128);
  for (int i = 0; i < 3; ++i) k_gldsb256<<<grid, 512>>>(A, B, O, M, N, K);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) k_gldsb256<<<grid, 512>>>(A, B, O, M, N, K);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  const double tf = 2.0 * M * N * K * reps / (ms * 1e-3) / 1e12;
  printf("%-36s %8.1f us  %6.1f TF/s\n", name, ms * 1e3 / reps, tf);
}

template <class C>
__global__ __launch_bounds__(C::NTH) void k_all(const float* A, const float* B, float* O, int M, int N, int K) {
  __shared__ float smem[C::SMEM_FLOATS];
  const int m0 = blockIdx.x * C::BM, n0 = blockIdx.y * C::BN;
  Acc<C> acc;
  acc.zero();
  RowMajorKC la{A, M, K};
  RowMajorMC lb{B, K, N};
  mainloop_all<C>(la, lb, m0, n0, K, acc, smem);
  const int c = n0 + acc_col<C>(0);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < C::WTM; ++i)
#pragma unroll
    for (int j = 0; j < C::WTN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) s += acc.v[i][j][r];
  O[(int64_t)blockIdx.x * C::NTH + threadIdx.x] = s + c;
}
template <class C>
void run_all(const char* name, const float* A, const float* B, float* O, int M, int N, int K) {
  dim3 grid(M / C::BM, N / C::BN);
  for (int i = 0; i < 3; ++i) k_all<C><<<grid, C::NTH>>>(A, B, O, M, N, K);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) k_all<C><<<grid, C::NTH>>>(A, B, O, M, N, K);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  const double tf = 2.0 * M * N * K * reps / (ms * 1e-3) / 1e12;
  printf("%-36s %8.1f us  %6.1f TF/s\n", name, ms * 1e3 / reps, tf);
}

template <class C, bool MC>
__global__ __launch_bounds__(C::NTH) void k_b(const float* A, const float* B, float* O, int M, int N, int K) {
  __shared__ float smem[C::SMEM_FLOATS];
  const int m0 = blockIdx.x * C::BM, n0 = blockIdx.y * C::BN;
  Acc<C> acc;
  acc.zero();
  RowMajorKC la{A, M, K};
  if constexpr (MC) {
    RowMajorMC lb{B, K, N};
    gemm_mainloop<C>(la, lb, m0, n0, 0, K, acc, smem);
  } else {
    RowMajorKC lb{B, N, K};
    gemm_mainloop<C>(la, lb, m0, n0, 0, K, acc, smem);
  }
  const int c = n0 + acc_col<C>(0);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < C::WTM; ++i)
#pragma unroll
    for (int j = 0; j < C::WTN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) s += acc.v[i][j][r];
  O[(int64_t)blockIdx.x * C::NTH + threadIdx.x] = s + c;
}

template <class C, bool MC>
void run(const char* name, const float* A, const float* B, float* O, int M, int N, int K) {
  dim3 grid(M / C::BM, N / C::BN);
  for (int i = 0; i < 3; ++i) k_b<C, MC><<<grid, C::NTH>>>(A, B, O, M, N, K);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) k_b<C, MC><<<grid, C::NTH>>>(A, B, O, M, N, K);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  const double tf = 2.0 * M * N * K * reps / (ms * 1e-3) / 1e12;
  printf("%-36s %8.1f us  %6.1f TF/s\n", name, ms * 1e3 / reps, tf);
}

int main() {
  const int M = 64 * 221 * 15, N = 128, K = 1024;
  const int Mmax = 64 * 128 * 40;  // the largest row count run below (4 rounds)
  float *A, *B, *O;
  hipMalloc(&A, (size_t)Mmax * K * 4);
  hipMalloc(&B, (size_t)N * K * 4);
  hipMalloc(&O, (size_t)Mmax * 256 * 4);
  std::vector<float> h((size_t)Mmax * K);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  hipMemcpy(A, h.data(), (size_t)Mmax * K * 4, hipMemcpyHostToDevice);
  hipMemcpy(B, h.data(), (size_t)N * K * 4, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; ++rep) {
    run_gldsb256("256x128 w8x1 BK16 glds ring3", A, B, O, M, N, K);
    run_gldsb256("256x128 w8x1 glds, 2.0 rounds", A, B, O, 256 * 256 * 2 * 2, N, K);
    run_gldsb<GemmCfg<64, 128, 2, 2, true, false, 16>>("64x128 w2x2 BK16  glds ring3", A, B, O, M, N, K);
    run<GemmCfg<64, 128, 2, 2, true, false, 16>, true>("64x128 w2x2 BK16  B MC (current)", A, B, O, M, N, K);
  }
  for (int rep = 0; rep < 3; ++rep) {
    run_ring<GemmCfg<64, 128, 2, 2, true, false, 16>>("64x128 w2x2 BK16  ring3", A, B, O, M, N, K);
    run_ring<GemmCfg<64, 128, 2, 2, true, false, 32>>("64x128 w2x2 BK32  ring3", A, B, O, M, N, K);
    run_ring<GemmCfg<128, 128, 4, 1, true, false, 16>>("128x128 w4x1 BK16 ring3", A, B, O, M, N, K);
    run<GemmCfg<64, 128, 2, 2, true, false, 16>, true>("64x128 w2x2 BK16  B MC (current)", A, B, O, M, N, K);
  }
  for (int rep = 0; rep < 2; ++rep) {
    run<GemmCfg<64, 128, 2, 2, true, false, 16>, true>("64x128 w2x2 BK16  B MC (current)", A, B, O, M, N, K);
    run_all<GemmCfg<64, 128, 2, 2, true, false, 16>>("64x128 w2x2 BK16  MC frags-first", A, B, O, M, N, K);
    run<GemmCfg<128, 128, 4, 2, true, false, 16>, true>("128x128 w4x2 BK16 B MC", A, B, O, M, N, K);
  }
  for (int rep = 0; rep < 2; ++rep) {  // larger wave tiles (64 x 128 per wave = 8 MFMA blocks, as k_wgrad)
    run<GemmCfg<256, 128, 4, 1, true, false, 16>, true>("256x128 w4x1 BK16 B MC", A, B, O, M, N, K);
    run<GemmCfg<512, 128, 8, 1, true, false, 16>, true>("512x128 w8x1 BK16 B MC", A, B, O, M, N, K);
    run<GemmCfg<256, 128, 4, 1, true, true, 16>, false>("256x128 w4x1 BK16 B KC", A, B, O, M, N, K);
    run<GemmCfg<128, 128, 2, 1, true, false, 16>, true>("128x128 w2x1 BK16 B MC", A, B, O, M, N, K);
  }
  // workgroup-round quantization: 5 resident 64x128 workgroups per CU -> 1280 per round
  for (int rounds10 : {10, 20, 25, 26, 30, 35, 40}) {
    const int Mr = 64 * 128 * rounds10;  // rounds10 / 10 rounds of 1280 workgroups
    char name[64];
    snprintf(name, sizeof name, "64x128 current, %.1f rounds", rounds10 / 10.0);
    run<GemmCfg<64, 128, 2, 2, true, false, 16>, true>(name, A, B, O, Mr, N, K);
  }
  return 0;
}
