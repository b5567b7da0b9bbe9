// fp32 MFMA GEMM core for gfx950 (CDNA4).
//
// All GEMM-shaped work on the STGCN-LSTM path goes through this mainloop with
// v_mfma_f32_32x32x2_f32 (exact f32 in / f32 accumulate, the f32 MFMA peak rate).
//   * A tile [BK][BM] and B tile [BK][BN] live in LDS k-major (m / n contiguous), so
//     a wave's fragment read (lane l -> row l&31, k = 2s + (l>>5)) is one
//     conflict-free ds_read_b32 per operand per k-step.
//   * Operands are staged global -> registers (float4 per lane) -> LDS, double
//     buffered with one barrier per K-tile: the global loads of tile k+1 are in flight
//     while the MFMAs of tile k issue.
//   * Loader functors describe where operand elements live: "KC" operands are
//     row-major with k contiguous (float4 along k, transposed on the LDS write);
//     "MC" operands have the row (m or n) contiguous (float4 along m, one vector
//     LDS write). Loaders return zeros outside the logical matrix.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smaml {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32;
constexpr int NT = 256;  // threads per workgroup (4 waves of 64)

__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

__device__ __forceinline__ float4 fma4(float w, float4 a, float4 acc) {
  acc.x = fmaf(w, a.x, acc.x);
  acc.y = fmaf(w, a.y, acc.y);
  acc.z = fmaf(w, a.z, acc.z);
  acc.w = fmaf(w, a.w, acc.w);
  return acc;
}

template <int BM_, int BN_, int WAVES_M_, int WAVES_N_, bool A_KC_, bool B_KC_>
struct GemmCfg {
  static constexpr int BM = BM_;
  static constexpr int BN = BN_;
  static constexpr int WAVES_M = WAVES_M_;
  static constexpr int WAVES_N = WAVES_N_;
  static constexpr bool A_KC = A_KC_;
  static constexpr bool B_KC = B_KC_;
  static_assert(WAVES_M * WAVES_N * 64 == NT, "4 waves per workgroup");
  static constexpr int WTM = BM / (WAVES_M * 32);  // 32x32 tiles per wave along M
  static constexpr int WTN = BN / (WAVES_N * 32);
  static_assert(WTM >= 1 && WTN >= 1, "wave tile");
  // KC operands are written transposed with ds_write_b32: a +1 pad makes the 32-lane
  // halves conflict-free. MC operands are written with ds_write_b128: keep 16-B rows.
  static constexpr int LDA = BM + (A_KC ? 1 : 4);
  static constexpr int LDB = BN + (B_KC ? 1 : 4);
  static constexpr int A_F4 = BM * BK / 4 / NT;
  static constexpr int B_F4 = BN * BK / 4 / NT;
  static_assert(A_F4 * 4 * NT == BM * BK && B_F4 * 4 * NT == BN * BK, "tile/threads");
  static constexpr int A_STAGE = BK * LDA;
  static constexpr int B_STAGE = BK * LDB;
  static constexpr int SMEM_FLOATS = 2 * (A_STAGE + B_STAGE);
};

// Fetch this thread's share of one operand tile into registers.
// KC: element (row r, k) ; MC: element (k, row r).  `row0`, `k0` absolute.
template <int ROWS, int F4, bool KC, class L>
__device__ __forceinline__ void fetch_tile(const L& ld, int row0, int k0, float4 (&r)[F4]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < F4; ++i) {
    const int f = tid + NT * i;
    if (KC) {
      const int rr = f / (BK / 4), q = f % (BK / 4);
      r[i] = ld(row0 + rr, k0 + 4 * q);
    } else {
      const int kk = f / (ROWS / 4), q = f % (ROWS / 4);
      r[i] = ld(k0 + kk, row0 + 4 * q);
    }
  }
}

template <int ROWS, int LD, int F4, bool KC>
__device__ __forceinline__ void store_tile(float* s, const float4 (&r)[F4]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < F4; ++i) {
    const int f = tid + NT * i;
    if (KC) {
      const int rr = f / (BK / 4), q = f % (BK / 4);
      float* p = s + (4 * q) * LD + rr;
      p[0] = r[i].x;
      p[LD] = r[i].y;
      p[2 * LD] = r[i].z;
      p[3 * LD] = r[i].w;
    } else {
      const int kk = f / (ROWS / 4), q = f % (ROWS / 4);
      st4(s + kk * LD + 4 * q, r[i]);
    }
  }
}

template <class C>
struct Acc {
  f32x16 v[C::WTM][C::WTN];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < C::WTM; ++i)
#pragma unroll
      for (int j = 0; j < C::WTN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) v[i][j][r] = 0.f;
  }
};

// Row / column of accumulator register r of tile (i, j) for this lane.
template <class C>
__device__ __forceinline__ int acc_row(int i, int r) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / C::WAVES_N;
  return wm * (C::WTM * 32) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
}
template <class C>
__device__ __forceinline__ int acc_col(int j) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wn = wave % C::WAVES_N;
  return wn * (C::WTN * 32) + j * 32 + (lane & 31);
}

// Optional per-K-tile hook run on the staged A tile (e.g. column sums for bias grads).
struct NoHook {
  __device__ __forceinline__ void operator()(const float*, int) const {}
};

// acc += sum_{k in [kbeg,kend)} A[m0+., k] * B[n0+., k]
template <class C, class LA, class LB, class Hook = NoHook>
__device__ __forceinline__ void gemm_mainloop(const LA& la, const LB& lb, int m0, int n0, int kbeg,
                                              int kend, Acc<C>& acc, float* smem,
                                              const Hook& hook = Hook()) {
  float* As = smem;
  float* Bs = smem + 2 * C::A_STAGE;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / C::WAVES_N, wn = wave % C::WAVES_N;
  const int a_off = wm * (C::WTM * 32) + (lane & 31);
  const int b_off = wn * (C::WTN * 32) + (lane & 31);
  const int khalf = lane >> 5;
  const int nkt = (kend - kbeg + BK - 1) / BK;
  if (nkt <= 0) return;

  float4 ra[C::A_F4], rb[C::B_F4];
  fetch_tile<C::BM, C::A_F4, C::A_KC>(la, m0, kbeg, ra);
  fetch_tile<C::BN, C::B_F4, C::B_KC>(lb, n0, kbeg, rb);
  store_tile<C::BM, C::LDA, C::A_F4, C::A_KC>(As, ra);
  store_tile<C::BN, C::LDB, C::B_F4, C::B_KC>(Bs, rb);
  __syncthreads();

  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nkt;
    if (more) {
      fetch_tile<C::BM, C::A_F4, C::A_KC>(la, m0, kbeg + (kt + 1) * BK, ra);
      fetch_tile<C::BN, C::B_F4, C::B_KC>(lb, n0, kbeg + (kt + 1) * BK, rb);
    }
    const float* as = As + cur * C::A_STAGE;
    const float* bs = Bs + cur * C::B_STAGE;
    hook(as, kt);
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
      const int kr = 2 * s + khalf;
      float a[C::WTM], b[C::WTN];
#pragma unroll
      for (int i = 0; i < C::WTM; ++i) a[i] = as[kr * C::LDA + a_off + 32 * i];
#pragma unroll
      for (int j = 0; j < C::WTN; ++j) b[j] = bs[kr * C::LDB + b_off + 32 * j];
#pragma unroll
      for (int i = 0; i < C::WTM; ++i)
#pragma unroll
        for (int j = 0; j < C::WTN; ++j)
          acc.v[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc.v[i][j], 0, 0, 0);
    }
    if (more) {
      store_tile<C::BM, C::LDA, C::A_F4, C::A_KC>(As + (cur ^ 1) * C::A_STAGE, ra);
      store_tile<C::BN, C::LDB, C::B_F4, C::B_KC>(Bs + (cur ^ 1) * C::B_STAGE, rb);
    }
    __syncthreads();
  }
}

}  // namespace smaml
