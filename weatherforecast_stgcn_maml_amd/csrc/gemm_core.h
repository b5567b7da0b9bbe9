// fp32 MFMA GEMM core for gfx950 (CDNA4).
//
// All GEMM-shaped work on the STGCN-LSTM path goes through this mainloop with
// v_mfma_f32_32x32x2_f32 (exact f32 in / f32 accumulate, the f32 MFMA peak rate).
//
// K order: inside a BK=32 tile, MFMA k-step s (0..15) of lane half h (= lane>>5) covers
// k = 16h + s, so one lane's 16 k-values of a row are contiguous: a k-contiguous ("KC")
// operand is kept row-major in LDS ([rows][BK+4], written with ds_write_b128) and each
// lane fetches 4 k-steps of a fragment with ONE conflict-free ds_read_b128 (row stride 36
// floats puts the 16 rows of every ds_read_b128 lane group on distinct 4-bank slots).
// An "MC" operand (rows contiguous, e.g. W_hh used as [k][n]) is kept k-major in LDS
// ([BK][rows+4], ds_write_b128) and read with ds_read_b32 (lanes read consecutive rows).
//
// Staging: global -> registers (float4 per lane) -> LDS, double buffered with one barrier
// per K-tile, so the global loads of tile k+1 are in flight while tile k's MFMAs issue.
// Loader functors describe where operand elements live and return zeros outside the
// logical matrix (see loaders.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace smaml {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32;  // default K-tile (GemmCfg's BK_ parameter)
#ifndef SMAML_PRIO
#define SMAML_PRIO 1  // raise the wave priority around the MFMA phase of each K-tile (A/B: -0.5 %)
#endif
#ifndef SMAML_IGLP
#define SMAML_IGLP 1  // LLVM iglp_opt DS/MFMA interleave strategy for the mainloops that ask for it
#endif                // (IG template argument; A/B: fwd_dual -7, wgrad -7, GCN -2 ms; the primal
                      // gate / BPTT / dual-BPTT loops are slower with it and keep the default order)
constexpr int NT = 256;  // threads per workgroup of the 4-wave configurations

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

__device__ __forceinline__ float f4get(const float4& v, int e) {
  return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w;
}

template <int BM_, int BN_, int WAVES_M_, int WAVES_N_, bool A_KC_, bool B_KC_, int BK_ = 32>
struct GemmCfg {
  static constexpr int BK = BK_;
  static_assert(BK % 16 == 0, "BK multiple of 16");
  static constexpr int BM = BM_;
  static constexpr int BN = BN_;
  static constexpr int WAVES_M = WAVES_M_;
  static constexpr int WAVES_N = WAVES_N_;
  static constexpr int NTH = WAVES_M * WAVES_N * 64;
  static constexpr bool A_KC = A_KC_;
  static constexpr bool B_KC = B_KC_;
  static constexpr int WTM = BM / (WAVES_M * 32);  // 32x32 tiles per wave along M
  static constexpr int WTN = BN / (WAVES_N * 32);
  static_assert(WTM >= 1 && WTN >= 1, "wave tile");
  // KC: row-major [rows][BK+4]; MC: k-major [BK][rows+4]
  static constexpr int LDA = A_KC ? BK + 4 : BM + 4;  // (BK+4) row stride: conflict-free ds_read_b128
  static constexpr int LDB = B_KC ? BK + 4 : BN + 4;
  static constexpr int A_STAGE = A_KC ? BM * LDA : BK * LDA;
  static constexpr int B_STAGE = B_KC ? BN * LDB : BK * LDB;
  static constexpr int A_F4 = BM * BK / 4 / NTH;
  static constexpr int B_F4 = BN * BK / 4 / NTH;
  static_assert(A_F4 * 4 * NTH == BM * BK && B_F4 * 4 * NTH == BN * BK, "tile/threads");
  static constexpr int SMEM_FLOATS = 2 * (A_STAGE + B_STAGE);
};

// Loaders that fetch a whole operand tile themselves (``kTileFetch``; loaders.h "tile
// loaders"): the K-tile's segment is chosen once per tile (uniform), rows are clamped instead of
// zero-filled, so the loads compile to branch-free saddr + vgpr-offset loads.
template <class L, class = void>
struct has_tile_fetch : std::false_type {};
template <class L>
struct has_tile_fetch<L, std::void_t<decltype(L::kTileFetch)>> : std::true_type {};

// Fetch this thread's share of one operand tile into registers.
// KC: element (row r, k) ; MC: element (k, row r).  `row0`, `k0` absolute.
template <int ROWS, int F4, int NTH, bool KC, int BK, class L>
__device__ __forceinline__ void fetch_tile(const L& ld, int row0, int k0, float4 (&r)[F4]) {
  if constexpr (has_tile_fetch<L>::value) {
    ld.template fetch<ROWS, F4, NTH, KC, BK>(row0, k0, r);
  } else {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < F4; ++i) {
      const int f = tid + NTH * i;
      if (KC) {
        const int rr = f / (BK / 4), q = f % (BK / 4);
        r[i] = ld(row0 + rr, k0 + 4 * q);
      } else {
        const int kk = f / (ROWS / 4), q = f % (ROWS / 4);
        r[i] = ld(k0 + kk, row0 + 4 * q);
      }
    }
  }
}

template <int ROWS, int LD, int F4, int NTH, bool KC, int BK>
__device__ __forceinline__ void store_tile(float* s, const float4 (&r)[F4]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < F4; ++i) {
    const int f = tid + NTH * i;
    if (KC) {
      const int rr = f / (BK / 4), q = f % (BK / 4);
      st4(s + rr * LD + 4 * q, r[i]);
    } else {
      const int kk = f / (ROWS / 4), q = f % (ROWS / 4);
      st4(s + kk * LD + 4 * q, r[i]);
    }
  }
}

// 4 consecutive k-steps (4q .. 4q+3 of lane half h) of a 32-row fragment at tile row `row`.
template <bool KC, int LD, int BK>
__device__ __forceinline__ float4 frag4(const float* s, int row, int h, int q) {
  if (KC) return *reinterpret_cast<const float4*>(s + row * LD + (BK / 2) * h + 4 * q);
  const float* p = s + ((BK / 2) * h + 4 * q) * LD + row;
  return make_float4(p[0], p[LD], p[2 * LD], p[3 * LD]);
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

// Optional hooks: operator() runs once per K-tile on the staged A tile; afrag(i, a) sees every
// A fragment this lane feeds to the MFMAs (4 k-steps of tile row i), e.g. for column sums
// of A (bias gradients) kept in registers instead of re-read from LDS.
struct NoHook {
  __device__ __forceinline__ void operator()(const float*, int) const {}
  __device__ __forceinline__ void afrag(int, const float4&) {}
};

template <class C, int IG = -1, class Hook = NoHook>
__device__ __forceinline__ void mma_tile(const float* as, const float* bs, Acc<C>& acc, Hook& hook) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / C::WAVES_N, wn = wave % C::WAVES_N;
  const int arow = wm * (C::WTM * 32) + (lane & 31);
  const int brow = wn * (C::WTN * 32) + (lane & 31);
  const int h = lane >> 5;
  if constexpr (IG >= 0) __builtin_amdgcn_iglp_opt(IG);
#pragma unroll
  for (int q = 0; q < C::BK / 8; ++q) {
    float4 a[C::WTM], b[C::WTN];
#pragma unroll
    for (int i = 0; i < C::WTM; ++i) a[i] = frag4<C::A_KC, C::LDA, C::BK>(as, arow + 32 * i, h, q);
#pragma unroll
    for (int j = 0; j < C::WTN; ++j) b[j] = frag4<C::B_KC, C::LDB, C::BK>(bs, brow + 32 * j, h, q);
#pragma unroll
    for (int i = 0; i < C::WTM; ++i) hook.afrag(i, a[i]);
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int i = 0; i < C::WTM; ++i)
#pragma unroll
        for (int j = 0; j < C::WTN; ++j)
          acc.v[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(a[i], e), f4get(b[j], e), acc.v[i][j], 0, 0, 0);
  }
}

// acc += sum_{k in [kbeg,kend)} A[m0+., k] * B[n0+., k]
// IG >= 0: ask LLVM for iglp_opt strategy IG in the MFMA phase (set per call site by A/B).
template <class C, int IG = -1, class LA, class LB, class Hook>
__device__ __forceinline__ void gemm_mainloop(const LA& la, const LB& lb, int m0, int n0, int kbeg,
                                              int kend, Acc<C>& acc, float* smem, Hook& hook) {
  float* As = smem;
  float* Bs = smem + 2 * C::A_STAGE;
  constexpr int BKc = C::BK;
  const int nkt = (kend - kbeg + BKc - 1) / BKc;
  if (nkt <= 0) return;

  float4 ra[C::A_F4], rb[C::B_F4];
  fetch_tile<C::BM, C::A_F4, C::NTH, C::A_KC, BKc>(la, m0, kbeg, ra);
  fetch_tile<C::BN, C::B_F4, C::NTH, C::B_KC, BKc>(lb, n0, kbeg, rb);
  store_tile<C::BM, C::LDA, C::A_F4, C::NTH, C::A_KC, BKc>(As, ra);
  store_tile<C::BN, C::LDB, C::B_F4, C::NTH, C::B_KC, BKc>(Bs, rb);
  __syncthreads();

  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nkt;
    if (more) {
      fetch_tile<C::BM, C::A_F4, C::NTH, C::A_KC, BKc>(la, m0, kbeg + (kt + 1) * BKc, ra);
      fetch_tile<C::BN, C::B_F4, C::NTH, C::B_KC, BKc>(lb, n0, kbeg + (kt + 1) * BKc, rb);
    }
    const float* as = As + cur * C::A_STAGE;
    const float* bs = Bs + cur * C::B_STAGE;
    hook(as, kt);
#if SMAML_PRIO
    __builtin_amdgcn_s_setprio(1);  // MFMA phase first in the SIMD's issue arbitration
#endif
    mma_tile<C, IG>(as, bs, acc, hook);
#if SMAML_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    if (more) {
      store_tile<C::BM, C::LDA, C::A_F4, C::NTH, C::A_KC, BKc>(As + (cur ^ 1) * C::A_STAGE, ra);
      store_tile<C::BN, C::LDB, C::B_F4, C::NTH, C::B_KC, BKc>(Bs + (cur ^ 1) * C::B_STAGE, rb);
    }
    __syncthreads();
  }
}

template <class C, int IG = -1, class LA, class LB>
__device__ __forceinline__ void gemm_mainloop(const LA& la, const LB& lb, int m0, int n0, int kbeg,
                                              int kend, Acc<C>& acc, float* smem) {
  NoHook hook;
  gemm_mainloop<C, IG>(la, lb, m0, n0, kbeg, kend, acc, smem, hook);
}

// Chunked mainloop for short K ranges (the split-K steps of small grids): with one wave per SIMD
// and a handful of K-tiles per workgroup, the double-buffered loop above pays one global-load
// latency per K-tile. Here NCH K-tiles are fetched per round trip (registers), staged into NCH
// LDS slots and then consumed, and chunk c+1's loads are in flight under chunk c's MFMAs.
// LDS: NCH * (A_STAGE + B_STAGE) floats (chunked_smem_floats).
template <class C, int NCH>
constexpr int chunked_smem_floats() {
  return NCH * (C::A_STAGE + C::B_STAGE);
}
template <class C, int NCH, class LA, class LB>
__device__ __forceinline__ void gemm_mainloop_chunked(const LA& la, const LB& lb, int m0, int n0, int kbeg,
                                                      int kend, Acc<C>& acc, float* smem) {
  constexpr int BKc = C::BK;
  float* As = smem;
  float* Bs = smem + NCH * C::A_STAGE;
  const int nkt = (kend - kbeg + BKc - 1) / BKc;
  if (nkt <= 0) return;
  float4 ra[NCH][C::A_F4], rb[NCH][C::B_F4];
  auto fetch = [&](int c0) {
#pragma unroll
    for (int i = 0; i < NCH; ++i)
      if (c0 + i < nkt) {
        fetch_tile<C::BM, C::A_F4, C::NTH, C::A_KC, BKc>(la, m0, kbeg + (c0 + i) * BKc, ra[i]);
        fetch_tile<C::BN, C::B_F4, C::NTH, C::B_KC, BKc>(lb, n0, kbeg + (c0 + i) * BKc, rb[i]);
      }
  };
  fetch(0);
  NoHook hook;
  for (int c0 = 0; c0 < nkt; c0 += NCH) {
    if (c0 > 0) __syncthreads();  // the previous chunk's MFMAs have read their slots
#pragma unroll
    for (int i = 0; i < NCH; ++i)
      if (c0 + i < nkt) {
        store_tile<C::BM, C::LDA, C::A_F4, C::NTH, C::A_KC, BKc>(As + i * C::A_STAGE, ra[i]);
        store_tile<C::BN, C::LDB, C::B_F4, C::NTH, C::B_KC, BKc>(Bs + i * C::B_STAGE, rb[i]);
      }
    __syncthreads();
    if (c0 + NCH < nkt) fetch(c0 + NCH);
#if SMAML_PRIO
    __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
    for (int i = 0; i < NCH; ++i)
      if (c0 + i < nkt) mma_tile<C>(As + i * C::A_STAGE, Bs + i * C::B_STAGE, acc, hook);
#if SMAML_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
  }
}

}  // namespace smaml

namespace smaml {

// Fused primal + tangent mainloop (second-order path):
//   acc_p += A . B            acc_t += A2 . B + A . B2
// over k in [0, K): A, A2 share the A layout/rows, B, B2 the B layout/rows. Per K-tile the
// four operand tiles are staged once (LDS: [A | A2 | B | B2] x 2 stages) and 3 MFMAs issue per
// fragment pair. A2 is known to be zero for k < a2_kbeg (the layer-0 input has no tangent):
// those K-tiles neither load A2 nor issue its MFMAs (a2_kbeg must be a multiple of BK).
template <class C>
struct DualStage {
  static constexpr int FLOATS = 2 * (2 * C::A_STAGE + 2 * C::B_STAGE);
};

template <class C, bool A2, bool PRIMAL = true>
__device__ __forceinline__ void dual_mma(const float* st, int arow, int brow, int h, Acc<C>& accp, Acc<C>& acct) {
  constexpr int BKc = C::BK;
  constexpr int SA = C::A_STAGE, SB = C::B_STAGE;
#pragma unroll
  for (int q = 0; q < BKc / 8; ++q) {
    float4 a[C::WTM], a2[C::WTM], b[C::WTN], b2[C::WTN];
#pragma unroll
    for (int i = 0; i < C::WTM; ++i) {
      a[i] = frag4<C::A_KC, C::LDA, BKc>(st, arow + 32 * i, h, q);
      if (A2) a2[i] = frag4<C::A_KC, C::LDA, BKc>(st + SA, arow + 32 * i, h, q);
    }
#pragma unroll
    for (int j = 0; j < C::WTN; ++j) {
      b[j] = frag4<C::B_KC, C::LDB, BKc>(st + 2 * SA, brow + 32 * j, h, q);
      b2[j] = frag4<C::B_KC, C::LDB, BKc>(st + 2 * SA + SB, brow + 32 * j, h, q);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int i = 0; i < C::WTM; ++i)
#pragma unroll
        for (int j = 0; j < C::WTN; ++j) {
          if (PRIMAL)
            accp.v[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(a[i], e), f4get(b[j], e), accp.v[i][j], 0, 0, 0);
          acct.v[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(a[i], e), f4get(b2[j], e), acct.v[i][j], 0, 0, 0);
          if (A2)
            acct.v[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(a2[i], e), f4get(b[j], e), acct.v[i][j], 0, 0, 0);
        }
  }
}

// PRIMAL = false: tangent only (acc_t += A2 . B + A . B2), acc_p untouched -- the primal
// product is already stored (second-order sweep with the inner step's activations kept).
template <class C, bool PRIMAL = true, class LA, class LA2, class LB, class LB2>
__device__ __forceinline__ void gemm_dual_mainloop(const LA& la, const LA2& la2, const LB& lb, const LB2& lb2,
                                                   int m0, int n0, int K, int a2_kbeg, Acc<C>& accp, Acc<C>& acct,
                                                   float* smem) {
  constexpr int BKc = C::BK;
  constexpr int SA = C::A_STAGE, SB = C::B_STAGE;
  constexpr int STAGE = 2 * SA + 2 * SB;
  const int nkt = (K + BKc - 1) / BKc;
  if (nkt <= 0) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / C::WAVES_N, wn = wave % C::WAVES_N;
  const int arow = wm * (C::WTM * 32) + (lane & 31);
  const int brow = wn * (C::WTN * 32) + (lane & 31);
  const int h = lane >> 5;
  float4 ra[C::A_F4], ra2[C::A_F4], rb[C::B_F4], rb2[C::B_F4];
  auto fetch = [&](int k0) {
    fetch_tile<C::BM, C::A_F4, C::NTH, C::A_KC, BKc>(la, m0, k0, ra);
    if (k0 >= a2_kbeg) fetch_tile<C::BM, C::A_F4, C::NTH, C::A_KC, BKc>(la2, m0, k0, ra2);
    fetch_tile<C::BN, C::B_F4, C::NTH, C::B_KC, BKc>(lb, n0, k0, rb);
    fetch_tile<C::BN, C::B_F4, C::NTH, C::B_KC, BKc>(lb2, n0, k0, rb2);
  };
  auto store = [&](float* st, int k0) {
    store_tile<C::BM, C::LDA, C::A_F4, C::NTH, C::A_KC, BKc>(st, ra);
    if (k0 >= a2_kbeg) store_tile<C::BM, C::LDA, C::A_F4, C::NTH, C::A_KC, BKc>(st + SA, ra2);
    store_tile<C::BN, C::LDB, C::B_F4, C::NTH, C::B_KC, BKc>(st + 2 * SA, rb);
    store_tile<C::BN, C::LDB, C::B_F4, C::NTH, C::B_KC, BKc>(st + 2 * SA + SB, rb2);
  };
  fetch(0);
  store(smem, 0);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    const int k0 = kt * BKc;
    const bool more = kt + 1 < nkt;
    if (more) fetch(k0 + BKc);
    const float* st = smem + cur * STAGE;
#if SMAML_PRIO
    __builtin_amdgcn_s_setprio(1);
#endif
    if (k0 >= a2_kbeg)
      dual_mma<C, true, PRIMAL>(st, arow, brow, h, accp, acct);
    else
      dual_mma<C, false, PRIMAL>(st, arow, brow, h, accp, acct);
#if SMAML_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    if (more) store(smem + (cur ^ 1) * STAGE, k0 + BKc);
    __syncthreads();
  }
}

}  // namespace smaml
