// Operand loaders for gemm_mainloop (gemm_core.h). A loader returns the float4 at a
// logical (row, k) [KC: 4 consecutive k] or (k, col) [MC: 4 consecutive cols] position
// of its operand, zero outside. "Seg" loaders concatenate several matrices along K,
// which is how the fused concatenated-K GEMMs ([x_t | h_{t-1}] . [W_ih | W_hh]^T and the
// tangent GEMMs of the second-order path) are expressed.
#pragma once
#include "gemm_core.h"
#include "kernels.h"

// Product form per GEMM family (gemm_core.h GemmCfg X6_: 1 = f32-accurate bf16x6 on the bf16 MFMA
// pipe, 0 = v_mfma_f32_32x32x2_f32); A/B-able at build time, default SMAML_X6.
#ifndef SMAML_X6_GATE
#define SMAML_X6_GATE (SMAML_X6 ? 2 : 0)  // LSTM forward gate GEMM (primal; staged with 256-row tiles: 268 -> 242 ms)
#endif
#ifndef SMAML_X6_GATED
#define SMAML_X6_GATED (SMAML_X6 ? 2 : 0)  // LSTM forward gate GEMM (primal + tangent; staged, 256-row tiles: 406 -> 385 ms)
#endif
#ifndef SMAML_X6_BWD
#define SMAML_X6_BWD (SMAML_X6 ? 2 : 0)  // BPTT step (primal), head dh_T (staged: A/B 286 -> 273 ms)
#endif
#ifndef SMAML_X6_BWDD
#define SMAML_X6_BWDD (SMAML_X6 ? 2 : 0)  // BPTT step (tangent), head duals (staged, one LDS stage: 423 -> 401 ms)
#endif
#ifndef SMAML_X6_WGRAD
#define SMAML_X6_WGRAD (SMAML_X6 ? 2 : 0)  // LSTM weight gradients (staged split: A/B 622 -> 499 ms)
#endif
#ifndef SMAML_X6_GCN
#define SMAML_X6_GCN (SMAML_X6 ? 2 : 0)  // GCN layers (staged: A/B 128 -> 121 ms)
#endif

// K-tile depth per GEMM family (A/B-able at build time: -DSMAML_GATE_BK=16 ...).
#ifndef SMAML_GATE_BK
#define SMAML_GATE_BK 16
#endif
#ifndef SMAML_GATE_WN
#define SMAML_GATE_WN 1  // gate GEMM column waves: 1 -> 128x128 (4 waves), 2 -> 128x256 (8 waves)
#endif
#ifndef SMAML_GATE_WM
#define SMAML_GATE_WM (SMAML_X6 ? 8 : 4)  // gate GEMM row waves (32 rows each): 4 -> 128-row tiles, 8 -> 256-row tiles
                                          // (staged split: the B tile's split is shared by 256 rows; 2 WGs/CU)
#endif
#ifndef SMAML_GATE_NST
#define SMAML_GATE_NST 2  // gate GEMMs' staged-split LDS stages
#endif
#ifndef SMAML_GATED_WM
#define SMAML_GATED_WM (SMAML_X6 ? 8 : 4)  // same, for the tangent (dual) gate kernel
#endif
#ifndef SMAML_NN_BK
#define SMAML_NN_BK 16
#endif
#ifndef SMAML_BWD_BM
#define SMAML_BWD_BM (SMAML_X6 ? 128 : 64)  // BPTT step tile rows (x 128 units; 2x2 waves of 64x64: with the bf16x6 products
                          // the larger wave tile halves the fragment splits per MFMA; A/B 64 -> 128: bwd 316 -> 278,
                          // tangent bwd 472 -> 429 ms per meta-step)
#endif
// Primal BPTT LDS diet (bf16x6 build): one staged-split LDS stage and the epilogue's transpose in two
// row halves, 64 KB -> 37 KB per workgroup (2 -> 3 workgroups per CU): A/B bwd 256 -> 244 ms.
#ifndef SMAML_BWD_NST
#define SMAML_BWD_NST (SMAML_X6 ? 1 : 2)  // primal BPTT staged-split LDS stages
#endif
#ifndef SMAML_BWD_HALFEPI
#define SMAML_BWD_HALFEPI (SMAML_X6 ? 1 : 0)  // primal BPTT epilogue in two row halves (BM*BN/2 floats of LDS)
#endif
#ifndef SMAML_BWD_WM
#define SMAML_BWD_WM 2
#endif
#ifndef SMAML_BWD_WN
#define SMAML_BWD_WN 2
#endif
#ifndef SMAML_GCN_BK
#define SMAML_GCN_BK (SMAML_X6 ? 32 : 16)  // (staged split: BK 32 measured 119 -> 116 ms)
#endif
// weight-gradient tile (BM x BN), waves WM x WN: all 4H = 512 gate rows of a layer in one
// tile (8 waves of 64 x 128), so the split-K slices read each [x | h] row once
// (profiles/r01_ab_wgrad_tiles.log: 874 -> 798 ms/meta-step against 128 x 128, BK 32)
#ifndef SMAML_WGRAD_THREADS
#define SMAML_WGRAD_THREADS (3072 * 256)  // split-K target: total threads of one weight-gradient launch
                                          // (A/B at config 2: 2048 -> 3072 x 256: wgrad 747 -> 711 ms)
#endif
#ifndef SMAML_EPI_PRELOAD_FWD
#define SMAML_EPI_PRELOAD_FWD 1  // fused forward step: load a tile's c_{t-1} before its stores
                                 // (r01 A/B: 339 -> 335.5 ms per meta-step)
#endif
#ifndef SMAML_TN_NST
#define SMAML_TN_NST 2  // weight-gradient staged-split LDS stages
#endif
#ifndef SMAML_TN_BK
#define SMAML_TN_BK 16
#endif
#ifndef SMAML_TN_BM
#define SMAML_TN_BM 512
#endif
#ifndef SMAML_TN_BN
#define SMAML_TN_BN 128
#endif
#ifndef SMAML_TN_WM
#define SMAML_TN_WM 8
#endif
#ifndef SMAML_TN_WN
#define SMAML_TN_WN 1
#endif

// Minimum resident waves per SIMD requested from the register allocator for the LSTM gate
// kernels (0 = compiler default). A/B-able at build time.
#ifndef SMAML_GATE_WPE
#define SMAML_GATE_WPE 4
#endif
#ifndef SMAML_GATED_WPE
#define SMAML_GATED_WPE 4  // same, for the tangent (dual) gate kernel (127 VGPRs with SMAML_DUAL_RELOAD)
#endif
#ifndef SMAML_BWDD_WPE
#define SMAML_BWDD_WPE 3  // same, for the tangent BPTT kernel (LDS caps it at 3 anyway)
#endif
#ifndef SMAML_BWD_WPE
#define SMAML_BWD_WPE 5  // same, for the primal BPTT kernel (<= 96 VGPRs)
#endif
#if SMAML_BWD_WPE > 0
#define SMAML_BWD_ATTR __attribute__((amdgpu_waves_per_eu(SMAML_BWD_WPE)))
#else
#define SMAML_BWD_ATTR
#endif
#if SMAML_BWDD_WPE > 0
#define SMAML_BWDD_ATTR __attribute__((amdgpu_waves_per_eu(SMAML_BWDD_WPE)))
#else
#define SMAML_BWDD_ATTR
#endif
#if SMAML_GATE_WPE > 0
#define SMAML_GATE_ATTR __attribute__((amdgpu_waves_per_eu(SMAML_GATE_WPE)))
#else
#define SMAML_GATE_ATTR
#endif
#if SMAML_GATED_WPE > 0
#define SMAML_GATED_ATTR __attribute__((amdgpu_waves_per_eu(SMAML_GATED_WPE)))
#else
#define SMAML_GATED_ATTR
#endif

namespace smaml {

struct RowMajorKC {  // [rows][K] with K contiguous
  const float* p;
  int rows, K;
  __device__ __forceinline__ float4 operator()(int r, int k) const {
    if (r >= rows || k >= K) return f4zero();
    return ld4(p + (int64_t)r * K + k);
  }
};

struct RowMajorMC {  // [K][cols] with cols contiguous
  const float* p;
  int64_t K;
  int cols;
  __device__ __forceinline__ float4 operator()(int64_t k, int c) const {
    if (k >= K || c >= cols) return f4zero();
    return ld4(p + k * cols + c);
  }
};

// A operand [rows][w0 | w1 | w2 | w3]: segment s is a row-major [rows][w_s] matrix
// (nullptr = zeros). Widths must be multiples of 4.
struct SegKC {
  const float* p[4];
  int w[4];
  int rows;
  __device__ __forceinline__ float4 operator()(int r, int k) const {
    if (r >= rows) return f4zero();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (k < w[s]) return p[s] ? ld4(p[s] + (int64_t)r * w[s] + k) : f4zero();
      k -= w[s];
    }
    return f4zero();
  }
};

// B operand for the LSTM gate GEMMs: logical row n = ug*128 + g*32 + jj maps to weight
// row g*H + ug*32 + jj of each segment matrix [4H][w_s] (k-concatenated).
struct SegGateB {
  const float* p[4];
  int w[4];
  int H;
  __device__ __forceinline__ float4 operator()(int n, int k) const {
    const int ug = n >> 7, rem = n & 127, g = rem >> 5, j = ug * 32 + (rem & 31);
    if (j >= H) return f4zero();
    const int64_t row = (int64_t)g * H + j;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (k < w[s]) return p[s] ? ld4(p[s] + row * w[s] + k) : f4zero();
      k -= w[s];
    }
    return f4zero();
  }
};

// B operand [K0 + K1][cols]: two row-major matrices stacked along K (cols contiguous).
struct SegMC {
  const float* p[2];
  int64_t K[2];
  int cols;
  __device__ __forceinline__ float4 operator()(int64_t k, int c) const {
    if (c >= cols) return f4zero();
    if (k < K[0]) return ld4(p[0] + k * cols + c);
    k -= K[0];
    if (k < K[1]) return ld4(p[1] + k * cols + c);
    return f4zero();
  }
};

// Weight-gradient B operand: Bcat[k] = [B1[k][0..c1) | (k >= Mshift ? B2[k-Mshift][0..c2) : 0)]
// (B1 == nullptr -> zeros: the layer-0 input has no tangent).
struct WgB {
  const float* B1;
  const float* B2;
  int c1, c2;
  int64_t K, Mshift;
  __device__ __forceinline__ float4 operator()(int64_t k, int j) const {
    if (k >= K) return f4zero();
    if (j < c1) return B1 ? ld4(B1 + k * c1 + j) : f4zero();
    j -= c1;
    if (j >= c2 || k < Mshift) return f4zero();
    return ld4(B2 + (k - Mshift) * c2 + j);
  }
};

// ---- tile loaders (gemm_core.h has_tile_fetch) -------------------------------------------
// Contract: every segment width is a multiple of BK (so a K-tile lies inside one segment, chosen
// once per tile with scalar code) and the GEMM's K is the sum of the widths (no K tail). Rows /
// columns past the matrix edge are CLAMPED to the last valid one instead of zero-filled: their
// products land in accumulator rows / columns the epilogues never store. Per-lane offsets are
// 32-bit byte offsets from a uniform 64-bit tile base (global_load ... saddr).
__device__ __forceinline__ float4 ldo(const float* base, uint32_t byteoff) {
  return *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(base) + byteoff);
}
// Non-temporal (streaming) 16-B load / store: `nt` cache policy, so data read or written once per
// launch does not evict what the launch re-reads from L2 (the per-task weight operands).
typedef float f32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld4_nt(const float* p) {
  const f32x4v v = __builtin_nontemporal_load(reinterpret_cast<const f32x4v*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st4_nt(float* p, const float4& v) {
  f32x4v w;
  w.x = v.x;
  w.y = v.y;
  w.z = v.z;
  w.w = v.w;
  __builtin_nontemporal_store(w, reinterpret_cast<f32x4v*>(p));
}
template <bool NT>
__device__ __forceinline__ float4 ldo_(const float* base, uint32_t byteoff) {
  if constexpr (NT)
    return ld4_nt(reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + byteoff));
  else
    return ldo(base, byteoff);
}

// The segment holding K index k0 (segment widths w[], k-concatenated): its base pointer, width and
// the offset inside it. Every member is read unconditionally and the choice is made on the values:
// the per-segment `if (kk >= ws) b = p[s]` chain became a select of member ADDRESSES, a dynamic
// index that kept the 4-segment loaders of the tangent gate kernel in scratch memory (two scratch
// loads per K-tile, the 112-120 B "spill" of rounds 1-2).
template <int NS, typename P>
__device__ __forceinline__ void seg_pick(const P (&p)[NS], const int (&w)[NS], int k0, P& b, int& ws, int& kk) {
  static_assert(NS >= 1 && NS <= 4, "up to 4 segments");
  // every member read unconditionally first, then selected as values
  const P p0 = p[0], p1 = p[NS > 1 ? 1 : 0], p2 = p[NS > 2 ? 2 : 0], p3 = p[NS > 3 ? 3 : 0];
  const int w0 = w[0], w1 = w[NS > 1 ? 1 : 0], w2 = w[NS > 2 ? 2 : 0];
  const int e1 = w0, e2 = e1 + (NS > 1 ? w1 : 0), e3 = e2 + (NS > 2 ? w2 : 0);
  const int s = (NS > 1 && k0 >= e1) + (NS > 2 && k0 >= e2) + (NS > 3 && k0 >= e3);
  b = s == 0 ? p0 : s == 1 ? p1 : s == 2 ? p2 : p3;
  kk = k0 - (s == 0 ? 0 : s == 1 ? e1 : s == 2 ? e2 : e3);
  ws = s == 0 ? w0 : s == 1 ? w1 : s == 2 ? w2 : w[NS - 1];
}

// KC operand [rows][w_s] per segment (row stride = width), k-concatenated. NT: streaming loads.
template <int NS, bool NT = false>
struct SegKCt {
  static constexpr bool kTileFetch = true;
  const float* p[NS];
  int w[NS];
  int rows;
  template <int ROWS, int F4, int NTH, bool KC, int BK>
  __device__ __forceinline__ void fetch(int row0, int k0, float4 (&r)[F4]) const {
    static_assert(KC, "SegKCt is a k-contiguous operand");
    const float* b;
    int ws, kk;
    seg_pick<NS>(p, w, k0, b, ws, kk);
    b += kk + (int64_t)row0 * ws;  // the tile's first row: 64-bit, uniform
#pragma unroll
    for (int i = 0; i < F4; ++i) {
      const int f = (int)threadIdx.x + NTH * i;
      const int dr = min(row0 + f / (BK / 4), rows - 1) - row0;
      r[i] = ldo_<NT>(b, 4u * (uint32_t)(dr * ws + 4 * (f % (BK / 4))));
    }
  }
};

// MC operand [K_s][cols] per segment (cols contiguous), k-concatenated.
template <int NS>
struct SegMCt {
  static constexpr bool kTileFetch = true;
  const float* p[NS];
  int K[NS];
  int cols;
  template <int ROWS, int F4, int NTH, bool KC, int BK>
  __device__ __forceinline__ void fetch(int col0, int k0, float4 (&r)[F4]) const {
    static_assert(!KC, "SegMCt is an n-contiguous operand");
    const float* b;
    int ks, kk;
    seg_pick<NS>(p, K, k0, b, ks, kk);
    b += (int64_t)kk * cols;
#pragma unroll
    for (int i = 0; i < F4; ++i) {
      const int f = (int)threadIdx.x + NTH * i;
      const int c = min(col0 + 4 * (f % (ROWS / 4)), cols - 4);
      r[i] = ldo(b, 4u * (uint32_t)((f / (ROWS / 4)) * cols + c));
    }
  }
};

// LSTM gate-GEMM B operand (SegGateB's row mapping: logical row n = ug*128 + g*32 + jj ->
// weight row g*H + ug*32 + jj of each [4H][w_s] segment), k-concatenated.
template <int NS>
struct SegGateBt {
  static constexpr bool kTileFetch = true;
  const float* p[NS];
  int w[NS];
  int H;
  template <int ROWS, int F4, int NTH, bool KC, int BK>
  __device__ __forceinline__ void fetch(int n0, int k0, float4 (&r)[F4]) const {
    static_assert(KC, "SegGateBt is a k-contiguous operand");
    const float* b;
    int ws, kk;
    seg_pick<NS>(p, w, k0, b, ws, kk);
    b += kk;
#pragma unroll
    for (int i = 0; i < F4; ++i) {
      const int f = (int)threadIdx.x + NTH * i;
      const int n = n0 + f / (BK / 4);
      const int ug = n >> 7, rem = n & 127;
      const int j = min(ug * 32 + (rem & 31), H - 1);
      const int row = (rem >> 5) * H + j;
      r[i] = ldo(b, 4u * (uint32_t)(row * ws + 4 * (f % (BK / 4))));
    }
  }
};

// Gate-GEMM B operand as pre-split bf16 images (gemm_core.h has_dma_image; launch_split_gate): the
// image of segment s, unit group ug (= n0 / 128), K-tile kt is the X6Img<128, KC, 16> at
// p[s] + (ug * (w[s] / 16) + kt) * GATE_IMG_BYTES, with SegGateBt's row mapping (image row
// g * 32 + jj = weight row g * H + ug * 32 + jj). Every wave copies its share of the image's 1-KB
// chunks with global_load_lds_dwordx4 (64 lanes x 16 B, lane-contiguous in LDS).
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;
template <int NS>
struct SegGateImg {
  static constexpr bool kDmaImage = true;
  const char* p[NS];
  int w[NS];
  template <int ROWS, bool KC, int BK, int NTH>
  __device__ __forceinline__ void issue(char* dst, int n0, int k0) const {
    static_assert(ROWS == 128 && KC && BK == 16, "gate images: 128 rows x 16 k");
    const char* b;
    int ws, kk;
    seg_pick<NS>(p, w, k0, b, ws, kk);
    const char* src = b + ((int64_t)(n0 >> 7) * (ws / BK) + kk / BK) * GATE_IMG_BYTES;
    const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6;
    constexpr int CH = GATE_IMG_BYTES / 1024, NW = NTH / 64;
#pragma unroll
    for (int c = 0; c < (CH + NW - 1) / NW; ++c) {
      const int ch = wave + NW * c;
      if (CH % NW == 0 || ch < CH)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + ch * 1024 + 16 * lane), (lds_void_t*)(dst + ch * 1024),
                                         16, 0, 0);
    }
  }
};

// Dropout mask on the x segment of an LSTM layer's input: x = drop(h_{l-1}) of one
// (task, t) slab; element (m, k) has index base + m*H + k (kernels.h Drop, kind 2).
struct XDrop {
  uint32_t site, thr;
  float sc;
  uint64_t base;
  int H;
  __device__ __forceinline__ float4 apply(float4 v, int m, int k) const {
    const uint64_t i0 = base + (uint64_t)m * H + k;
    v.x = drop_keep(site, i0, thr) ? v.x * sc : 0.f;
    v.y = drop_keep(site, i0 + 1, thr) ? v.y * sc : 0.f;
    v.z = drop_keep(site, i0 + 2, thr) ? v.z * sc : 0.f;
    v.w = drop_keep(site, i0 + 3, thr) ? v.w * sc : 0.f;
    return v;
  }
};

// acc(m, j) *= mask of element base + m*H + j (the BPTT's layer-above segment, whose dX
// reaches h_l through drop(h_l)).
template <class C>
__device__ __forceinline__ void drop_acc(Acc<C>& acc, const XDrop& d, int m0, int n0) {
#pragma unroll
  for (int i = 0; i < C::WTM; ++i)
#pragma unroll
    for (int jj = 0; jj < C::WTN; ++jj) {
      const int j = n0 + acc_col<C>(jj);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint64_t idx = d.base + (uint64_t)(m0 + acc_row<C>(i, r)) * d.H + j;
        acc.v[i][jj][r] = drop_keep(d.site, idx, d.thr) ? acc.v[i][jj][r] * d.sc : 0.f;
      }
    }
}

// SegKC whose segments 0 (x) and 2 (R x) are dropout-masked (tangent gate GEMM, layers >= 1).
struct SegKCDrop {
  SegKC s;
  XDrop d;
  __device__ __forceinline__ float4 operator()(int r, int k) const {
    if (r >= s.rows) return f4zero();
    int kk = k;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (kk < s.w[q]) {
        if (!s.p[q]) return f4zero();
        const float4 v = ld4(s.p[q] + (int64_t)r * s.w[q] + kk);
        return (q == 0 || q == 2) ? d.apply(v, r, kk) : v;
      }
      kk -= s.w[q];
    }
    return f4zero();
  }
};

// Gate nonlinearities. SMAML_FAST_GATES (default) uses the hardware transcendentals:
// v_exp_f32 on x*log2(e) and v_rcp_f32 (1 ulp), and for tanh 1 - 2/(1+e^{2|x|}) with an odd
// Taylor polynomial below |x| < 0.125 (no cancellation near 0). Relative error <~1e-6 per
// evaluation (|x| < ~16), absolute error <~2e-7; the parity tests bound the end-to-end effect.
#ifndef SMAML_FAST_GATES
#define SMAML_FAST_GATES 1
#endif
#if SMAML_FAST_GATES
__device__ __forceinline__ float sigmoidf_(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}
__device__ __forceinline__ float tanhf_(float x) {
  // branchless (both forms, then a select): a per-element branch here splits the epilogues into
  // exec-masked blocks and serialises their memory operations
  const float a = fabsf(x);
  const float x2 = x * x;
  const float p = x * fmaf(x2, fmaf(x2, fmaf(x2, -0.053968254f, 0.13333334f), -0.33333334f), 1.0f);
  const float e = __builtin_amdgcn_exp2f(2.8853900817779268f * a);
  const float r = copysignf(1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + e), x);
  return a < 0.125f ? p : r;
}
#else
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ float tanhf_(float x) { return tanhf(x); }
#endif

// LSTM cell state with a fixed operation order: c_t = f c_{t-1} + i g and its tangent
// R(c_t) = R(f) c_{t-1} + f R(c_{t-1}) + R(i) g + i R(g). Every kernel that stores c_t (or R c_t)
// forms it here, so the backward kernels re-derive it bitwise from the stored gates and c_{t-1}
// instead of loading it (one 4-B read per element less in the HBM-bound BPTT epilogues).
__device__ __forceinline__ float lstm_cell_c(float gi, float gf, float gg, float cp) { return fmaf(gf, cp, gi * gg); }
__device__ __forceinline__ float lstm_cell_rc(float gi, float gf, float gg, float cp, float ri, float rf, float rg,
                                              float rcp) {
  return fmaf(gi, rg, fmaf(ri, gg, fmaf(gf, rcp, rf * cp)));
}


// Uniform (SGPR) base + 32-bit byte offset: lets the compiler use global_* saddr addressing
// with the constant part of the offset folded into the instruction's immediate.
__device__ __forceinline__ float ldb(const float* base, uint32_t byteoff) {
  return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + byteoff);
}
__device__ __forceinline__ void stb(float* base, uint32_t byteoff, float v) {
  *reinterpret_cast<float*>(reinterpret_cast<char*>(base) + byteoff) = v;
}

// XCD-aware tile mapping for the gate GEMMs: the 4 unit-group workgroups of one row tile
// are dispatched 8 apart (same XCD under round-robin placement: L2 sharing of the A rows)
// and within 32 consecutive blocks. Grid: gridDim.x = gate_blocks(ntm, ngrp) per problem
// (ngrp = 4H/128). Below 8 row tiles (batch-1 steps) the padded layout would leave whole XCDs
// idle (only blocks with blockIdx % 8 < ntm do work), so there the tiles are packed: tm fastest.
// Speed-only: a different placement changes nothing but speed. Returns false for padding.
__host__ __device__ inline int gate_blocks(int ntm, int ngrp) { return ntm < 8 ? ntm * ngrp : (ntm + 7) / 8 * 8 * ngrp; }
__device__ __forceinline__ bool gate_tile(int L, int ntm, int ngrp, int& tm, int& ug) {
  if (ntm < 8) {
    ug = L / ntm;
    tm = L - ug * ntm;
    return ug < ngrp;
  }
  const int per = 8 * ngrp;
  const int q = L / per, rem = L - q * per;
  ug = rem >> 3;
  tm = q * 8 + (rem & 7);
  return tm < ntm;
}

__device__ __forceinline__ bool gate_tile(int ntm, int ngrp, int& tm, int& ug) {
  return gate_tile((int)blockIdx.x, ntm, ngrp, tm, ug);
}

#ifndef SMAML_XCD_REMAP
#define SMAML_XCD_REMAP 0  // LSTM step kernels: XCD-contiguous workgroup order (0 = hardware order).
#endif                     // Measured slower at config 2 (2494 -> 2557 ms per meta-step: BPTT +13,
                           // tangent BPTT +35, forward +12 ms; profiles/r02_ab_xcd_remap.log).
// Workgroup coordinates after an XCD-contiguous remap. The hardware places linear workgroup id L
// on XCD L % 8 (round robin), so in hardware order every XCD runs tiles of every (task, layer)
// problem and each XCD's 4 MB L2 must hold all of their weight operands (the BPTT's B is the
// whole 1024 x 128 weight slice per tile: 0.5 MB, 1 MB with the tangent's): it thrashes and the
// operand streams from HBM. Here logical ids are dealt so that XCD k runs one contiguous range of
// the (z, y, x) order, x fastest: a few (task, layer) problems per XCD. Bijective for any count
// (q = n / 8 ids on each XCD, one more on the first n % 8). Speed only.
struct Blk {
  int x, y, z;
};
__device__ __forceinline__ Blk xcd_block() {
  if (!SMAML_XCD_REMAP) return {(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
  const int gx = gridDim.x, gy = gridDim.y;
  const int n = gx * gy * (int)gridDim.z;
  const int L = (int)blockIdx.x + gx * ((int)blockIdx.y + gy * (int)blockIdx.z);
  const int q = n >> 3, r = n & 7, xcd = L & 7;
  const int lg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (L >> 3);
  const int rest = lg / gx;
  return {lg - rest * gx, rest % gy, rest / gy};
}

// Wavefront problems (kernels.h FwdWave / BwdWave): the problem owning block bx, and a field
// of it, selected with scalar compares (no dynamic indexing into the by-value kernel argument).
template <class WV>
__device__ __forceinline__ int wave_index(const WV& wv, int bx) {
  constexpr int NQ = (int)(sizeof(wv.l) / sizeof(wv.l[0]));
  int p = 0;
#pragma unroll
  for (int q = 1; q < NQ; ++q)
    if (q < wv.n && bx >= wv.off[q]) p = q;
  return p;
}
template <class T, int N>
__device__ __forceinline__ T wave_sel(const T (&a)[N], int p) {
  T v = a[0];
#pragma unroll
  for (int q = 1; q < N; ++q)
    if (q == p) v = a[q];
  return v;
}
// BPTT diagonal block -> (problem p, row tile mb), problem-major as launched.
template <class WV>
__device__ __forceinline__ int bwd_block(const WV& wv, int bx, int& mb) {
  const int p = wave_index(wv, bx);
  mb = bx - wave_sel(wv.off, p);
  return p;
}

template <class WV, class LO>
__device__ __forceinline__ void wave_problem(const WV& wv, int bx, int& l, int& t, LO& lo, int& b0) {
  const int p = wave_index(wv, bx);
  l = wave_sel(wv.l, p);
  t = wave_sel(wv.t, p);
  lo = wave_sel(wv.lo, p);
  b0 = wave_sel(wv.off, p);
}

// acc -> smem [BM][BN] (row-major), for epilogues that work on row-contiguous float4 groups
// instead of the accumulator's column-per-lane layout; ends with a barrier. The caller's mainloop
// must have retired its LDS reads (gemm_mainloop / gemm_dual_mainloop end with a barrier) and
// smem must hold BM * BN floats.
template <class C>
__device__ __forceinline__ void acc_to_lds(const Acc<C>& acc, float* smem) {
#pragma unroll
  for (int i = 0; i < C::WTM; ++i)
#pragma unroll
    for (int jj = 0; jj < C::WTN; ++jj) {
      const int col = acc_col<C>(jj);
#pragma unroll
      for (int r = 0; r < 16; ++r) smem[acc_row<C>(i, r) * C::BN + col] = acc.v[i][jj][r];
    }
  __syncthreads();
}

// Half of the tile (rows [h*BM/2, (h+1)*BM/2)) -> smem [BM/2][BN]: written by the waves that own
// those rows (WAVES_M == 2); ends with a barrier. Lets an epilogue run in two halves over BM*BN/2 floats.
template <class C>
__device__ __forceinline__ void acc_to_lds_half(const Acc<C>& acc, float* smem, int h) {
  static_assert(C::WAVES_M == 2, "one row half per wave row");
  const int wm = (int)(threadIdx.x >> 6) / C::WAVES_N;
  if (wm == h) {
#pragma unroll
    for (int i = 0; i < C::WTM; ++i)
#pragma unroll
      for (int jj = 0; jj < C::WTN; ++jj) {
        const int col = acc_col<C>(jj);
#pragma unroll
        for (int r = 0; r < 16; ++r) smem[(acc_row<C>(i, r) - h * (C::BM / 2)) * C::BN + col] = acc.v[i][jj][r];
      }
  }
  __syncthreads();
}
template <class C>
struct HalfRows {  // the epilogue's view of one row half of C's tile
  static constexpr int BM = C::BM / 2, BN = C::BN, NTH = C::NTH;
};

__device__ __forceinline__ float4 sel4(bool c, float4 a) { return c ? a : f4zero(); }
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ void f4set(float4& v, int e, float x) {
  if (e == 0) v.x = x;
  if (e == 1) v.y = x;
  if (e == 2) v.z = x;
  if (e == 3) v.w = x;
}
#ifndef SMAML_FWD_EPI_T
#define SMAML_FWD_EPI_T 1  // fused forward steps' cell epilogues through gate_epilogue_t (float4 items)
#endif

// Row offset (within the 32-row tile) of accumulator register r: (r&3) + 8*(r>>2).
__device__ __forceinline__ constexpr int racc(int r) { return (r & 3) + 8 * (r >> 2); }

__device__ __forceinline__ void sto(float* base, uint32_t byteoff, const float4& v) {
  *reinterpret_cast<float4*>(reinterpret_cast<char*>(base) + byteoff) = v;
}

// Transposed gate epilogue of the fused forward steps (round 3). A gate tile of C (WAVES_N == 1:
// wave w owns tile rows 32w .. 32w+31; its 4 accumulator tiles are the 4 gates of the tile's 32
// units) is handed out in items of 4 consecutive units of one row, so the epilogue's loads and
// stores are 16 B wide (4x fewer memory instructions than the accumulator layout's 4-B accesses):
// each wave writes its own rows, plus badd, through a private 8 KB of the (idle) staging LDS in two
// 16-row passes (the 32-float gate blocks of row rl swapped pairwise when (rl ^ rl >> 2) is odd, so
// the ds_write_b32 and ds_read_b128 are bank-conflict free) and reads them back as float4 items.
// Per pass a lane has 2 items: ld(ml, u) issues both items' loads before st(ml, u, pre, v) stores
// either (ml = tile row, u = tile unit, pre[g] = gate g of units u .. u+3). Starts with a barrier
// (the mainloop's last LDS reads), leaves the LDS in use until the caller's next barrier.
template <class C, class LD, class ST>
__device__ __forceinline__ void gate_epilogue_t(const Acc<C>& acc, const float (&badd)[4], float* smem, LD&& ld,
                                                ST&& st) {
  static_assert(C::WAVES_N == 1 && C::WTM == 1 && C::WTN == 4, "wave = 32 rows x 4 gates x 32 units");
  static_assert(C::SMEM_FLOATS >= C::WAVES_M * 2048, "8 KB of LDS per wave");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, jj = lane & 31, h = lane >> 5;
  float* ws = smem + wave * 2048;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    // p = 0: the mainloop's LDS reads are done; p = 1: pass 0's reads are done
    __syncthreads();
#pragma unroll
    for (int r = 8 * p; r < 8 * p + 8; ++r) {
      const int rl = racc(r) + 4 * h - 16 * p;
      const int sw = (rl ^ (rl >> 2)) & 1;
#pragma unroll
      for (int g = 0; g < 4; ++g) ws[rl * 128 + (g ^ sw) * 32 + jj] = acc.v[0][g][r] + badd[g];
    }
    __syncthreads();
    decltype(ld(0, 0)) v[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = lane + 64 * k;
      v[k] = ld(wave * 32 + 16 * p + (i >> 3), 4 * (i & 7));
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = lane + 64 * k, rl = i >> 3, q = i & 7;
      const int sw = (rl ^ (rl >> 2)) & 1;
      float4 pre[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) pre[g] = ld4(ws + rl * 128 + (g ^ sw) * 32 + 4 * q);
      st(wave * 32 + 16 * p + rl, 4 * q, pre, v[k]);
    }
  }
}


// Gate accumulators of one gate tile (wave = 32 rows x 4 gates x 32 units, the layout fwd_cell reads)
// loaded from rows of a [.][4H] pre-activation table x (XgDedup: layer 0's input projection), instead
// of zeroed: the K loop then adds the recurrent segment on top. Rows past M load row M - 1 (never
// stored); units past H read unit H - 1 (never stored).
template <class C, int H>
__device__ __forceinline__ void acc_load_gates(Acc<C>& acc, const float* __restrict__ x, int m0, int ug, int M) {
  static_assert(C::WTM == 1 && C::WTN == 4, "wave = one 32-row tile of the 4 gates");
  constexpr int UPB = C::WAVES_N;
  const int j = min((ug * UPB + (int)(threadIdx.x >> 6) % UPB) * 32 + (int)(threadIdx.x & 31), H - 1);
  const int rb = m0 + acc_row<C>(0, 0);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const uint32_t m = (uint32_t)min(rb + racc(r), M - 1);
#pragma unroll
    for (int g = 0; g < 4; ++g) acc.v[0][g][r] = ldb(x, 4u * (m * (4 * H) + (uint32_t)(g * H + j)));
  }
}

// LSTM kernels are instantiated per hidden size (compile-time strides).
#define SMAML_DISPATCH_H(HV, ...)                              \
  switch (HV) {                                                \
    case 32: { constexpr int HT = 32; __VA_ARGS__; } break;    \
    case 64: { constexpr int HT = 64; __VA_ARGS__; } break;    \
    case 128: { constexpr int HT = 128; __VA_ARGS__; } break;  \
    case 256: { constexpr int HT = 256; __VA_ARGS__; } break;  \
    default: break;                                            \
  }

}  // namespace smaml
