// GEMM core for gfx950 (CDNA4): f32 operands, f32 accumulation.
//
// All GEMM-shaped work on the STGCN-LSTM path goes through these mainloops. Products (GemmCfg X6_):
//   2 (default, "staged bf16x6"): the thread that stages a float4 of an operand splits it into three
//     bf16 pieces (x = x0 + x1 + x2, exact to 2^-27 |x|) written to bf16 LDS planes; each 16-k step
//     issues six v_mfma_f32_32x32x16_bf16 (the piece products a_i b_j with i + j <= 2, f32
//     accumulation): f32-accurate products at 6/16 of the f32 MFMA's cost (mfma_x6, split4);
//   1 ("fragment split"): f32 LDS images, the split on each wave's MFMA fragments (split3);
//   0: v_mfma_f32_32x32x2_f32 (exact f32 products) from f32 LDS images (-DSMAML_X6=0).
// Special values: the split is exact for every finite |x| < 3.3961e38; an inf operand, or a finite
// one at or above that (its RNE piece x0 overflows to inf), makes the products NaN (inf - inf),
// where f32 MFMA products could give inf or, for |x| in [3.3961e38, FLT_MAX], a finite value.
//
// f32 LDS images (X6_ 0 / 1), K order: inside a K-tile, MFMA k-step s of lane half h (= lane>>5)
// covers k = (BK/2) h + s, so one lane's k-values of a row are contiguous: a k-contiguous ("KC")
// operand is kept row-major in LDS ([rows][BK+4], written with ds_write_b128) and each lane fetches
// 4 k-steps of a fragment with ONE conflict-free ds_read_b128. An "MC" operand (rows contiguous,
// e.g. W_hh used as [k][n]) is kept k-major in LDS ([BK][rows+4]) and read with ds_read_b32.
// The staged bf16 images (X6Img) are described at their definition.
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
#ifndef SMAML_X6
#define SMAML_X6 1  // default product form of GemmCfg: 1 = bf16x6 (f32-accurate, see mfma_x6), 0 = f32 MFMA
#endif

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

// bf16-piece LDS image of one operand tile for the staged split (GemmCfg X6_ = 2): three planes
// (x0, x1, x2), each bf16. KC operands: [rows][BK] per plane, 16-B chunks XOR-swizzled by row so the
// ds_read_b128 fragment reads are conflict-free; MC operands: [BK][rows] per plane, read transposed
// by ds_read_b64_tr_b16 (a 32-lane half reads 64 contiguous bytes of each of 4 consecutive image
// rows). Rows of a multiple of 128 elements are unpadded (stride 2*rows B, a multiple of 256) with
// the 64-B blocks of image row k XOR-swizzled by (k mod 4), which spreads those 4 reads over all
// 64 banks (round 3: the padded stride cost the tangent BPTT its third workgroup per CU); narrower
// ones keep the padded stride 2*rows + 64 B (== 64 or 192 mod 256).
template <int ROWS, bool KC, int BK, bool SWZ = true>
struct X6Img {
  static constexpr int NCH = BK / 8;                       // 16-B chunks per KC row
  static constexpr bool MSW = SWZ && !KC && ROWS % 128 == 0;  // MC image swizzled instead of padded
  static constexpr int RS = KC ? 2 * BK : MSW ? 2 * ROWS : 2 * ROWS + 64;  // bytes per image row
  static constexpr int PLANE = KC ? ROWS * RS : BK * RS;   // bytes per plane
  static constexpr int BYTES = 3 * PLANE;
  static_assert(!KC || NCH == 2 || NCH == 4 || NCH == 8, "KC staged split: BK 16, 32 or 64");
  static_assert(KC || ROWS % 64 == 0, "MC staged split: rows multiple of 64");
  __device__ static __forceinline__ int swz(int r) {
    return NCH == 2 ? (r >> 3) & 1 : NCH == 4 ? (r >> 2) & 3 : (r >> 1) & 7;
  }
  // MC: byte offset of byte b (even, 8-B chunks never split) of image row k within a plane
  __device__ static __forceinline__ int mc(int k, int b) { return k * RS + (MSW ? b ^ ((k & 3) << 6) : b); }
};

template <int BM_, int BN_, int WAVES_M_, int WAVES_N_, bool A_KC_, bool B_KC_, int BK_ = 32, int X6_ = SMAML_X6,
          int NST_ = 2, bool MSW_ = true>
struct GemmCfg {
  static constexpr bool MSW = MSW_;  // staged MC images: swizzled (unpadded) where the rows allow (X6Img)
  static constexpr int X6S_NST = NST_;  // staged split: LDS stages (1 = register prefetch, two barriers)
  static constexpr int BK = BK_;
  // products: 0 = v_mfma_f32_32x32x2_f32; 1 = bf16x6 with the split on the MFMA fragments (mma_tile);
  // 2 = bf16x6 with the split done once per element at the LDS store (gemm_mainloop, "staged")
  static constexpr bool X6 = X6_ != 0;
  static constexpr bool X6S = X6_ == 2;
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
  using AImg = X6Img<BM, A_KC, BK, MSW>;
  using BImg = X6Img<BN, B_KC, BK, MSW>;
  static constexpr int X6S_STAGE = AImg::BYTES + BImg::BYTES;  // bytes per staged-split stage
  static constexpr int SMEM_FLOATS = (X6S && NST_ * X6S_STAGE / 4 > 2 * (A_STAGE + B_STAGE))
                                        ? NST_ * X6S_STAGE / 4
                                        : 2 * (A_STAGE + B_STAGE);
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

// acc -> P[m][j] (rows m0.., columns n0..; [M][H] rows)
template <class C>
__device__ __forceinline__ void store_acc_rows(const Acc<C>& acc, float* P, int m0, int n0, int M, int H) {
#pragma unroll
  for (int i = 0; i < C::WTM; ++i)
#pragma unroll
    for (int jj = 0; jj < C::WTN; ++jj) {
      const int j = n0 + acc_col<C>(jj);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + acc_row<C>(i, r);
        if (m < M && j < H) P[(int64_t)m * H + j] = acc.v[i][jj][r];
      }
    }
}

// Optional hooks: operator() runs once per K-tile on the staged A tile; afrag(i, a) sees every
// A fragment this lane feeds to the MFMAs (4 k-steps of tile row i), e.g. for column sums
// of A (bias gradients) kept in registers instead of re-read from LDS.
struct NoHook {
  __device__ __forceinline__ void operator()(const float*, int) const {}
  __device__ __forceinline__ void afrag(int, const float4&) {}
};

// ---- fp32 products on the bf16 MFMA pipe (SMAML_X6) ---------------------------------------
// x = x0 + x1 + x2 with each piece a bf16 (x0 = RNE(x), x1 = RNE(x - x0), x2 = RNE(x - x0 - x1);
// the differences are exact in f32), so |x - x0 - x1 - x2| <= 2^-27 |x|. The product
// a.b = sum_{i+j<=2} a_i.b_j + O(2^-26 |a||b|) needs six v_mfma_f32_32x32x16_bf16 (each a_i.b_j
// is exact in f32; accumulation in f32 as in the f32 MFMA): an f32-accurate product at
// 6 x 32 = 192 SIMD cycles per 32x32x16 step against 8 x 64 = 512 for v_mfma_f32_32x32x2_f32.
// The fragment layout is the f32 one: for a 16-k step lane half h holds k = 8h .. 8h+7 of its row
// in frag4(q = 2s) and frag4(q = 2s + 1), exactly the bf16 MFMA operand layout (8 consecutive k per
// lane half), so the LDS images, loaders and hooks are unchanged; the split runs on the fragments.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

struct Split3 {
  bf16x8_t p0, p1, p2;
};

__device__ __forceinline__ uint32_t pk_bf16(float x, float y) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){x, y}, bf16x2_t));
}

__device__ __forceinline__ Split3 split3(const float4& lo, const float4& hi) {
  const float x[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  u32x4_t q0, q1, q2;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float a = x[2 * e], b = x[2 * e + 1];
    uint32_t u = pk_bf16(a, b);
    q0[e] = u;
    a -= __builtin_bit_cast(float, u << 16);
    b -= __builtin_bit_cast(float, u & 0xffff0000u);
    u = pk_bf16(a, b);
    q1[e] = u;
    a -= __builtin_bit_cast(float, u << 16);
    b -= __builtin_bit_cast(float, u & 0xffff0000u);
    q2[e] = pk_bf16(a, b);
  }
  return Split3{__builtin_bit_cast(bf16x8_t, q0), __builtin_bit_cast(bf16x8_t, q1), __builtin_bit_cast(bf16x8_t, q2)};
}

// acc += a . b over one 16-k step, smallest terms first.
__device__ __forceinline__ f32x16 mfma_x6(const Split3& a, const Split3& b, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p2, b.p0, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p1, b.p1, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p0, b.p2, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p1, b.p0, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p0, b.p1, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p0, b.p0, acc, 0, 0, 0);
  return acc;
}

template <class C, int IG = -1, class Hook = NoHook>
__device__ __forceinline__ void mma_tile(const float* as, const float* bs, Acc<C>& acc, Hook& hook) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / C::WAVES_N, wn = wave % C::WAVES_N;
  const int arow = wm * (C::WTM * 32) + (lane & 31);
  const int brow = wn * (C::WTN * 32) + (lane & 31);
  const int h = lane >> 5;
  if constexpr (IG >= 0) __builtin_amdgcn_iglp_opt(IG);
  if constexpr (C::X6) {
#pragma unroll
  for (int s = 0; s < C::BK / 16; ++s) {
    Split3 a[C::WTM];
#pragma unroll
    for (int i = 0; i < C::WTM; ++i) {
      const float4 lo = frag4<C::A_KC, C::LDA, C::BK>(as, arow + 32 * i, h, 2 * s);
      const float4 hi = frag4<C::A_KC, C::LDA, C::BK>(as, arow + 32 * i, h, 2 * s + 1);
      hook.afrag(i, lo);
      hook.afrag(i, hi);
      a[i] = split3(lo, hi);
    }
#pragma unroll
    for (int j = 0; j < C::WTN; ++j) {
      const Split3 b = split3(frag4<C::B_KC, C::LDB, C::BK>(bs, brow + 32 * j, h, 2 * s),
                              frag4<C::B_KC, C::LDB, C::BK>(bs, brow + 32 * j, h, 2 * s + 1));
#pragma unroll
      for (int i = 0; i < C::WTM; ++i) acc.v[i][j] = mfma_x6(a[i], b, acc.v[i][j]);
    }
  }
  } else {
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
}

// ---- staged split (GemmCfg X6_ = 2) ----------------------------------------------------------
// The thread that fetched a float4 of an operand splits it once (split3 on 4 values) and writes the
// three bf16 pieces into the planes of the tile's X6Img; the MFMA phase reads bf16 fragments
// directly (KC: one ds_read_b128 per plane; MC: two ds_read_b64_tr_b16 per plane), so the split
// costs 5.5 VALU per element per workgroup instead of per wave that reads the fragment.
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));

#ifndef SMAML_DIAG_NOSPLIT
#define SMAML_DIAG_NOSPLIT 0  // timing diagnostic only (wrong results): 1 = the staged split stores raw bits, no VALU
#endif
__device__ __forceinline__ void split4(const float4& v, uint2& p0, uint2& p1, uint2& p2) {
  if constexpr (SMAML_DIAG_NOSPLIT) {
    p0 = make_uint2(__builtin_bit_cast(uint32_t, v.x), __builtin_bit_cast(uint32_t, v.y));
    p1 = make_uint2(__builtin_bit_cast(uint32_t, v.z), __builtin_bit_cast(uint32_t, v.w));
    p2 = p0;
    return;
  }
  const float x[4] = {v.x, v.y, v.z, v.w};
  uint32_t q0[2], q1[2], q2[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    float a = x[2 * e], b = x[2 * e + 1];
    uint32_t u = pk_bf16(a, b);
    q0[e] = u;
    a -= __builtin_bit_cast(float, u << 16);
    b -= __builtin_bit_cast(float, u & 0xffff0000u);
    u = pk_bf16(a, b);
    q1[e] = u;
    a -= __builtin_bit_cast(float, u << 16);
    b -= __builtin_bit_cast(float, u & 0xffff0000u);
    q2[e] = pk_bf16(a, b);
  }
  p0 = make_uint2(q0[0], q0[1]);
  p1 = make_uint2(q1[0], q1[1]);
  p2 = make_uint2(q2[0], q2[1]);
}

// Split this thread's staged float4s of one operand tile into the image at `img` (byte base).
template <int ROWS, int F4, int NTH, bool KC, int BK, bool SWZ = true>
__device__ __forceinline__ void store_tile_x6(char* img, const float4 (&r)[F4]) {
  using I = X6Img<ROWS, KC, BK, SWZ>;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < F4; ++i) {
    const int f = tid + NTH * i;
    int off;
    if (KC) {
      const int rr = f / (BK / 4), q = f % (BK / 4);
      off = rr * I::RS + 16 * ((q >> 1) ^ I::swz(rr)) + 8 * (q & 1);
    } else {
      const int kk = f / (ROWS / 4), q = f % (ROWS / 4);
      off = I::mc(kk, 8 * q);
    }
    uint2 p0, p1, p2;
    split4(r[i], p0, p1, p2);
    *reinterpret_cast<uint2*>(img + off) = p0;
    *reinterpret_cast<uint2*>(img + I::PLANE + off) = p1;
    *reinterpret_cast<uint2*>(img + 2 * I::PLANE + off) = p2;
  }
}

// B operand loaders that deliver PRE-SPLIT bf16 images (``kDmaImage``; loaders.h SegGateImg): the
// K-tile's image is copied global -> LDS with direct-to-LDS loads (no staging VGPRs, no split, no
// ds_write), issued into the stage the tile will be read from.
template <class L, class = void>
struct has_dma_image : std::false_type {};
template <class L>
struct has_dma_image<L, std::void_t<decltype(L::kDmaImage)>> : std::true_type {};

// B operand staging for the staged mainloops: f32 float4s, split at the LDS store; or (DMA) the
// image issued straight into the stage.
template <class C, class LB, bool DMA = has_dma_image<LB>::value>
struct BStage {
  float4 r[C::B_F4];
  __device__ __forceinline__ void fetch(const LB& lb, int n0, int k0, char*) {
    fetch_tile<C::BN, C::B_F4, C::NTH, C::B_KC, C::BK>(lb, n0, k0, r);
  }
  __device__ __forceinline__ void store(char* img) const {
    store_tile_x6<C::BN, C::B_F4, C::NTH, C::B_KC, C::BK, C::MSW>(img, r);
  }
};
template <class C, class LB>
struct BStage<C, LB, true> {
  static_assert(C::X6S && C::X6S_NST == 2, "pre-split B images: two LDS stages (issued into the idle one)");
  __device__ __forceinline__ void fetch(const LB& lb, int n0, int k0, char* img) {
    lb.template issue<C::BN, C::B_KC, C::BK, C::NTH>(img, n0, k0);
  }
  __device__ __forceinline__ void store(char*) const {}
};

// A operand staging: this thread's f32 float4s of the tile, split into the bf16 planes at the LDS store.
template <class C, class LA>
struct AStage {
  float4 r[C::A_F4];
  __device__ __forceinline__ void fetch(const LA& la, int m0, int k0, char*) {
    fetch_tile<C::BM, C::A_F4, C::NTH, C::A_KC, C::BK>(la, m0, k0, r);
  }
  __device__ __forceinline__ void store(char* img) const {
    store_tile_x6<C::BM, C::A_F4, C::NTH, C::A_KC, C::BK, C::MSW>(img, r);
  }
};

// The three pieces of the 32-row fragment at tile row `row` (this lane's row = row + (lane & 31)
// for KC; the fragment's first row for MC), MFMA step s (k = 16s + 8h .. 16s + 8h + 7).
template <int ROWS, bool KC, int BK, bool SWZ = true>
__device__ __forceinline__ Split3 frag_x6(const char* img, int row, int s) {
  using I = X6Img<ROWS, KC, BK, SWZ>;
  const int lane = threadIdx.x & 63;
  Split3 f;
  if (KC) {
    const int r = row + (lane & 31), h = lane >> 5;
    const int off = r * I::RS + 16 * ((2 * s + h) ^ I::swz(r));
    f.p0 = *reinterpret_cast<const bf16x8_t*>(img + off);
    f.p1 = *reinterpret_cast<const bf16x8_t*>(img + I::PLANE + off);
    f.p2 = *reinterpret_cast<const bf16x8_t*>(img + 2 * I::PLANE + off);
  } else {
    // ds_read_b64_tr_b16: per 16-lane group g, lane 4q+p addresses image row kb+q, columns
    // c0+4p..c0+4p+3; lane i receives column c0+i of rows kb..kb+3 (element q = row kb+q).
    const int g = lane >> 4, i = lane & 15;
    const int h = g >> 1;
    const int col = row + 16 * (g & 1) + 4 * (i & 3);
    const int off = I::mc(16 * s + 8 * h + (i >> 2), 2 * col);  // (row k + 4 below: same swizzle)
    typedef __attribute__((address_space(3))) bf16x4_t* lp;
    auto rd = [&](int o) {
      const bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lp)(img + o));
      const bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lp)(img + o + 4 * I::RS));
      return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    };
    f.p0 = rd(off);
    f.p1 = rd(I::PLANE + off);
    f.p2 = rd(2 * I::PLANE + off);
  }
  return f;
}

// MFMAs of the B fragments j in [J0, J1) (all of them by default).
template <class C, int IG = -1, int J0 = 0, int J1 = C::WTN>
__device__ __forceinline__ void mma_tile_x6s(const char* as, const char* bs, Acc<C>& acc) {
  const int wave = threadIdx.x >> 6;
  const int wm = wave / C::WAVES_N, wn = wave % C::WAVES_N;
  if constexpr (IG >= 0) __builtin_amdgcn_iglp_opt(IG);
#pragma unroll
  for (int s = 0; s < C::BK / 16; ++s) {
    Split3 a[C::WTM];
#pragma unroll
    for (int i = 0; i < C::WTM; ++i) a[i] = frag_x6<C::BM, C::A_KC, C::BK, C::MSW>(as, wm * (C::WTM * 32) + 32 * i, s);
#pragma unroll
    for (int j = J0; j < J1; ++j) {
      const Split3 b = frag_x6<C::BN, C::B_KC, C::BK, C::MSW>(bs, wn * (C::WTN * 32) + 32 * j, s);
#pragma unroll
      for (int i = 0; i < C::WTM; ++i) acc.v[i][j] = mfma_x6(a[i], b, acc.v[i][j]);
    }
  }
}

// Hooks may see the staged A float4s before the split (stage_a); see ColSumHook (kernels.hip).
template <class H, class = void>
struct has_stage_a : std::false_type {};
template <class H>
struct has_stage_a<H, std::void_t<decltype(&H::template stage_a<1>)>> : std::true_type {};

template <class C, int IG, class LA, class LB, class Hook>
__device__ __forceinline__ void gemm_mainloop_x6s(const LA& la, const LB& lb, int m0, int n0, int kbeg, int kend,
                                                  Acc<C>& acc, float* smem, Hook& hook) {
  constexpr int BKc = C::BK;
  constexpr int SA = C::AImg::BYTES;
  char* st0 = reinterpret_cast<char*>(smem);
  const int nkt = (kend - kbeg + BKc - 1) / BKc;
  if (nkt <= 0) return;
  constexpr bool DMA = has_dma_image<LB>::value;
  AStage<C, LA> ra;
  BStage<C, LB> rb;
  auto store = [&](char* st) {
    if constexpr (has_stage_a<Hook>::value) hook.template stage_a<C::A_F4>(ra.r);
    ra.store(st);
    rb.store(st + SA);
    if constexpr (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's image chunks landed
  };
  ra.fetch(la, m0, kbeg, st0);
  rb.fetch(lb, n0, kbeg, st0 + SA);
  store(st0);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nkt;
    if (more) {
      // (two stages: the idle one was last read by tile kt - 1's MFMAs, before the barrier)
      char* idle = st0 + (C::X6S_NST == 1 ? 0 : (cur ^ 1) * C::X6S_STAGE);
      ra.fetch(la, m0, kbeg + (kt + 1) * BKc, idle);
      rb.fetch(lb, n0, kbeg + (kt + 1) * BKc, idle + SA);
    }
    const char* st = st0 + (C::X6S_NST == 1 ? 0 : cur * C::X6S_STAGE);
    if constexpr (C::X6S_NST == 1) {
#if SMAML_PRIO
      __builtin_amdgcn_s_setprio(1);
#endif
      mma_tile_x6s<C, IG>(st, st + SA, acc);
#if SMAML_PRIO
      __builtin_amdgcn_s_setprio(0);
#endif
      if (more) {
        __syncthreads();  // every wave has read the stage
        store(st0);
      }
    } else {
#if SMAML_PRIO
      __builtin_amdgcn_s_setprio(1);
#endif
      mma_tile_x6s<C, IG>(st, st + SA, acc);
#if SMAML_PRIO
      __builtin_amdgcn_s_setprio(0);
#endif
      if (more) store(st0 + (cur ^ 1) * C::X6S_STAGE);
    }
    __syncthreads();
  }
}

// acc += sum_{k in [kbeg,kend)} A[m0+., k] * B[n0+., k]
// IG >= 0: ask LLVM for iglp_opt strategy IG in the MFMA phase (set per call site by A/B).
template <class C, int IG = -1, class LA, class LB, class Hook>
__device__ __forceinline__ void gemm_mainloop(const LA& la, const LB& lb, int m0, int n0, int kbeg,
                                              int kend, Acc<C>& acc, float* smem, Hook& hook) {
  if constexpr (C::X6S) {
    gemm_mainloop_x6s<C, IG>(la, lb, m0, n0, kbeg, kend, acc, smem, hook);
  } else {
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
      if (c0 + i < nkt) mma_tile<C, -1, NoHook>(As + i * C::A_STAGE, Bs + i * C::B_STAGE, acc, hook);
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
#ifndef SMAML_DUAL_X6S_STAGES
#define SMAML_DUAL_X6S_STAGES 1  // LDS stages of the staged-split dual mainloop (1: register prefetch, two barriers)
#endif
template <class C>
struct DualStage {
  static constexpr int X6S_BYTES = 2 * C::X6S_STAGE;  // [A | A2 | B | B2] images of one stage
  static constexpr int X6S_FLOATS = SMAML_DUAL_X6S_STAGES * X6S_BYTES / 4;
  static constexpr int FLOATS = C::X6S ? (X6S_FLOATS > C::BM * C::BN ? X6S_FLOATS : C::BM * C::BN)
                                       : 2 * (2 * C::A_STAGE + 2 * C::B_STAGE);
};

template <class C, bool A2, bool PRIMAL = true>
__device__ __forceinline__ void dual_mma(const float* st, int arow, int brow, int h, Acc<C>& accp, Acc<C>& acct) {
  constexpr int BKc = C::BK;
  constexpr int SA = C::A_STAGE, SB = C::B_STAGE;
  if constexpr (C::X6) {
#pragma unroll
  for (int s = 0; s < BKc / 16; ++s) {
    Split3 a[C::WTM], a2[C::WTM];
#pragma unroll
    for (int i = 0; i < C::WTM; ++i) {
      a[i] = split3(frag4<C::A_KC, C::LDA, BKc>(st, arow + 32 * i, h, 2 * s),
                    frag4<C::A_KC, C::LDA, BKc>(st, arow + 32 * i, h, 2 * s + 1));
      if (A2)
        a2[i] = split3(frag4<C::A_KC, C::LDA, BKc>(st + SA, arow + 32 * i, h, 2 * s),
                       frag4<C::A_KC, C::LDA, BKc>(st + SA, arow + 32 * i, h, 2 * s + 1));
    }
#pragma unroll
    for (int j = 0; j < C::WTN; ++j) {
      const Split3 b2 = split3(frag4<C::B_KC, C::LDB, BKc>(st + 2 * SA + SB, brow + 32 * j, h, 2 * s),
                               frag4<C::B_KC, C::LDB, BKc>(st + 2 * SA + SB, brow + 32 * j, h, 2 * s + 1));
#pragma unroll
      for (int i = 0; i < C::WTM; ++i) acct.v[i][j] = mfma_x6(a[i], b2, acct.v[i][j]);
      if (PRIMAL || A2) {
        const Split3 b = split3(frag4<C::B_KC, C::LDB, BKc>(st + 2 * SA, brow + 32 * j, h, 2 * s),
                                frag4<C::B_KC, C::LDB, BKc>(st + 2 * SA, brow + 32 * j, h, 2 * s + 1));
#pragma unroll
        for (int i = 0; i < C::WTM; ++i) {
          if (PRIMAL) accp.v[i][j] = mfma_x6(a[i], b, accp.v[i][j]);
          if (A2) acct.v[i][j] = mfma_x6(a2[i], b, acct.v[i][j]);
        }
      }
    }
  }
  } else {
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
}

// Staged split of the four operand tiles (C::X6S): images [A | A2 | B | B2] per stage. With one
// stage (SMAML_DUAL_X6S_STAGES = 1) the next K-tile waits in registers during the MFMAs and is
// stored between two barriers, which keeps the LDS at the epilogue's BM x BN floats.
template <class C, bool PRIMAL, class LA, class LA2, class LB, class LB2>
__device__ __forceinline__ void gemm_dual_mainloop_x6s(const LA& la, const LA2& la2, const LB& lb, const LB2& lb2,
                                                       int m0, int n0, int K, int a2_kbeg, Acc<C>& accp,
                                                       Acc<C>& acct, float* smem) {
  constexpr int BKc = C::BK;
  constexpr int SA = C::AImg::BYTES, SB = C::BImg::BYTES;
  constexpr int STAGE = 2 * SA + 2 * SB;
  constexpr int NST = SMAML_DUAL_X6S_STAGES;
  char* st0 = reinterpret_cast<char*>(smem);
  const int nkt = (K + BKc - 1) / BKc;
  if (nkt <= 0) return;
  const int wave = threadIdx.x >> 6;
  const int wm = wave / C::WAVES_N, wn = wave % C::WAVES_N;
  float4 ra[C::A_F4], ra2[C::A_F4];
  BStage<C, LB> rb;
  BStage<C, LB2> rb2;
  static_assert(!has_dma_image<LB>::value && !has_dma_image<LB2>::value, "dual mainloop: f32 B operands");
  auto fetch = [&](int k0) {
    fetch_tile<C::BM, C::A_F4, C::NTH, C::A_KC, BKc>(la, m0, k0, ra);
    if (k0 >= a2_kbeg) fetch_tile<C::BM, C::A_F4, C::NTH, C::A_KC, BKc>(la2, m0, k0, ra2);
    rb.fetch(lb, n0, k0, nullptr);
    rb2.fetch(lb2, n0, k0, nullptr);
  };
  auto store = [&](char* st, int k0) {
    store_tile_x6<C::BM, C::A_F4, C::NTH, C::A_KC, BKc, C::MSW>(st, ra);
    if (k0 >= a2_kbeg) store_tile_x6<C::BM, C::A_F4, C::NTH, C::A_KC, BKc, C::MSW>(st + SA, ra2);
    rb.store(st + 2 * SA);
    rb2.store(st + 2 * SA + SB);
  };
  auto mma = [&](const char* st, bool a2on) {
    if constexpr (!PRIMAL) {
      // tangent only: all A.B2 products of the step, then all A2.B ones, so only one of A / A2 (and
      // one B fragment) is live at a time; per accumulator the order (A.B2 before A2.B) is unchanged
#pragma unroll
      for (int s = 0; s < BKc / 16; ++s) {
        {
          Split3 a[C::WTM];
#pragma unroll
          for (int i = 0; i < C::WTM; ++i) a[i] = frag_x6<C::BM, C::A_KC, BKc, C::MSW>(st, wm * (C::WTM * 32) + 32 * i, s);
#pragma unroll
          for (int j = 0; j < C::WTN; ++j) {
            const Split3 b2 = frag_x6<C::BN, C::B_KC, BKc, C::MSW>(st + 2 * SA + SB, wn * (C::WTN * 32) + 32 * j, s);
#pragma unroll
            for (int i = 0; i < C::WTM; ++i) acct.v[i][j] = mfma_x6(a[i], b2, acct.v[i][j]);
          }
        }
        if (a2on) {
          Split3 a2[C::WTM];
#pragma unroll
          for (int i = 0; i < C::WTM; ++i)
            a2[i] = frag_x6<C::BM, C::A_KC, BKc, C::MSW>(st + SA, wm * (C::WTM * 32) + 32 * i, s);
#pragma unroll
          for (int j = 0; j < C::WTN; ++j) {
            const Split3 b = frag_x6<C::BN, C::B_KC, BKc, C::MSW>(st + 2 * SA, wn * (C::WTN * 32) + 32 * j, s);
#pragma unroll
            for (int i = 0; i < C::WTM; ++i) acct.v[i][j] = mfma_x6(a2[i], b, acct.v[i][j]);
          }
        }
      }
      return;
    }
#pragma unroll
    for (int s = 0; s < BKc / 16; ++s) {
      Split3 a[C::WTM], a2[C::WTM];
#pragma unroll
      for (int i = 0; i < C::WTM; ++i) {
        a[i] = frag_x6<C::BM, C::A_KC, BKc, C::MSW>(st, wm * (C::WTM * 32) + 32 * i, s);
        if (a2on) a2[i] = frag_x6<C::BM, C::A_KC, BKc, C::MSW>(st + SA, wm * (C::WTM * 32) + 32 * i, s);
      }
#pragma unroll
      for (int j = 0; j < C::WTN; ++j) {
        const int br = wn * (C::WTN * 32) + 32 * j;
        const Split3 b2 = frag_x6<C::BN, C::B_KC, BKc, C::MSW>(st + 2 * SA + SB, br, s);
#pragma unroll
        for (int i = 0; i < C::WTM; ++i) acct.v[i][j] = mfma_x6(a[i], b2, acct.v[i][j]);
        if (PRIMAL || a2on) {
          const Split3 b = frag_x6<C::BN, C::B_KC, BKc, C::MSW>(st + 2 * SA, br, s);
#pragma unroll
          for (int i = 0; i < C::WTM; ++i) {
            if (PRIMAL) accp.v[i][j] = mfma_x6(a[i], b, accp.v[i][j]);
            if (a2on) acct.v[i][j] = mfma_x6(a2[i], b, acct.v[i][j]);
          }
        }
      }
    }
  };
  fetch(0);
  store(st0, 0);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * BKc;
    const bool more = kt + 1 < nkt;
    if (more) fetch(k0 + BKc);
    const char* st = st0 + (NST == 1 ? 0 : (kt & 1) * STAGE);
#if SMAML_PRIO
    __builtin_amdgcn_s_setprio(1);
#endif
    if (k0 >= a2_kbeg)
      mma(st, true);
    else
      mma(st, false);
#if SMAML_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    if (more) {
      if (NST == 1) __syncthreads();  // every wave has read the stage
      store(st0 + (NST == 1 ? 0 : ((kt + 1) & 1) * STAGE), k0 + BKc);
    }
    __syncthreads();
  }
}

// PRIMAL = false: tangent only (acc_t += A2 . B + A . B2), acc_p untouched -- the primal
// product is already stored (second-order sweep with the inner step's activations kept).
template <class C, bool PRIMAL = true, class LA, class LA2, class LB, class LB2>
__device__ __forceinline__ void gemm_dual_mainloop(const LA& la, const LA2& la2, const LB& lb, const LB2& lb2,
                                                   int m0, int n0, int K, int a2_kbeg, Acc<C>& accp, Acc<C>& acct,
                                                   float* smem) {
  if constexpr (C::X6S) {
    gemm_dual_mainloop_x6s<C, PRIMAL>(la, la2, lb, lb2, m0, n0, K, a2_kbeg, accp, acct, smem);
  } else {
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
}

}  // namespace smaml
