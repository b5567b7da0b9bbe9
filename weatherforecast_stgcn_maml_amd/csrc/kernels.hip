// HIP kernels for the STGCN-LSTM MAML hot path on gfx950 (MI355X).
//
// Reference semantics (file:line in Yalt8826/WeatherForecast_STGCN_MAML):
//   k_gcn_layer        GCNConv x4 + ReLU      hybrid_model.py:60-78, model.py:23-26 (PyG 2.x
//                      gcn_norm; F3: only rows t=0 see neighbours, rows t>=1 are x W^T + b)
//   k_lstm_fwd_step    nn.LSTM cell, gates [i,f,g,o]   hybrid_model.py:42-49,93-102
//   k_head_loss        Linear head + view/reshape + MSELoss (F4 row permutation)
//                      hybrid_model.py:105-115, train_hybrid_maml_v5.py:119,133
//   k_lstm_bwd_step    BPTT of the cell (loss.backward through LSTM)   train_hybrid_maml_v5.py:134
//   k_wgrad            dW_ih | dW_hh | db  as a split-K GEMM over B*N*T rows
//   k_inner_sgd        clip_grad_norm_(1.0) + SGD(lr)   train_hybrid_maml_v5.py:135-139
//   k_adamw            clip + AdamW (outer)             train_hybrid_maml_v5.py:174-179,245-249
//
// Every GEMM-shaped contraction takes f32 operands and accumulates in f32 through gemm_core.h:
// by default as f32-accurate "bf16x6" products on v_mfma_f32_32x32x16_bf16 (each operand split
// into three bf16 pieces, six piece products per 16-k step; gemm_core.h mfma_x6), or with
// -DSMAML_X6=0 on v_mfma_f32_32x32x2_f32. All reductions are in a fixed order (no float
// atomics), so results are bitwise reproducible run to run and across ranks.
#include <cmath>
#include <mutex>
#include <utility>
#include <vector>

#include "kernels.h"
#include "loaders.h"

namespace smaml {

using CfgNT = GemmCfg<128, 128, 2, 2, true, true, 32, SMAML_X6_BWD>;    // C = A . B^T (both k-contiguous)
using CfgGate = GemmCfg<32 * SMAML_GATE_WM, 128 * SMAML_GATE_WN, SMAML_GATE_WM, SMAML_GATE_WN, true, true, SMAML_GATE_BK, SMAML_X6_GATE,
                        SMAML_GATE_NST>;  // LSTM forward: wave = 32 rows x 4 gates
// split-K gate step of small grids (k_lstm_fwd_part / _cell / _cell_q): 128-row tiles whatever the
// fused step uses (config 4 A/B with the bf16x6 products: 256-row 1.137 -> 128-row 1.031 ms per sample-step)
using CfgGateP = GemmCfg<128, 128 * SMAML_GATE_WN, 4, SMAML_GATE_WN, true, true, SMAML_GATE_BK, SMAML_X6_GATE>;
using CfgNN = GemmCfg<64, 128, 2, 2, true, false, SMAML_NN_BK, SMAML_X6_BWD>;  // C = A . B   (B n-contiguous)
// (weight gradients keep the padded MC images: the swizzle's address math measured 502 -> 509 ms there,
// profiles/r03_ab_wide_swizzle_crecompute.log, and their LDS sets no occupancy: one workgroup per CU)
using CfgTN = GemmCfg<SMAML_TN_BM, SMAML_TN_BN, SMAML_TN_WM, SMAML_TN_WN, false, false, SMAML_TN_BK, SMAML_X6_WGRAD,
                      SMAML_TN_NST, false>;  // C = A^T . B (split-K weight grads)

// ------------------------------------------------------------------------------------
// Block-wide deterministic sum (fixed shuffle tree + fixed wave order).
__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0) {
    for (int i = 0; i < NT / 64; ++i) s += red[i];
  }
  return s;
}

__device__ __forceinline__ double block_sum_d(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0) {
    for (int i = 0; i < NT / 64; ++i) s += red[i];
  }
  return s;
}

// ====================================================================================
// GCN layer: out = relu( (A_hat X) W^T + b ), A_hat applied to the first N rows of every
// sample (t = 0 block) via an ELL gather in the A-operand prologue (aggregate-then-
// transform), identity elsewhere (F3).
struct GcnA {
  const float* const* tab;  // layer 1: per-sample window pointers into the feature stream
  const float* buf;         // layers 2-4: [g][rows_per_sample][cin]
  int64_t sstride;
  const int* ec;
  const float* ev;
  FastDiv rps_div;
  int rps, ell_rows, cin, R;
  __device__ __forceinline__ float4 operator()(int r, int k) const {
    if (r >= R || k >= cin) return f4zero();
    const int g = (int)rps_div.div((uint32_t)r), q = r - g * rps;
    const float* base = tab ? tab[g] : buf + (int64_t)g * sstride;
    if (q < ell_rows) {
      float4 s = f4zero();
#pragma unroll
      for (int e = 0; e < ELLW; ++e) {
        const float wv = ev[q * ELLW + e];
        if (wv != 0.f) s = fma4(wv, ld4(base + (int64_t)ec[q * ELLW + e] * cin + k), s);
      }
      return s;
    }
    return ld4(base + (int64_t)q * cin + k);
  }
};

// Rows with no neighbours (t >= 1, F3): layer 1 reads the sample's window, layers 2-4 the
// previous layer's [g][rps][cin] buffer, which is simply row-major [R][cin].
struct GcnPlain {
  const float* const* tab;
  const float* buf;
  FastDiv rps_div;
  int rps, cin, R;
  __device__ __forceinline__ float4 operator()(int r, int k) const {
    if (r >= R || k >= cin) return f4zero();
    if (buf) return ld4(buf + (int64_t)r * cin + k);
    const int g = (int)rps_div.div((uint32_t)r);
    return ld4(tab[g] + (int64_t)(r - g * rps) * cin + k);
  }
};

// 8 waves, 128 rows x 256 cols: one workgroup covers a row block's whole Hc=256 output,
// so each input row is read once.
using CfgGcn = GemmCfg<128, 256, 2, 4, true, true, SMAML_GCN_BK, SMAML_X6_GCN>;

__global__ __launch_bounds__(CfgGcn::NTH) void k_gcn_layer(GcnA la, RowMajorKC lb, const float* __restrict__ bias,
                                                           float* __restrict__ out, int cout, int remap, int relu,
                                                           int T, int N, int B, FastDiv ndiv, FastDiv bdiv, Drop dr,
                                                           uint32_t dsite, int drps) {
  __shared__ float smem[CfgGcn::SMEM_FLOATS];
  const int m0 = blockIdx.x * CfgGcn::BM, n0 = blockIdx.y * CfgGcn::BN;
  Acc<CfgGcn> acc;
  acc.zero();
  // only tiles that reach a sample's t = 0 block (its first N rows) need the ELL gather
  const int q0 = m0 - (int)la.rps_div.div((uint32_t)m0) * la.rps;
  if (q0 < la.ell_rows || q0 + CfgGcn::BM > la.rps) {
    gemm_mainloop<CfgGcn, SMAML_IGLP>(la, lb, m0, n0, 0, la.cin, acc, smem);
  } else if (la.buf && la.cin % CfgGcn::BK == 0) {
    // layers 2-4 away from the t = 0 rows: plain row-major operands, branch-free tile loaders
    gemm_mainloop<CfgGcn, SMAML_IGLP>(SegKCt<1>{{la.buf}, {la.cin}, la.R}, SegKCt<1>{{lb.p}, {lb.K}, lb.rows}, m0,
                                      n0, 0, la.cin, acc, smem);
  } else {
    const GcnPlain lp{la.tab, la.buf, la.rps_div, la.rps, la.cin, la.R};
    gemm_mainloop<CfgGcn, SMAML_IGLP>(lp, lb, m0, n0, 0, la.cin, acc, smem);
  }
  const int64_t M = (int64_t)B * N;
  float bc[CfgGcn::WTN];
#pragma unroll
  for (int j = 0; j < CfgGcn::WTN; ++j) {
    const int c = n0 + acc_col<CfgGcn>(j);
    bc[j] = c < cout ? bias[c] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < CfgGcn::WTM; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + acc_row<CfgGcn>(i, r);
      if (row >= la.R) continue;
      uint64_t didx = 0;  // dropout element index of (row, column 0)
      if (dr.gcn()) {
        const int g = (int)la.rps_div.div((uint32_t)row), q = row - g * la.rps;
        const int z = (int)bdiv.div((uint32_t)g), s = g - z * B;
        didx = (((uint64_t)dr.task_id[z] * B + s) * drps + q) * cout;
      }
      int64_t orow = row;
      if (remap) {  // [g][t*N+n] -> [z][t][s*N+n]
        const int g = (int)la.rps_div.div((uint32_t)row), q = row - g * la.rps;
        const int z = (int)bdiv.div((uint32_t)g), s = g - z * B;
        const int t = (int)ndiv.div((uint32_t)q), n = q - t * N;
        orow = ((int64_t)z * T + t) * M + (int64_t)s * N + n;
      }
      float* o = out + orow * cout;
#pragma unroll
      for (int j = 0; j < CfgGcn::WTN; ++j) {
        const int c = n0 + acc_col<CfgGcn>(j);
        if (c >= cout) continue;
        float v = acc.v[i][j][r] + bc[j];
        if (relu) v = fmaxf(v, 0.f);
        if (dr.gcn()) v = drop_keep(dsite, didx + c, dr.thr_gcn) ? v * dr.sc_gcn : 0.f;
        o[c] = v;
      }
    }
}

void launch_gcn_layer(hipStream_t s, const Dims& d, int layer, int Zb, int B, const float* const* xtab,
                      const float* src, float* dst, bool remap_lstm, bool relu, const float* W,
                      const float* b, int cin, int cout, const int* ell_c, const float* ell_v,
                      int rows_per_sample, int ell_rows, const Drop* drop, int drop_rps) {
  // train-mode dropout after the ReLU of conv1..conv3 (hybrid_model.py:67,70,73)
  Drop dr{};
  uint32_t dsite = 0;
  if (drop && drop->gcn() && layer < 3) {
    dr = *drop;
    dsite = drop_site(dr.seed, 1, dr.step, layer);
  }
  GcnA la;
  la.tab = xtab;
  la.buf = src;
  la.sstride = (int64_t)rows_per_sample * cin;
  la.ec = ell_c;
  la.ev = ell_v;
  la.rps_div = FastDiv((uint32_t)rows_per_sample);
  la.rps = rows_per_sample;
  la.ell_rows = ell_rows;
  la.cin = cin;
  la.R = Zb * rows_per_sample;
  RowMajorKC lb{W, cout, cin};
  dim3 grid((la.R + CfgGcn::BM - 1) / CfgGcn::BM, (cout + CfgGcn::BN - 1) / CfgGcn::BN);
  k_gcn_layer<<<grid, CfgGcn::NTH, 0, s>>>(la, lb, b, dst, cout, remap_lstm ? 1 : 0, relu ? 1 : 0, d.T, d.N, B,
                                           FastDiv((uint32_t)d.N), FastDiv((uint32_t)B), dr, dsite,
                                           drop_rps > 0 ? drop_rps : rows_per_sample);
}

// ====================================================================================
// LSTM forward step (layer l, time t) for all tasks z (blockIdx.z):
//   pre[m, g*H+j] = [x_t | h_{t-1}][m] . [W_ih | W_hh][g*H+j] + b_ih + b_hh
// Column tile = 32 hidden units x 4 gates, so each lane holds i,f,g,o of the same
// (row, unit) in the same accumulator register and the cell update is in-register.
template <int H, bool DROP = false>
struct LstmFwdA {
  const float* X;   // layer input at time t: [M][cin]
  const float* Hp;  // h_{t-1}: [M][H] (nullptr at t = 0)
  int M, cin;
  XDrop d;          // DROP: x = drop(h_{l-1})
  __device__ __forceinline__ float4 operator()(int m, int k) const {
    if (m >= M) return f4zero();
    if (k < cin) return DROP ? d.apply(ld4(X + (int64_t)m * cin + k), m, k) : ld4(X + (int64_t)m * cin + k);
    k -= cin;
    if (!Hp || k >= H) return f4zero();
    return ld4(Hp + (int64_t)m * H + k);
  }
};

template <int H>
struct LstmFwdB {  // logical row n = ug*128 + g*32 + jj  ->  weight row g*H + ug*32 + jj
  const float* Wih;
  const float* Whh;
  int cin;
  __device__ __forceinline__ float4 operator()(int n, int k) const {
    const int ug = n >> 7, rem = n & 127, g = rem >> 5, j = ug * 32 + (rem & 31);
    if (j >= H) return f4zero();
    const int row = g * H + j;
    if (k < cin) return ld4(Wih + (int64_t)row * cin + k);
    k -= cin;
    if (k >= H) return f4zero();
    return ld4(Whh + (int64_t)row * H + k);
  }
};

// Per-task slabs are addressed with 32-bit offsets (T*M*4H < 2^31 is checked at reserve).
// Cell epilogue of one gate tile (acc = the i, f, g, o pre-activations of 32 units x 32 rows
// per wave, bias not yet added): gates, c_t = f c_{t-1} + i g, h_t = o tanh(c_t).
template <int H, bool PRE = false, class CfgGate = ::smaml::CfgGate>
__device__ __forceinline__ void fwd_cell(const Acc<CfgGate>& acc, const float* __restrict__ th, const LayerOff& lo,
                                         float* __restrict__ Gz, float* __restrict__ Cz, float* __restrict__ Hz,
                                         int m0, int ug, int t, int M) {
  constexpr int UPB = CfgGate::WAVES_N;
  const int j = (ug * UPB + (int)(threadIdx.x >> 6) % UPB) * 32 + (threadIdx.x & 31);
  if (j >= H) return;
  float bsum[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) bsum[g] = th[lo.bih + g * H + j] + th[lo.bhh + g * H + j];
  const int rb = m0 + acc_row<CfgGate>(0, 0);
  const bool full = m0 + CfgGate::BM <= M;
  const uint32_t tM = (uint32_t)t * (uint32_t)M;
  // PRE: c_{t-1} of all 16 rows before the first store: the stores (slab t) cannot alias these
  // loads (slab t-1), but the compiler cannot prove it and serialises load latency row by row.
  float cpv[16];
  if constexpr (PRE) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = rb + racc(r);
      cpv[r] = (t > 0 && (full || m < M)) ? ldb(Cz, 4u * ((tM - (uint32_t)M + (uint32_t)m) * H + j)) : 0.f;
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = rb + racc(r);
    if (!full && m >= M) continue;
    const uint32_t row = tM + (uint32_t)m;
    const uint32_t oh = row * H + j;
    const uint32_t og = row * (4 * H) + j;
    const float gi = sigmoidf_(acc.v[0][0][r] + bsum[0]);
    const float gf = sigmoidf_(acc.v[0][1][r] + bsum[1]);
    const float gg = tanhf_(acc.v[0][2][r] + bsum[2]);
    const float go = sigmoidf_(acc.v[0][3][r] + bsum[3]);
    const float cp = PRE ? cpv[r] : (t > 0 ? ldb(Cz, 4u * (oh - (uint32_t)M * H)) : 0.f);
    const float c = lstm_cell_c(gi, gf, gg, cp);
    const float h = go * tanhf_(c);
    stb(Gz, 4u * (og), gi);
    stb(Gz, 4u * (og + H), gf);
    stb(Gz, 4u * (og + 2 * H), gg);
    stb(Gz, 4u * (og + 3 * H), go);
    stb(Cz, 4u * (oh), c);
    stb(Hz, 4u * (oh), h);
  }
}

// fwd_cell through the transposed epilogue (loaders.h gate_epilogue_t): per item (row, 4 units)
// one 16-B c_{t-1} load and six 16-B stores (i, f, g, o, c, h). XG: the pre-activations also get the
// row's XgDedup entries (layer 0's input projection, xg = the step's block of window rows): four more
// 16-B loads per item.
template <int H, class CG, bool XG = false>
__device__ __forceinline__ void fwd_cell_t(const Acc<CG>& acc, const float* __restrict__ th, const LayerOff& lo,
                                           float* __restrict__ Gz, float* __restrict__ Cz, float* __restrict__ Hz,
                                           int m0, int ug, int t, int M, float* smem, const float* xg = nullptr) {
  const int j = ug * 32 + (int)(threadIdx.x & 31);
  float bsum[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) bsum[g] = j < H ? th[lo.bih + g * H + j] + th[lo.bhh + g * H + j] : 0.f;
  const bool full = m0 + CG::BM <= M, past = t > 0;
  const uint32_t tM = (uint32_t)t * (uint32_t)M, pM = past ? (uint32_t)M * H : 0u;
  auto coords = [&](int ml, int u, int& m, int& jq) {
    m = m0 + ml;
    jq = ug * 32 + u;
    if (!full) m = min(m, M - 1);  // clamped rows read a valid address (not stored)
    jq = min(jq, H - 4);
  };
  gate_epilogue_t<CG>(
      acc, bsum, smem,
      [&](int ml, int u) {
        int m, jq;
        coords(ml, u, m, jq);
        return ldo(Cz, 4u * ((tM + (uint32_t)m) * H - pM + (uint32_t)jq));  // c_{t-1} (t = 0: selected out)
      },
      [&](int ml, int u, const float4 (&pre0)[4], const float4& cpv) {
        if ((!full && m0 + ml >= M) || ug * 32 + u >= H) return;
        const uint32_t row = tM + (uint32_t)(m0 + ml), jq = (uint32_t)(ug * 32 + u);
        const float4 cp = sel4(past, cpv);
        float4 pre[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          pre[g] = pre0[g];
          if (XG && xg) {
            const float4 x = ldo(xg, 4u * ((uint32_t)(m0 + ml) * (4 * H) + (uint32_t)(g * H) + jq));
            pre[g] = make_float4(pre[g].x + x.x, pre[g].y + x.y, pre[g].z + x.z, pre[g].w + x.w);
          }
        }
        float4 gi, gf, gg, go, c, hh;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float i_ = sigmoidf_(f4get(pre[0], e)), f_ = sigmoidf_(f4get(pre[1], e));
          const float g_ = tanhf_(f4get(pre[2], e)), o_ = sigmoidf_(f4get(pre[3], e));
          const float c_ = lstm_cell_c(i_, f_, g_, f4get(cp, e));
          f4set(gi, e, i_);
          f4set(gf, e, f_);
          f4set(gg, e, g_);
          f4set(go, e, o_);
          f4set(c, e, c_);
          f4set(hh, e, o_ * tanhf_(c_));
        }
        const uint32_t og = 4u * (row * (4 * H) + jq), oh = 4u * (row * H + jq);
        sto(Gz, og, gi);
        sto(Gz, og + 4u * H, gf);
        sto(Gz, og + 8u * H, gg);
        sto(Gz, og + 12u * H, go);
        sto(Cz, oh, c);
        sto(Hz, oh, hh);
      });
}

#ifndef SMAML_DIAG_FWD
#define SMAML_DIAG_FWD 0  // timing diagnostics only (wrong results): 1 = forward step without its epilogue,
#endif                    // 2 = without its GEMM
// XG (xg != null): layer 0's input projection of this step's windows comes from the XgDedup table
// (launch_xg_dedup): the accumulators start from it and the K loop covers the recurrent segment only.
template <int H, bool DROP, bool IMG = false>
__device__ __forceinline__ void lstm_fwd_step(const float* __restrict__ F, float* __restrict__ HsAll,
                                              float* __restrict__ CsAll, float* __restrict__ GsAll, int64_t lsz,
                                              const float* __restrict__ theta, int64_t tstride, FwdWave wv, int T,
                                              int M, const Drop& dr, float* smem, const GateImgs* gi = nullptr,
                                              const float* xg = nullptr, int64_t xg_zstride = 0, int xg_N = 0) {
  int l, t, b0;
  LayerOff lo;
  const Blk bk = xcd_block();
  wave_problem(wv, bk.x, l, t, lo, b0);
  const float* X = l == 0 ? F : HsAll + (int64_t)(l - 1) * lsz;
  float* Hs = HsAll + (int64_t)l * lsz;
  float* Cs = CsAll + (int64_t)l * lsz;
  float* Gs = GsAll + (int64_t)l * lsz * 4;
  const int z = bk.z;
  const float* th = theta + (int64_t)z * tstride;
  const int cin = lo.cin;
  const int64_t slab = (int64_t)z * T * M;
  float* Gz = Gs + slab * (4 * H);
  float* Cz = Cs + slab * H;
  float* Hz = Hs + slab * H;
  const float* Hp = t > 0 ? Hz + (int64_t)(t - 1) * M * H : nullptr;
  LstmFwdB<H> lb{th + lo.wih, th + lo.whh, cin};
  int tm, ug;
  constexpr int UPB = CfgGate::WAVES_N;  // 32-unit groups per workgroup
  if (!gate_tile(bk.x - b0, wv.ntm ? wv.ntm : (M + CfgGate::BM - 1) / CfgGate::BM, (H + 32 * UPB - 1) / (32 * UPB), tm,
                 ug))
    return;
  tm += wv.tm0;
  const int m0 = tm * CfgGate::BM, n0 = ug * CfgGate::BN;
  Acc<CfgGate> acc;
  int kbeg = 0;  // (XG: the K loop starts past the input segment)
  acc.zero();
  // (the table is added in the epilogue: loading it into the accumulators before the K loop keeps 64 more
  // registers live through the loop's prologue and spills)
  const float* xgt = !DROP && xg && l == 0 ? xg + (int64_t)z * xg_zstride + xg_dedup_row0(t, M, xg_N) * (4 * H) : nullptr;
  if (xgt) kbeg = cin;
  if (SMAML_DIAG_FWD == 2) {  // timing diagnostic: cell epilogue only (no K loop)
    fwd_cell_t<H, CfgGate, !DROP>(acc, th, lo, Gz, Cz, Hz, m0, ug, t, M, smem, xgt);
    return;
  }
  if (DROP && l > 0) {
    // nn.LSTM inter-layer dropout: layer l reads drop(h_{l-1, t})
    const XDrop xd{drop_site(dr.seed, 2, dr.step, l - 1), dr.thr_lstm, dr.sc_lstm,
                   ((uint64_t)dr.task_id[z] * T + t) * M * H, H};
    LstmFwdA<H, true> la{X + (slab + (int64_t)t * M) * cin, Hp, M, cin, xd};
    gemm_mainloop<CfgGate>(la, lb, m0, n0, 0, cin + (t > 0 ? H : 0), acc, smem);
  } else {
    const SegKCt<2> la{{X + (slab + (int64_t)t * M) * cin, Hp}, {cin, H}, M};
    if constexpr (IMG) {  // weight tiles as pre-split images (launch_split_gate)
      const char* ib = gi->th + (int64_t)z * gi->tstride;
      int64_t o0 = 0, o1 = 0;  // (layer l's segment offsets, selected with scalar compares)
#pragma unroll
      for (int q = 0; q < MAX_LAYERS; ++q)
        if (q == l) {
          o0 = gi->off[q][0];
          o1 = gi->off[q][1];
        }
      const SegGateImg<2> lbi{{ib + o0, ib + o1}, {cin, H}};
      gemm_mainloop<CfgGate>(la, lbi, m0, n0, kbeg, cin + (t > 0 ? H : 0), acc, smem);
    } else {
      const SegGateBt<2> lbt{{th + lo.wih, th + lo.whh}, {cin, H}, H};
      gemm_mainloop<CfgGate>(la, lbt, m0, n0, kbeg, cin + (t > 0 ? H : 0), acc, smem);
    }
  }

  if (SMAML_DIAG_FWD == 1) {  // timing diagnostic: GEMM phase only (every accumulator kept live)
    float sum = 0.f;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int r = 0; r < 16; ++r) sum += acc.v[0][g][r];
    if (sum == 12345.678f) Gz[threadIdx.x] = sum;  // (never true in practice; the MFMAs stay)
    return;
  }
  if constexpr (SMAML_FWD_EPI_T && CfgGate::WAVES_N == 1) {
    fwd_cell_t<H, CfgGate, !DROP>(acc, th, lo, Gz, Cz, Hz, m0, ug, t, M, smem, xgt);
  } else {
    static_assert(!SMAML_XG_DEDUP_DEFAULT || (SMAML_FWD_EPI_T && CfgGate::WAVES_N == 1),
                  "the XG table is added by the transposed epilogue");
    fwd_cell<H, SMAML_EPI_PRELOAD_FWD != 0>(acc, th, lo, Gz, Cz, Hz, m0, ug, t, M);
  }
}

double fwd_wave(const Dims& d, const Work& w, const ParamOff& po, int diag, int blocks_per_problem, bool dual,
                FwdWave& wv) {
  double fl = 0.0;
  int n = 0, off = 0;
  for (int l = 0; l < d.L; ++l) {
    const int t = diag - l;
    if (t < 0 || t >= d.T) continue;
    const LayerOff& lo = po.lay[l];
    wv.l[n] = l;
    wv.t[n] = t;
    wv.lo[n] = lo;
    wv.off[n] = off;
    off += blocks_per_problem;
    ++n;
    const double k1 = lo.cin + (t > 0 ? d.H : 0);
    const double k2 = (l > 0 ? 2.0 : 1.0) * lo.cin + (t > 0 ? 2.0 * d.H : 0.0);
    fl += 2.0 * w.Z * w.M * 4 * d.H * (dual ? k1 + k2 : k1);
  }
  wv.n = n;
  wv.off[n] = off;
  for (int q = n + 1; q <= MAX_LAYERS; ++q) wv.off[q] = off;
  return fl;
}

// The dropout variant holds the mask state beside the 4-gate tile: it gets the register budget
// of 3 waves/SIMD instead of 4 (no spill).
template <int H, bool IMG>
__global__ SMAML_GATE_ATTR __launch_bounds__(CfgGate::NTH) void k_lstm_fwd_step(const float* __restrict__ F, float* __restrict__ HsAll,
                                                      float* __restrict__ CsAll, float* __restrict__ GsAll,
                                                      int64_t lsz, const float* __restrict__ theta, int64_t tstride,
                                                      FwdWave wv, int T, int M, Drop dr, GateImgs gi, XgDedup xd) {
  __shared__ float smem[CfgGate::SMEM_FLOATS];
  lstm_fwd_step<H, false, IMG>(F, HsAll, CsAll, GsAll, lsz, theta, tstride, wv, T, M, dr, smem, &gi, xd.xg, xd.zstride,
                               xd.N);
}

// Layer 0's input projection of a step whose every task reads B consecutive windows, once per distinct
// stream row (kernels.h XgDedup): out[z][r][g H + j] = F_row(r) . W_ih0[g H + j] with the gate GEMM's own
// tile (CfgGate), column mapping, K order and weight images. The tangent gate kernel starts its
// accumulators from these rows and adds the recurrent segment: bitwise what it computes with the input
// segment in its own K loop. The primal gate kernel adds the row in its epilogue (after the recurrent
// products and the bias; loading it into the accumulators spilled): equal up to f32 rounding. Compact row r: r < M -> F[0][r] (the t = 0 rows, window
// b = r / N); else stream row s = (r - M) / N + 1, read from the (window, step) slot (s - t, t) with
// t = min(s, T - 1) (the GCN wrote every slot of that stream row with the same features).
struct XgRowsA {
  const float* F;  // [T][M][cin] (one task)
  int M, N, T, cin, rows;
  FastDiv ndiv;
  int compact;     // F in XgDedup order (Work::fcompact): row r is F's row r
  __device__ __forceinline__ float4 operator()(int r, int k) const {
    r = min(r, rows - 1);
    int64_t row = r;
    if (r >= M && !compact) {
      const int rr = r - M;
      const int s1 = (int)ndiv.div((uint32_t)rr);
      const int s = s1 + 1, t = min(s, T - 1);
      row = (int64_t)t * M + (int64_t)(s - t) * N + (rr - s1 * N);
    }
    return ld4(F + row * cin + k);
  }
};
template <int H, bool IMG>
__global__ SMAML_GATE_ATTR __launch_bounds__(CfgGate::NTH) void k_xg_dedup(const float* __restrict__ F, int64_t f_zstride,
                                                                        XgRowsA a, const float* __restrict__ W,
                                                                        int64_t w_zstride, const char* __restrict__ img,
                                                                        int64_t img_zstride, float* __restrict__ out,
                                                                        int64_t o_zstride) {
  __shared__ float smem[CfgGate::SMEM_FLOATS];
  const int z = blockIdx.z;
  constexpr int UPB = CfgGate::WAVES_N;
  int tm, ug;
  if (!gate_tile((int)blockIdx.x, (a.rows + CfgGate::BM - 1) / CfgGate::BM, (H + 32 * UPB - 1) / (32 * UPB), tm, ug))
    return;
  const int m0 = tm * CfgGate::BM, n0 = ug * CfgGate::BN;
  a.F = F + (int64_t)z * f_zstride;
  Acc<CfgGate> acc;
  acc.zero();
  if constexpr (IMG)
    gemm_mainloop<CfgGate>(a, SegGateImg<1>{{img + (int64_t)z * img_zstride}, {a.cin}}, m0, n0, 0, a.cin, acc, smem);
  else
    gemm_mainloop<CfgGate>(a, SegGateBt<1>{{W + (int64_t)z * w_zstride}, {a.cin}, H}, m0, n0, 0, a.cin, acc, smem);
  float* o = out + (int64_t)z * o_zstride;
  const float zero[4] = {0.f, 0.f, 0.f, 0.f};
  const bool full = m0 + CfgGate::BM <= a.rows;
  gate_epilogue_t<CfgGate>(
      acc, zero, smem, [&](int, int) { return 0; },
      [&](int ml, int u, const float4 (&pre)[4], int) {
        if ((!full && m0 + ml >= a.rows) || ug * 32 + u >= H) return;
        const uint32_t row = (uint32_t)(m0 + ml), jq = (uint32_t)(ug * 32 + u);
#pragma unroll
        for (int g = 0; g < 4; ++g) sto(o, 4u * (row * (4 * H) + g * H + jq), pre[g]);
      });
}

void launch_xg_dedup(hipStream_t s, const Dims& d, const Work& w, const float* params, int64_t tstride,
                     const ParamOff& po, const char* img, int64_t img_tstride, int64_t img_off, float* out) {
  const int rows = (int)xg_dedup_rows(w.B, d.T, d.N);
  const int ntm = (rows + CfgGate::BM - 1) / CfgGate::BM;
  const int ngrp = (d.H + 32 * CfgGate::WAVES_N - 1) / (32 * CfgGate::WAVES_N);
  dim3 grid(gate_blocks(ntm, ngrp), 1, w.Z);
  const int cin = po.lay[0].cin;
  const XgRowsA a{nullptr, w.M, d.N, d.T, cin, rows, FastDiv((uint32_t)d.N), w.fcompact};
  const int64_t fz = (int64_t)d.T * w.M * cin;
  count_variant(w, V_XG_DEDUP);
  if (img) {
    SMAML_DISPATCH_H(d.H, (k_xg_dedup<HT, true><<<grid, CfgGate::NTH, 0, s>>>(
                              w.F, fz, a, nullptr, 0, img + img_off, img_tstride, out, w.xgd.zstride)));
  } else {
    SMAML_DISPATCH_H(d.H, (k_xg_dedup<HT, false><<<grid, CfgGate::NTH, 0, s>>>(
                              w.F, fz, a, params + po.lay[0].wih, tstride, nullptr, 0, out, w.xgd.zstride)));
  }
}

template <int H>
__global__ __attribute__((amdgpu_waves_per_eu(3))) __launch_bounds__(CfgGate::NTH) void k_lstm_fwd_step_drop(
    const float* __restrict__ F, float* __restrict__ HsAll, float* __restrict__ CsAll, float* __restrict__ GsAll,
    int64_t lsz, const float* __restrict__ theta, int64_t tstride, FwdWave wv, int T, int M, Drop dr) {
  __shared__ float smem[CfgGate::SMEM_FLOATS];
  lstm_fwd_step<H, true>(F, HsAll, CsAll, GsAll, lsz, theta, tstride, wv, T, M, dr, smem);
}

// ---- split-K variant for small grids (batch-1 adaptation: M = N = 441 sequences) ----------
// A step's critical path is one wave's K loop; when the diagonal has too few gate tiles to fill
// the chip, S workgroups share a tile, each over a contiguous range of K-tiles, and write their
// accumulators to a partial slab (w.wpart, lane order); k_lstm_fwd_cell sums the S partials in
// a fixed order (deterministic) and runs the cell epilogue. Dropout-free steps only.
template <class C>
__device__ __forceinline__ float* part_slab(float* part, int S, int split) {
  constexpr int PER = C::WTM * C::WTN * 16 * C::NTH;
  return part + (((int64_t)blockIdx.z * gridDim.x + blockIdx.x) * S + split) * PER;
}
template <class C>
__device__ __forceinline__ void store_part(const Acc<C>& acc, float* slab) {
#pragma unroll
  for (int i = 0; i < C::WTM; ++i)
#pragma unroll
    for (int j = 0; j < C::WTN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int f = ((i * C::WTN + j) * 4 + q) * C::NTH + (int)threadIdx.x;
        st4(slab + 4 * f, make_float4(acc.v[i][j][4 * q], acc.v[i][j][4 * q + 1], acc.v[i][j][4 * q + 2],
                                      acc.v[i][j][4 * q + 3]));
      }
}
template <class C>
__device__ __forceinline__ void add_part(Acc<C>& acc, const float* slab) {
#pragma unroll
  for (int i = 0; i < C::WTM; ++i)
#pragma unroll
    for (int j = 0; j < C::WTN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = ld4(slab + 4 * (((i * C::WTN + j) * 4 + q) * C::NTH + (int)threadIdx.x));
        acc.v[i][j][4 * q] += v.x;
        acc.v[i][j][4 * q + 1] += v.y;
        acc.v[i][j][4 * q + 2] += v.z;
        acc.v[i][j][4 * q + 3] += v.w;
      }
}
// K-tile range [kbeg, kend) of split `split` out of S over a K-long reduction.
__device__ __forceinline__ void split_range(int K, int S, int split, int bk, int& kbeg, int& kend) {
  const int kt = (K + bk - 1) / bk, per = (kt + S - 1) / S;
  kbeg = split * per * bk;
  kend = min(K, kbeg + per * bk);
}

#ifndef SMAML_FWD_PART_NCH
#define SMAML_FWD_PART_NCH 3  // K-tiles per load round trip in the split-K gate step (0: double-buffered loop)
#endif
#ifndef SMAML_BWD_PART_NCH
#define SMAML_BWD_PART_NCH 8  // same, split-K BPTT step
#endif
template <class C, int NCH>
constexpr int part_smem_floats() {
  return NCH > 0 && chunked_smem_floats<C, (NCH > 0 ? NCH : 1)>() > C::SMEM_FLOATS
             ? chunked_smem_floats<C, (NCH > 0 ? NCH : 1)>()
             : C::SMEM_FLOATS;
}
template <class C, int NCH, class LA, class LB>
__device__ __forceinline__ void part_mainloop(const LA& la, const LB& lb, int m0, int n0, int kbeg, int kend,
                                              Acc<C>& acc, float* smem) {
  if constexpr (NCH > 0)
    gemm_mainloop_chunked<C, NCH>(la, lb, m0, n0, kbeg, kend, acc, smem);
  else
    gemm_mainloop<C>(la, lb, m0, n0, kbeg, kend, acc, smem);
}

template <int H>
__global__ __launch_bounds__(CfgGateP::NTH) void k_lstm_fwd_part(
    const float* __restrict__ F, const float* __restrict__ HsAll, int64_t lsz, const float* __restrict__ theta,
    int64_t tstride, FwdWave wv, int T, int M, int S, float* __restrict__ part) {
  __shared__ float smem[part_smem_floats<CfgGateP, SMAML_FWD_PART_NCH>()];
  int l, t, b0;
  LayerOff lo;
  wave_problem(wv, (int)blockIdx.x, l, t, lo, b0);
  const float* X = l == 0 ? F : HsAll + (int64_t)(l - 1) * lsz;
  const int z = blockIdx.z;
  const float* th = theta + (int64_t)z * tstride;
  const int cin = lo.cin;
  const int64_t slab = (int64_t)z * T * M;
  const float* Hp = t > 0 ? HsAll + (int64_t)l * lsz + (slab + (int64_t)(t - 1) * M) * H : nullptr;
  int tm, ug;
  constexpr int UPB = CfgGateP::WAVES_N;
  if (!gate_tile((int)blockIdx.x - b0, (M + CfgGateP::BM - 1) / CfgGateP::BM, (H + 32 * UPB - 1) / (32 * UPB), tm, ug))
    return;
  const int m0 = tm * CfgGateP::BM, n0 = ug * CfgGateP::BN;
  int kbeg, kend;
  split_range(cin + (t > 0 ? H : 0), S, (int)blockIdx.y, CfgGateP::BK, kbeg, kend);
  Acc<CfgGateP> acc;
  acc.zero();
  if (kbeg < kend) {
    const SegGateBt<2> lb{{th + lo.wih, th + lo.whh}, {cin, H}, H};
    const SegKCt<2> la{{X + (slab + (int64_t)t * M) * cin, Hp}, {cin, H}, M};
    part_mainloop<CfgGateP, SMAML_FWD_PART_NCH>(la, lb, m0, n0, kbeg, kend, acc, smem);
  }
  store_part<CfgGateP>(acc, part_slab<CfgGateP>(part, S, (int)blockIdx.y));
}

template <int H>
__global__ __launch_bounds__(CfgGateP::NTH) void k_lstm_fwd_cell(float* __restrict__ HsAll, float* __restrict__ CsAll,
                                                               float* __restrict__ GsAll, int64_t lsz,
                                                               const float* __restrict__ theta, int64_t tstride,
                                                               FwdWave wv, int T, int M, int S,
                                                               const float* __restrict__ part) {
  int l, t, b0;
  LayerOff lo;
  wave_problem(wv, (int)blockIdx.x, l, t, lo, b0);
  int tm, ug;
  constexpr int UPB = CfgGateP::WAVES_N;
  if (!gate_tile((int)blockIdx.x - b0, (M + CfgGateP::BM - 1) / CfgGateP::BM, (H + 32 * UPB - 1) / (32 * UPB), tm, ug))
    return;
  Acc<CfgGateP> acc;
  acc.zero();
  float* p0 = const_cast<float*>(part);
  for (int q = 0; q < S; ++q) add_part<CfgGateP>(acc, part_slab<CfgGateP>(p0, S, q));
  const int z = blockIdx.z;
  const int64_t slab = (int64_t)z * T * M;
  fwd_cell<H, true, CfgGateP>(acc, theta + (int64_t)z * tstride, lo, GsAll + (int64_t)l * lsz * 4 + slab * (4 * H),
              CsAll + (int64_t)l * lsz + slab * H, HsAll + (int64_t)l * lsz + slab * H, tm * CfgGateP::BM, ug, t, M);
}

// The same cell step spread over 4x the threads: blockIdx.y = q picks accumulator registers
// 4q..4q+3 (4 rows) of every gate, so each thread's S x 4 partial loads are independent and
// in flight together, then 4 rows' c_{t-1} loads. Sums the partials in the same order as
// k_lstm_fwd_cell (bitwise identical results).
template <int H>
__global__ __launch_bounds__(CfgGateP::NTH) void k_lstm_fwd_cell_q(float* __restrict__ HsAll, float* __restrict__ CsAll,
                                                                 float* __restrict__ GsAll, int64_t lsz,
                                                                 const float* __restrict__ theta, int64_t tstride,
                                                                 FwdWave wv, int T, int M, int S,
                                                                 const float* __restrict__ part) {
  static_assert(CfgGateP::WTM == 1 && CfgGateP::WTN == 4, "one 32-row tile of 4 gates per wave");
  constexpr int PER = CfgGateP::WTM * CfgGateP::WTN * 16 * CfgGateP::NTH;
  constexpr int UPB = CfgGateP::WAVES_N;
  int l, t, b0;
  LayerOff lo;
  wave_problem(wv, (int)blockIdx.x, l, t, lo, b0);
  int tm, ug;
  if (!gate_tile((int)blockIdx.x - b0, (M + CfgGateP::BM - 1) / CfgGateP::BM, (H + 32 * UPB - 1) / (32 * UPB), tm, ug))
    return;
  const int q = blockIdx.y, z = blockIdx.z, tid = threadIdx.x;
  const float* base = part + ((int64_t)z * gridDim.x + blockIdx.x) * S * PER + 4 * (q * CfgGateP::NTH + tid);
  float4 a[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) a[g] = f4zero();
  for (int sp = 0; sp < S; ++sp)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 v = ld4(base + (int64_t)sp * PER + 4 * (g * 4 * CfgGateP::NTH));
      a[g] = make_float4(a[g].x + v.x, a[g].y + v.y, a[g].z + v.z, a[g].w + v.w);
    }
  const float* th = theta + (int64_t)z * tstride;
  const int j = (ug * UPB + (tid >> 6) % UPB) * 32 + (tid & 31);
  if (j >= H) return;
  float bsum[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) bsum[g] = th[lo.bih + g * H + j] + th[lo.bhh + g * H + j];
  const int64_t slab = (int64_t)z * T * M;
  float* Gz = GsAll + (int64_t)l * lsz * 4 + slab * (4 * H);
  float* Cz = CsAll + (int64_t)l * lsz + slab * H;
  float* Hz = HsAll + (int64_t)l * lsz + slab * H;
  const int rb = tm * CfgGateP::BM + acc_row<CfgGateP>(0, 0) + 8 * q;  // row of register 4q
  const uint32_t tM = (uint32_t)t * (uint32_t)M;
  float cpv[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int m = rb + e;
    cpv[e] = (t > 0 && m < M) ? ldb(Cz, 4u * ((tM - (uint32_t)M + (uint32_t)m) * H + j)) : 0.f;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int m = rb + e;
    if (m >= M) continue;
    const uint32_t row = tM + (uint32_t)m;
    const uint32_t oh = row * H + j;
    const uint32_t og = row * (4 * H) + j;
    const float gi = sigmoidf_(f4get(a[0], e) + bsum[0]);
    const float gf = sigmoidf_(f4get(a[1], e) + bsum[1]);
    const float gg = tanhf_(f4get(a[2], e) + bsum[2]);
    const float go = sigmoidf_(f4get(a[3], e) + bsum[3]);
    const float c = lstm_cell_c(gi, gf, gg, cpv[e]);
    const float h = go * tanhf_(c);
    stb(Gz, 4u * (og), gi);
    stb(Gz, 4u * (og + H), gf);
    stb(Gz, 4u * (og + 2 * H), gg);
    stb(Gz, 4u * (og + 3 * H), go);
    stb(Cz, 4u * (oh), c);
    stb(Hz, 4u * (oh), h);
  }
}
#ifndef SMAML_FWD_CELL_Q
#define SMAML_FWD_CELL_Q 1  // split-K gate step's cell kernel over 4x the threads (0: k_lstm_fwd_cell)
#endif

#ifndef SMAML_SPLIT_WGS
#define SMAML_SPLIT_WGS 256  // split while the launch stays within this many workgroups
#endif
// Split count for a launch of `tiles` workgroup tiles over K (max over its problems): enough
// workgroups for ~one per CU, each split keeping >= 4 K-tiles, bounded by the partial slab.
static int small_grid_splits(int64_t tiles, int K, int bk, int64_t per_split_floats, int64_t cap_floats,
                             int smax) {
  int S = 1;
  while (S < smax && tiles * (S * 2) <= SMAML_SPLIT_WGS && (K / bk) / (S * 2) >= 4 &&
         per_split_floats * (S * 2) <= cap_floats)
    S *= 2;
  return S;
}

// Split count of diagonal `diag`'s small-grid (CfgGateP) form: > 1 = the split-K pair or the kw kernel.
static int fwd_wave_splits(const Dims& d, const Work& w, const ParamOff& po, int diag) {
  const int ntmP = (w.M + CfgGateP::BM - 1) / CfgGateP::BM;
  const int ngrpP = (d.H + 32 * CfgGateP::WAVES_N - 1) / (32 * CfgGateP::WAVES_N);
  FwdWave wvP{};
  fwd_wave(d, w, po, diag, gate_blocks(ntmP, ngrpP), false, wvP);
  int kmax = 0;
  for (int q = 0; q < wvP.n; ++q) kmax = std::max(kmax, wvP.lo[q].cin + (wvP.t[q] > 0 ? d.H : 0));
  const int64_t per = (int64_t)wvP.off[wvP.n] * w.Z * CfgGateP::NTH * CfgGateP::WTM * CfgGateP::WTN * 16;
  return small_grid_splits((int64_t)wvP.n * ntmP * ngrpP * w.Z, kmax, CfgGateP::BK, per, w.wpart_floats,
                           w.kn.split_max);
}

bool fwd_wave_kw(const Dims& d, const Work& w, const ParamOff& po, int diag) {
  return !w.drop.lstm() && small_kw_ok(d, w) && fwd_wave_splits(d, w, po, diag) > 1;
}

bool fwd_wave_big(const Dims& d, const Work& w, const ParamOff& po, int diag) {
  return !w.drop.lstm() && fwd_wave_splits(d, w, po, diag) <= 1;
}

void launch_lstm_fwd_wave(hipStream_t s, const Dims& d, const Work& w, int diag, const float* theta,
                          int64_t tstride, const ParamOff& po, double* flops, int chunk, int nch) {
  const int64_t lsz = (int64_t)w.Z * d.T * w.M * d.H;
  const int ntm = (w.M + CfgGate::BM - 1) / CfgGate::BM;
  const int ngrp = (d.H + 32 * CfgGate::WAVES_N - 1) / (32 * CfgGate::WAVES_N);
  FwdWave wv{};
  const double fl = fwd_wave(d, w, po, diag, gate_blocks(ntm, ngrp), false, wv);
  if (flops) *flops = fl;
  if (wv.n == 0) return;
  if (nch > 1) {  // this launch's row tiles only, always on the big tiles (see launch_lstm_bwd_wave)
    const int lo = (int)((int64_t)ntm * chunk / nch), hi = (int)((int64_t)ntm * (chunk + 1) / nch);
    if (hi <= lo) return;
    fwd_wave(d, w, po, diag, gate_blocks(hi - lo, ngrp), false, wv);
    wv.tm0 = lo;
    wv.ntm = hi - lo;
  }
  dim3 grid(wv.off[wv.n], 1, w.Z);
  if (w.drop.lstm()) {
    count_variant(w, V_FWD_DROP);
    SMAML_DISPATCH_H(d.H, k_lstm_fwd_step_drop<HT><<<grid, CfgGate::NTH, 0, s>>>(w.F, w.Hs, w.Cs, w.Gs, lsz, theta,
                                                                                   tstride, wv, d.T, w.M, w.drop));
    return;
  }
  if (nch <= 1) {
    // split-K over the small-grid tile (CfgGateP): its own block offsets per problem
    const int ntmP = (w.M + CfgGateP::BM - 1) / CfgGateP::BM;
    const int ngrpP = (d.H + 32 * CfgGateP::WAVES_N - 1) / (32 * CfgGateP::WAVES_N);
    FwdWave wvP{};
    fwd_wave(d, w, po, diag, gate_blocks(ntmP, ngrpP), false, wvP);
    const dim3 gridP(wvP.off[wvP.n], 1, w.Z);
    const int S = fwd_wave_splits(d, w, po, diag);
    if (S > 1 && small_kw_ok(d, w)) {
      launch_lstm_fwd_kw(s, d, w, diag, theta, tstride, po);
      return;
    }
    if (S > 1) {
      count_variant(w, V_FWD_SPLIT);
      dim3 gp(gridP.x, S, gridP.z);
      SMAML_DISPATCH_H(d.H, k_lstm_fwd_part<HT><<<gp, CfgGateP::NTH, 0, s>>>(w.F, w.Hs, lsz, theta, tstride, wvP,
                                                                               d.T, w.M, S, w.wpart));
      if (SMAML_FWD_CELL_Q) {
        dim3 gq(gridP.x, 4, gridP.z);
        SMAML_DISPATCH_H(d.H, k_lstm_fwd_cell_q<HT><<<gq, CfgGateP::NTH, 0, s>>>(w.Hs, w.Cs, w.Gs, lsz, theta,
                                                                                  tstride, wvP, d.T, w.M, S, w.wpart));
      } else {
        SMAML_DISPATCH_H(d.H, k_lstm_fwd_cell<HT><<<gridP, CfgGateP::NTH, 0, s>>>(w.Hs, w.Cs, w.Gs, lsz, theta,
                                                                                  tstride, wvP, d.T, w.M, S, w.wpart));
      }
      return;
    }
  }
  count_variant(w, V_FWD);
  XgDedup xd = w.xgd;
  if (xd.src != theta) xd.xg = nullptr;  // (a table of other weights is never read)
  if (w.gimg.th && w.gimg_src == theta) {
    count_variant(w, V_FWD_IMG);
    SMAML_DISPATCH_H(d.H, (k_lstm_fwd_step<HT, true><<<grid, CfgGate::NTH, 0, s>>>(
                              w.F, w.Hs, w.Cs, w.Gs, lsz, theta, tstride, wv, d.T, w.M, w.drop, w.gimg, xd)));
  } else {
    SMAML_DISPATCH_H(d.H, (k_lstm_fwd_step<HT, false><<<grid, CfgGate::NTH, 0, s>>>(
                              w.F, w.Hs, w.Cs, w.Gs, lsz, theta, tstride, wv, d.T, w.M, w.drop, w.gimg, xd)));
  }
}

// ---- pre-split gate-GEMM weight images --------------------------------------------------
int64_t gate_img_bytes(const Dims& d, GateImgs* gi) {
  const int nug = (d.H + 31) / 32;
  int64_t off = 0;
  for (int l = 0; l < d.L; ++l)
    for (int sg = 0; sg < 2; ++sg) {
      if (gi) gi->off[l][sg] = off;
      const int w = sg == 0 ? (l == 0 ? d.Hc : d.H) : d.H;
      off += (int64_t)nug * (w / 16) * GATE_IMG_BYTES;
    }
  if (gi) gi->tstride = off;
  return off;
}

// One thread per (task, image, row, 4 k): weight row g*H + ug*32 + jj of image row n = g*32 + jj,
// columns 16 kt + 4 q .. + 3 of the segment; split into three bf16 planes at the staged-split
// store's offsets (gemm_core.h store_tile_x6, KC, BK 16).
__global__ void k_split_gate(const float* __restrict__ theta, int64_t tstride, ParamOff po, int L, int H, int Hc,
                             int nimg, int64_t img_tstride, char* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int z = blockIdx.y;
  if (i >= (int64_t)nimg * 512) return;
  const int q = (int)(i & 3), n = (int)((i >> 2) & 127), img = (int)(i >> 9);
  const int nug = (H + 31) / 32;
  int rem = img, l = 0, sg = 0, w = Hc;
  for (l = 0; l < L; ++l) {
    w = l == 0 ? Hc : H;
    const int a = nug * (w / 16);
    if (rem < a) { sg = 0; break; }
    rem -= a;
    const int b = nug * (H / 16);
    if (rem < b) { sg = 1; w = H; break; }
    rem -= b;
  }
  const int kts = w / 16, ug = rem / kts, kt = rem - ug * kts;
  const LayerOff lo = po.lay[l];
  const float* W = theta + (int64_t)z * tstride + (sg == 0 ? lo.wih : lo.whh);
  const int j = min(ug * 32 + (n & 31), H - 1);
  const float4 v = ld4(W + (int64_t)((n >> 5) * H + j) * w + 16 * kt + 4 * q);
  uint2 p0, p1, p2;
  split4(v, p0, p1, p2);
  constexpr int PLANE = 128 * 32;
  char* o = dst + (int64_t)z * img_tstride + (int64_t)img * GATE_IMG_BYTES + n * 32 + 16 * ((q >> 1) ^ ((n >> 3) & 1)) +
            8 * (q & 1);
  *reinterpret_cast<uint2*>(o) = p0;
  *reinterpret_cast<uint2*>(o + PLANE) = p1;
  *reinterpret_cast<uint2*>(o + 2 * PLANE) = p2;
}

void launch_split_gate(hipStream_t s, const Dims& d, const ParamOff& po, const float* theta, int64_t tstride, int Z,
                       const GateImgs& gi, char* dst) {
  const int nimg = (int)(gi.tstride / GATE_IMG_BYTES);
  const int64_t threads = (int64_t)nimg * 512;
  k_split_gate<<<dim3((unsigned)((threads + 255) / 256), Z), 256, 0, s>>>(theta, tstride, po, d.L, d.H, d.Hc, nimg,
                                                                          gi.tstride, dst);
}

// ====================================================================================
// Head + loss: pred[m, c'] = h_T[m] . Wo[c'] + bo[c'];  loss = mean (pred - y)^2 with the
// F4 pairing: pred row (n*Hf + h) of sample s is compared with target row (h'*N + n')
// of the SAME flat row index r = n*Hf + h  (h' = r / N, n' = r % N).
__global__ __launch_bounds__(NT) void k_head_loss(const float* __restrict__ hT_base, int64_t hT_zstride,
                                                  const float* __restrict__ theta, int64_t tstride, int64_t wo,
                                                  int64_t bo, const float* const* __restrict__ xtab,
                                                  float* __restrict__ pred, float* __restrict__ dpred,
                                                  float* __restrict__ lpart, int lblocks, int M, int H,
                                                  int HfC, int N, int Hf, int C, int yrow0, int yld, int B,
                                                  float dscale) {
  __shared__ float smem[CfgNT::SMEM_FLOATS];
  const int z = blockIdx.z;
  const float* th = theta + (int64_t)z * tstride;
  RowMajorKC la{hT_base + (int64_t)z * hT_zstride, M, H};
  RowMajorKC lb{th + wo, HfC, H};
  const int m0 = blockIdx.x * CfgNT::BM;
  Acc<CfgNT> acc;
  acc.zero();
  gemm_mainloop<CfgNT>(la, lb, m0, 0, 0, H, acc, smem);
  float lsum = 0.f;
#pragma unroll
  for (int i = 0; i < CfgNT::WTM; ++i)
#pragma unroll
    for (int j = 0; j < CfgNT::WTN; ++j) {
      const int cc = acc_col<CfgNT>(j);
      if (cc >= HfC) continue;
      const float bc = th[bo + cc];
      const int h = cc / C, c = cc - h * C;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + acc_row<CfgNT>(i, r);
        if (m >= M) continue;
        const float p = acc.v[i][j][r] + bc;
        const int64_t o = ((int64_t)z * M + m) * HfC + cc;
        if (pred) pred[o] = p;
        if (xtab) {
          const int s = m / N, n = m - s * N;
          const int rr = n * Hf + h;
          const int hp = rr / N, np = rr - hp * N;
          const float* xs = xtab[z * B + s];
          const float y = xs[((int64_t)(yrow0 + hp) * N + np) * yld + c];
          const float df = p - y;
          lsum = fmaf(df, df, lsum);
          if (dpred) dpred[o] = dscale * df;
        }
      }
    }
  if (lpart) {
    const float s = block_sum(lsum, smem);
    if (threadIdx.x == 0) lpart[(int64_t)z * lblocks + blockIdx.x] = s;
  }
}

// dst[z][m][j] = drop(src[z][m][j]) with the head-input mask (kind 3; hybrid_model.py:108):
// h_T -> drop(h_T), R h_T -> drop(R h_T), and in place on dh_T / R dh_T.
__global__ void k_drop_rows(const float* src, int64_t src_zstride, float* dst, int M, int H, Drop dr) {
  const int z = blockIdx.y;
  const uint32_t site = drop_site(dr.seed, 3, dr.step, 0);
  const int64_t n = (int64_t)M * H;
  const uint64_t base = (uint64_t)dr.task_id[z] * (uint64_t)n;
  const float* sz = src + (int64_t)z * src_zstride;
  float* dz = dst + (int64_t)z * n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dz[i] = drop_keep(site, base + i, dr.thr_lstm) ? sz[i] * dr.sc_lstm : 0.f;
}

void launch_drop_rows(hipStream_t s, const Work& w, int H, const float* src, int64_t src_zstride, float* dst) {
  const int64_t n = (int64_t)w.M * H;
  int nb = (int)((n + NT - 1) / NT);
  if (nb > 1024) nb = 1024;
  k_drop_rows<<<dim3(nb, w.Z), NT, 0, s>>>(src, src_zstride, dst, w.M, H, w.drop);
}

__global__ void k_dropout_inplace(float* x, int64_t n, uint32_t site, uint32_t thr, float sc) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] = drop_keep(site, (uint64_t)i, thr) ? x[i] * sc : 0.f;
}

void launch_dropout_inplace(hipStream_t s, float* x, int64_t n, float p, uint32_t seed, int layer) {
  const uint32_t thr = (uint32_t)std::min<double>(std::llround((double)p * 16777216.0), 16777216.0);
  int nb = (int)((n + NT - 1) / NT);
  if (nb > 4096) nb = 4096;
  k_dropout_inplace<<<nb, NT, 0, s>>>(x, n, drop_site(seed, 1, 0, layer), thr, 1.f / (1.f - p));
}

// The head's input rows: h_T of the top layer (z stride T*M*H), or drop(h_T) under dropout.
const float* head_input(const Dims& d, const Work& w, bool tangent, int64_t* zstride) {
  if (w.drop.lstm()) {
    *zstride = (int64_t)w.M * d.H;
    return tangent ? w.RhTd : w.hTd;
  }
  *zstride = (int64_t)d.T * w.M * d.H;
  const int64_t lsz = (int64_t)w.Z * d.T * w.M * d.H;
  return (tangent ? w.RHs : w.Hs) + (int64_t)(d.L - 1) * lsz + (int64_t)(d.T - 1) * w.M * d.H;
}

// Small-M head (batch-1 adaptation: M = 441 rows): the MFMA tile kernel above gets ceil(M/128)
// workgroups and a serial epilogue. Here one workgroup per row m (one thread per output column):
// h_T[m] is staged in LDS, each thread streams its Wo row (L2-resident) with all loads in flight.
// Loss partial per row (head_lblocks = M), summed in row order by k_loss_final.
__global__ __launch_bounds__(128) void k_head_loss_small(const float* __restrict__ hT_base, int64_t hT_zstride,
                                                         const float* __restrict__ theta, int64_t tstride, int64_t wo,
                                                         int64_t bo, const float* const* __restrict__ xtab,
                                                         float* __restrict__ pred, float* __restrict__ dpred,
                                                         float* __restrict__ lpart, int lblocks, int M, int H, int HfC,
                                                         int N, int Hf, int C, int yrow0, int yld, int B, float dscale) {
  __shared__ __attribute__((aligned(16))) float hs[SMAML_HEAD_MAX_H];  // read as float4
  __shared__ float red[2];
  const int z = blockIdx.z, m = blockIdx.x, cc = threadIdx.x;
  const float* th = theta + (int64_t)z * tstride;
  const float* h = hT_base + (int64_t)z * hT_zstride + (int64_t)m * H;
  for (int k = cc; k < H; k += blockDim.x) hs[k] = h[k];
  __syncthreads();
  float lsum = 0.f;
  if (cc < HfC) {
    const float* wr = th + wo + (int64_t)cc * H;
    float4 acc = f4zero();
#pragma unroll 8
    for (int k = 0; k < H; k += 4) {
      const float4 wv = ld4(wr + k);
      const float4 hv = *reinterpret_cast<const float4*>(hs + k);
      acc = make_float4(fmaf(wv.x, hv.x, acc.x), fmaf(wv.y, hv.y, acc.y), fmaf(wv.z, hv.z, acc.z),
                        fmaf(wv.w, hv.w, acc.w));
    }
    const float p = ((acc.x + acc.y) + (acc.z + acc.w)) + th[bo + cc];
    const int64_t o = ((int64_t)z * M + m) * HfC + cc;
    if (pred) pred[o] = p;
    if (xtab) {
      const int sm = m / N, n = m - sm * N;
      const int hh = cc / C, c = cc - hh * C;
      const int rr = n * Hf + hh;  // F4 pairing (see k_head_loss)
      const int hp = rr / N, np = rr - hp * N;
      const float df = p - xtab[z * B + sm][((int64_t)(yrow0 + hp) * N + np) * yld + c];
      lsum = df * df;
      if (dpred) dpred[o] = dscale * df;
    }
  }
  if (lpart) {
    // fixed-order block sum over the (<= 2) waves
    float v = lsum;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) lpart[(int64_t)z * lblocks + m] = blockDim.x > 64 ? red[0] + red[1] : red[0];
  }
}

bool head_small(const Dims& d, int M) {
  return M <= SMAML_HEAD_SMALL_M && d.HfC <= 128 && d.H % 4 == 0 && d.H <= SMAML_HEAD_MAX_H;
}
int head_lblocks(const Dims& d, int M) { return head_small(d, M) ? M : (M + CfgNT::BM - 1) / CfgNT::BM; }
static int head_small_threads(const Dims& d) { return d.HfC > 64 ? 128 : 64; }

// dWo[c][j] = sum_m dpred[m][c] h_T[m][j], dbo[c] = sum_m dpred[m][c] for small M: one workgroup
// per output row c, HW row groups x H units; each row group sums its contiguous share of the rows
// in order, then the groups are added in a fixed order through LDS (deterministic).
// With theta (no LSTM dropout): blocks HfC .. also form the top layer's dh_T = dpred . Wo into dH
// [Z][M][H], HWG rows per block, one thread per (row, unit) -- the head's two backward products in
// one launch instead of this kernel plus a k_gemm_nn (launch_head_dh) at batch-1 sizes.
constexpr int HWG = 8;  // row groups
__global__ __launch_bounds__(1024) void k_head_wgrad_small(const float* __restrict__ dpred, int64_t dp_zstride,
                                                         const float* __restrict__ hT, int64_t hz, int M, int H,
                                                         int HfC, float* __restrict__ grad, int64_t P, int64_t wo,
                                                         int64_t bo, const float* __restrict__ theta, int64_t tstride,
                                                         float* __restrict__ dH) {
  __shared__ float red[HWG][SMAML_HEAD_MAX_H + 1];
  const int c = blockIdx.x, z = blockIdx.y, j = threadIdx.x % H, rg = threadIdx.x / H;
  if (c >= HfC) {  // dh_T rows (uniform per block: no barrier below is skipped by part of a block)
    const int m = (c - HfC) * HWG + rg;
    if (m >= M) return;
    const float* dp = dpred + (int64_t)z * dp_zstride + (int64_t)m * HfC;
    const float* W = theta + (int64_t)z * tstride + wo + j;
    float a = 0.f;
#pragma unroll 8
    for (int k = 0; k < HfC; ++k) a = fmaf(dp[k], W[(int64_t)k * H], a);
    dH[((int64_t)z * M + m) * H + j] = a;
    return;
  }
  const float* dp = dpred + (int64_t)z * dp_zstride + c;
  const float* h = hT + (int64_t)z * hz + j;
  const int per = (M + HWG - 1) / HWG, mb = rg * per, me = min(M, mb + per);
  float a = 0.f, b = 0.f;
#pragma unroll 8
  for (int m = mb; m < me; ++m) {
    const float d0 = dp[(int64_t)m * HfC];
    a = fmaf(d0, h[(int64_t)m * H], a);
    b += d0;
  }
  red[rg][j] = a;
  if (j == 0) red[rg][H] = b;
  __syncthreads();
  if (rg == 0) {
    float s = 0.f, sb = 0.f;
#pragma unroll
    for (int g = 0; g < HWG; ++g) s += red[g][j];
    float* gz = grad + (int64_t)z * P;
    gz[wo + (int64_t)c * H + j] = s;
    if (j == 0) {
#pragma unroll
      for (int g = 0; g < HWG; ++g) sb += red[g][H];
      gz[bo + c] = sb;
    }
  }
}

void launch_head_wgrad_small(hipStream_t s, const Dims& d, const Work& w, const float* dpred, const float* hT,
                             int64_t hz, float* grad, int64_t P, int64_t wo, int64_t bo, const float* theta,
                             int64_t tstride) {
  const int dh_blocks = theta ? (w.M + HWG - 1) / HWG : 0;
  k_head_wgrad_small<<<dim3(d.HfC + dh_blocks, w.Z), HWG * d.H, 0, s>>>(
      dpred, (int64_t)w.M * d.HfC, hT, hz, w.M, d.H, d.HfC, grad, P, wo, bo, theta, tstride, w.dH);
}

void launch_head_loss(hipStream_t s, const Dims& d, const Work& w, const float* theta, int64_t tstride,
                      const ParamOff& po, const float* const* xtab, float dscale, bool want_loss) {
  const int64_t lsz = (int64_t)w.Z * d.T * w.M * d.H;
  const float* top = w.Hs + (int64_t)(d.L - 1) * lsz;
  if (w.drop.lstm()) launch_drop_rows(s, w, d.H, top + (int64_t)(d.T - 1) * w.M * d.H, (int64_t)d.T * w.M * d.H, w.hTd);
  int64_t hz = 0;
  const float* hT = head_input(d, w, false, &hz);
  if (head_small(d, w.M)) {
    k_head_loss_small<<<dim3(w.M, 1, w.Z), head_small_threads(d), 0, s>>>(
        hT, hz, theta, tstride, po.wo, po.bo, want_loss ? xtab : nullptr, w.pred, want_loss ? w.dpred : nullptr,
        want_loss ? w.lpart : nullptr, w.lblocks, w.M, d.H, d.HfC, d.N, d.Hf, d.C, d.T + 1, d.Cin0, w.B, dscale);
    return;
  }
  dim3 grid((w.M + CfgNT::BM - 1) / CfgNT::BM, 1, w.Z);
  // targets from the feature stream: rows T+1 .. T+Hf after the window start, first C channels (F5)
  k_head_loss<<<grid, NT, 0, s>>>(hT, hz, theta, tstride, po.wo, po.bo,
                                  want_loss ? xtab : nullptr, w.pred, want_loss ? w.dpred : nullptr,
                                  want_loss ? w.lpart : nullptr, w.lblocks, w.M, d.H, d.HfC, d.N, d.Hf,
                                  d.C, d.T + 1, d.Cin0, w.B, dscale);
}

void launch_head_loss_y(hipStream_t s, const Dims& d, const Work& w, const float* hT, const float* theta,
                        const ParamOff& po, const float* const* ytab, float* pred, float* dpred, float dscale) {
  // explicit targets: ytab[s] -> y [Hf*N][C] in the reference's layout (dataset.py:40-48)
  if (head_small(d, w.M)) {
    k_head_loss_small<<<dim3(w.M, 1, 1), head_small_threads(d), 0, s>>>(
        hT, 0, theta, 0, po.wo, po.bo, ytab, pred, ytab ? dpred : nullptr, ytab ? w.lpart : nullptr, w.lblocks, w.M,
        d.H, d.HfC, d.N, d.Hf, d.C, 0, d.C, w.B, dscale);
    return;
  }
  dim3 grid((w.M + CfgNT::BM - 1) / CfgNT::BM, 1, 1);
  k_head_loss<<<grid, NT, 0, s>>>(hT, 0, theta, 0, po.wo, po.bo, ytab, pred, ytab ? dpred : nullptr,
                                  ytab ? w.lpart : nullptr, w.lblocks, w.M, d.H, d.HfC, d.N, d.Hf, d.C, 0, d.C,
                                  w.B, dscale);
}

__global__ void k_loss_final(const float* __restrict__ lpart, int lblocks, float inv_count,
                             float* __restrict__ out) {
  __shared__ float red[NT / 64];
  const int z = blockIdx.x;
  float v = 0.f;
  for (int i = threadIdx.x; i < lblocks; i += NT) v += lpart[(int64_t)z * lblocks + i];
  const float s = block_sum(v, red);
  if (threadIdx.x == 0) out[z] = s * inv_count;
}

void launch_loss_final(hipStream_t s, const Work& w, float inv_count, float* out) {
  k_loss_final<<<w.Z, NT, 0, s>>>(w.lpart, w.lblocks, inv_count, out);
}

// ====================================================================================
// Generic C = A . B (A k-contiguous, B n-contiguous) with plain store; used for
//   dh_T = dpred . Wo      (head backward into the top layer's dH at t = T-1)
//   dX_l = dG_l . W_ih_l   (input grads of LSTM layer l > 0 over all T*M rows)
__global__ __launch_bounds__(NT) void k_gemm_nn(const float* __restrict__ A, int64_t a_zstride, int rows,
                                                int K, const float* __restrict__ theta, int64_t tstride,
                                                int64_t woff, int ncols, float* __restrict__ out,
                                                int64_t o_zstride) {
  __shared__ float smem[CfgNN::SMEM_FLOATS];
  const int z = blockIdx.z;
  RowMajorKC la{A + (int64_t)z * a_zstride, rows, K};
  RowMajorMC lb{theta + (int64_t)z * tstride + woff, K, ncols};
  const int m0 = blockIdx.x * CfgNN::BM, n0 = blockIdx.y * CfgNN::BN;
  Acc<CfgNN> acc;
  acc.zero();
  gemm_mainloop<CfgNN>(la, lb, m0, n0, 0, K, acc, smem);
  float* o = out + (int64_t)z * o_zstride;
#pragma unroll
  for (int j = 0; j < CfgNN::WTN; ++j) {
    const int c = n0 + acc_col<CfgNN>(j);
    if (c >= ncols) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + acc_row<CfgNN>(0, r);
      if (m < rows) o[(int64_t)m * ncols + c] = acc.v[0][j][r];
    }
  }
}

void launch_head_dh(hipStream_t s, const Dims& d, const Work& w, const float* theta, int64_t tstride,
                    const ParamOff& po) {
  // dh_T of the top layer: [Z][M][H], added by the BPTT step (L-1, T-1)
  dim3 grid((w.M + CfgNN::BM - 1) / CfgNN::BM, (d.H + CfgNN::BN - 1) / CfgNN::BN, w.Z);
  k_gemm_nn<<<grid, CfgNN::NTH, 0, s>>>(w.dpred, (int64_t)w.M * d.HfC, w.M, d.HfC, theta, tstride, po.wo, d.H,
                                w.dH, (int64_t)w.M * d.H);
  if (w.drop.lstm()) launch_drop_rows(s, w, d.H, w.dH, (int64_t)w.M * d.H, w.dH);  // d drop(h_T) -> d h_T
}

// ====================================================================================
// LSTM backward step (layer l, time t), one anti-diagonal of (l, t) per launch (BwdWave):
//   dh = [dG(l+1,t) | dG(l,t+1)] . [W_ih(l+1) ; W_hh(l)]  (+ head dh_T at l = L-1, t = T-1)
//                                   [f32-accurate bf16x6 products, K = 8H, 4H at the borders]
//   dc = dc_carry + dh * o * (1 - tanh(c_t)^2)
//   dG_t = [dc*g*i(1-i), dc*c_{t-1}*f(1-f), dc*i*(1-g^2), dh*tanh(c_t)*o(1-o)]  (in place over G_t)
//   dc_carry = dc * f
// In place is safe: a workgroup reads G_t only for its own rows and units before writing them,
// and its GEMM reads other (l, t) slabs finished on the previous diagonal.
// 64x64 tiles for small grids (few tasks per rank) so the launch fills the chip.
using CfgNNs = GemmCfg<64, 64, 2, 2, true, false, SMAML_NN_BK, SMAML_X6_BWD>;
// BPTT step tile (A/B-able at build time): rows x 128 units, waves WM x WN
using CfgBwd = GemmCfg<SMAML_BWD_BM, 128, SMAML_BWD_WM, SMAML_BWD_WN, true, false, SMAML_NN_BK, SMAML_X6_BWD,
                       SMAML_BWD_NST>;

double bwd_wave(const Dims& d, const Work& w, const ParamOff& po, int e, int blocks_per_problem, bool dual,
                BwdWave& wv) {
  double fl = 0.0;
  int n = 0, off = 0;
  for (int l = d.L - 1; l >= 0; --l) {
    const int t = d.T - 1 - (e - (d.L - 1 - l));
    if (t < 0 || t >= d.T) continue;
    wv.l[n] = l;
    wv.t[n] = t;
    wv.lo[n] = po.lay[l];
    wv.wih_up[n] = l + 1 < d.L ? po.lay[l + 1].wih : 0;
    wv.off[n] = off;
    off += blocks_per_problem;
    ++n;
    const int segs = (l + 1 < d.L ? 1 : 0) + (t + 1 < d.T ? 1 : 0);
    fl += (dual ? 3.0 : 1.0) * 2.0 * w.Z * w.M * 4 * d.H * d.H * segs;
  }
  wv.n = n;
  for (int q = n; q <= MAX_LAYERS; ++q) wv.off[q] = off;
  return fl;
}

// Cell backward of one BPTT tile (acc = dh from the fused K = 8H GEMM, head dh_T not yet added):
// dc, dG (in place over G_t, or into a separate slab), the cell-state carry and (optionally) the
// kept dh.
//
// The accumulators are first transposed through LDS (the mainloop's staging buffers, idle by
// then) so that every lane then works on float4 groups of 4 consecutive hidden units of one row:
// all epilogue memory traffic becomes 16-B loads / stores (4x fewer instructions than the
// accumulator's column-per-lane layout, whole 128-B lines per 8 lanes) and one address serves 4
// elements. Each item's 7 loads (gates, c_t, c_{t-1}, the dc carry, dh_T) are in flight together;
// SMAML_EPI_DEPTH 2 also loads item k+1 before item k is computed (more registers: slower as
// measured). Program order keeps the in-place dG over G safe: an item's elements are
// read before they are written and items never share elements. Uniform conditions (t = 0, the
// first step) are selects on loads from valid addresses, so no branch splits the loads.
#ifndef SMAML_DIAG_BWD
#define SMAML_DIAG_BWD 0  // timing diagnostics only (wrong results): 1 = BPTT step without its epilogue,
#endif                    // 2 = without its GEMM
#ifndef SMAML_EPI_DEPTH
#define SMAML_EPI_DEPTH 1  // epilogue items in flight per thread (1 or 2; A/B-able at build time)
#endif
template <class C>
constexpr int epi_smem_floats() {
  constexpr int E = SMAML_BWD_HALFEPI ? C::BM * C::BN / 2 : C::BM * C::BN;
  return C::SMEM_FLOATS > E ? C::SMEM_FLOATS : E;
}


template <int H, class CfgNN, bool HEAD, bool CHECK>
__device__ __forceinline__ void bwd_cell_(const float* smem, const float* Gz, float* dGz, float* __restrict__ dhz,
                                          const float* __restrict__ Cz, const float* __restrict__ dHz,
                                          float* __restrict__ dcz, int m0, int n0, int t, int T, int M) {
  constexpr int G4 = 4 * H;
  constexpr int GPR = CfgNN::BN / 4;                          // float4 groups per tile row
  constexpr int NIT = CfgNN::BM * GPR / CfgNN::NTH;           // items per thread
  static_assert(NIT * CfgNN::NTH == CfgNN::BM * GPR && NIT % 2 == 0, "epilogue items");
  const bool first = (t == T - 1), past = t > 0;
  const int64_t pM = past ? (int64_t)M * H : 0;  // c_{t-1} offset (t = 0: masked)
  const int64_t tM = (int64_t)t * M;
  struct V {  // c_t is re-derived from the gates and c_{t-1} (lstm_cell_c), not loaded
    float4 g[4], cp, dc, hd;
  };
  auto coords = [&](int k, int& r, int& m, int& j) {
    const int item = (int)threadIdx.x + CfgNN::NTH * k;
    r = item / GPR;
    m = m0 + r;
    j = n0 + 4 * (item % GPR);
  };
  auto load = [&](int k, V& v) {
    int r, m, j;
    coords(k, r, m, j);
    if (CHECK) {  // out-of-range items read a valid element (their results are not stored)
      m = min(m, M - 1);
      j = min(j, H - 4);
    }
    const int64_t row = tM + m;
    const float* gp = Gz + row * G4 + j;
#pragma unroll
    for (int g = 0; g < 4; ++g) v.g[g] = ld4(gp + g * H);
    v.cp = ld4(Cz + row * H - pM + j);
    v.dc = ld4(dcz + (int64_t)m * H + j);
    if (HEAD) v.hd = ld4(dHz + (int64_t)m * H + j);
  };
  auto step = [&](int k, const V& v) {
    int r, m, j;
    coords(k, r, m, j);
    if (CHECK && (m >= M || j >= H)) return;
    float4 dh = *reinterpret_cast<const float4*>(smem + r * CfgNN::BN + (j - n0));
    if (HEAD) dh = make_float4(dh.x + v.hd.x, dh.y + v.hd.y, dh.z + v.hd.z, dh.w + v.hd.w);
    const float4 cp = sel4(past, v.cp), dc = sel4(!first, v.dc);
    float4 o[4], odc;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float gi = f4get(v.g[0], e), gf = f4get(v.g[1], e), gg = f4get(v.g[2], e), go = f4get(v.g[3], e);
      const float d = f4get(dh, e);
      const float tc = tanhf_(lstm_cell_c(gi, gf, gg, f4get(cp, e)));
      const float dct = f4get(dc, e) + d * go * (1.f - tc * tc);
      const float r0 = dct * gg * gi * (1.f - gi), r1 = dct * f4get(cp, e) * gf * (1.f - gf);
      const float r2 = dct * gi * (1.f - gg * gg), r3 = d * tc * go * (1.f - go);
      const float rc = dct * gf;
      if (e == 0) { o[0].x = r0; o[1].x = r1; o[2].x = r2; o[3].x = r3; odc.x = rc; }
      if (e == 1) { o[0].y = r0; o[1].y = r1; o[2].y = r2; o[3].y = r3; odc.y = rc; }
      if (e == 2) { o[0].z = r0; o[1].z = r1; o[2].z = r2; o[3].z = r3; odc.z = rc; }
      if (e == 3) { o[0].w = r0; o[1].w = r1; o[2].w = r2; o[3].w = r3; odc.w = rc; }
    }
    const int64_t row = tM + m;
    float* gp = dGz + row * G4 + j;
#pragma unroll
    for (int g = 0; g < 4; ++g) st4(gp + g * H, o[g]);
    st4(dcz + (int64_t)m * H + j, odc);
    if (dhz) st4(dhz + row * H + j, dh);
  };
  if constexpr (SMAML_EPI_DEPTH >= 2) {  // two items in flight (more registers)
    V va, vb;
    load(0, va);
#pragma unroll 1
    for (int k = 0; k < NIT; k += 2) {
      load(k + 1, vb);
      step(k, va);
      if (k + 2 < NIT) load(k + 2, va);
      step(k + 1, vb);
    }
  } else {  // one item's 7 x 16-B loads in flight; its stores drain under the next item's loads
    V v;
#pragma unroll 1
    for (int k = 0; k < NIT; ++k) {
      load(k, v);
      step(k, v);
    }
  }
}

template <int H, class CfgNN, bool HEAD>
__device__ __forceinline__ void bwd_cell(const Acc<CfgNN>& acc, float* smem, const float* Gz, float* dGz,
                                         float* __restrict__ dhz, const float* __restrict__ Cz,
                                         const float* __restrict__ dHz, float* __restrict__ dcz, int m0, int n0,
                                         int t, int T, int M) {
  if constexpr (SMAML_BWD_HALFEPI) {
    using HC = HalfRows<CfgNN>;
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
      if (h) __syncthreads();  // the first half's readers are done with the LDS
      acc_to_lds_half<CfgNN>(acc, smem, h);
      const int mh = m0 + h * HC::BM;
      if (mh + HC::BM <= M && n0 + HC::BN <= H)
        bwd_cell_<H, HC, HEAD, false>(smem, Gz, dGz, dhz, Cz, dHz, dcz, mh, n0, t, T, M);
      else
        bwd_cell_<H, HC, HEAD, true>(smem, Gz, dGz, dhz, Cz, dHz, dcz, mh, n0, t, T, M);
    }
  } else {
    acc_to_lds<CfgNN>(acc, smem);
    if (m0 + CfgNN::BM <= M && n0 + CfgNN::BN <= H)  // all but the last row tile: no bounds checks
      bwd_cell_<H, CfgNN, HEAD, false>(smem, Gz, dGz, dhz, Cz, dHz, dcz, m0, n0, t, T, M);
    else
      bwd_cell_<H, CfgNN, HEAD, true>(smem, Gz, dGz, dhz, Cz, dHz, dcz, m0, n0, t, T, M);
  }
}

// GsAll: gates in; dGAll: dG out (== GsAll: in place) and the neighbours' dG read by the GEMM;
// dhAll (optional): the step's dh kept for the second-order sweep ([L][Z][T][M][H]).
// DROP: the layer-above segment carries dX of layer l+1's input drop(h_l): its contribution
// is masked before the recurrent segment accumulates (two mainloops instead of one).
template <int H, class CfgNN, bool DROP>
__global__ SMAML_BWD_ATTR __launch_bounds__(CfgNN::NTH) void k_lstm_bwd_step(const float* GsAll, float* dGAll,
                                                      float* __restrict__ dhAll, const float* __restrict__ CsAll,
                                                      const float* __restrict__ dHhead, float* __restrict__ dcAll,
                                                      int64_t lsz, const float* __restrict__ theta, int64_t tstride,
                                                      BwdWave wv, int L, int T, int M, Drop dr) {
  __shared__ float smem[epi_smem_floats<CfgNN>()];
  constexpr int G4 = 4 * H;
  const Blk bk = xcd_block();
  int mb;
  const int p = bwd_block(wv, bk.x, mb);
  mb += wv.tm0;
  const int l = wave_sel(wv.l, p), t = wave_sel(wv.t, p);
  const LayerOff lo = wave_sel(wv.lo, p);
  const int64_t wih_up = wave_sel(wv.wih_up, p);
  const int z = bk.z;
  const int m0 = mb * CfgNN::BM, n0 = bk.y * CfgNN::BN;
  const int64_t slab = (int64_t)z * T * M;
  const float* th = theta + (int64_t)z * tstride;
  const float* Gz = GsAll + (int64_t)l * lsz * 4 + slab * G4;  // gates in
  float* dGz = dGAll + (int64_t)l * lsz * 4 + slab * G4;        // dG out
  float* dhz = dhAll ? dhAll + (int64_t)l * lsz + slab * H : nullptr;
  const float* Cz = CsAll + (int64_t)l * lsz + slab * H;
  float* dcz = dcAll + ((int64_t)l * gridDim.z + z) * M * H;
  Acc<CfgNN> acc;
  acc.zero();
  {
    // segments [above | next], compacted with selects (static indices keep the loaders in registers)
    const bool up = l + 1 < L, nx = t + 1 < T;
    const float* pa = dGAll + (int64_t)(l + 1) * lsz * 4 + (slab + (int64_t)t * M) * G4;
    const float* pn = dGz + (int64_t)(t + 1) * M * G4;
    const int ns = (up ? 1 : 0) + (nx ? 1 : 0);
    if (DROP && up) {
      const XDrop xd{drop_site(dr.seed, 2, dr.step, l), dr.thr_lstm, dr.sc_lstm,
                     ((uint64_t)dr.task_id[z] * T + t) * M * H, H};
      gemm_mainloop<CfgNN>(SegKC{{pa, nullptr, nullptr, nullptr}, {G4, 0, 0, 0}, M},
                           SegMC{{th + wih_up, nullptr}, {G4, 0}, H}, m0, n0, 0, G4, acc, smem);
      drop_acc<CfgNN>(acc, xd, m0, n0);
      if (nx)
        gemm_mainloop<CfgNN>(SegKC{{pn, nullptr, nullptr, nullptr}, {G4, 0, 0, 0}, M},
                             SegMC{{th + lo.whh, nullptr}, {G4, 0}, H}, m0, n0, 0, G4, acc, smem);
    } else {
      const SegKCt<2> la{{up ? pa : pn, pn}, {G4, G4}, M};
      const SegMCt<2> lb{{up ? th + wih_up : th + lo.whh, th + lo.whh}, {G4, G4}, H};
      if (ns && SMAML_DIAG_BWD != 2) gemm_mainloop<CfgNN>(la, lb, m0, n0, 0, ns * G4, acc, smem);
    }
  }
  if (SMAML_DIAG_BWD == 1) {  // timing diagnostic: GEMM phase only (keep the result live)
    acc_to_lds<CfgNN>(acc, smem);
    if (t < 0) dGz[threadIdx.x] = smem[threadIdx.x];
    return;
  }
  if (l == L - 1 && t == T - 1)  // the head's dh_T enters at the top layer's last step only
    bwd_cell<H, CfgNN, true>(acc, smem, Gz, dGz, dhz, Cz, dHhead + (int64_t)z * M * H, dcz, m0, n0, t, T, M);
  else
    bwd_cell<H, CfgNN, false>(acc, smem, Gz, dGz, dhz, Cz, dHhead + (int64_t)z * M * H, dcz, m0, n0, t, T, M);
}

// Split-K BPTT step for small grids (see k_lstm_fwd_part): partial dh over a K-tile range of the
// fused [above | next] GEMM, then k_lstm_bwd_cell sums the partials in order and runs bwd_cell.
template <int H, class CfgNN>
__global__ __launch_bounds__(CfgNN::NTH) void k_lstm_bwd_part(const float* dGAll, int64_t lsz,
                                                                            const float* __restrict__ theta,
                                                                            int64_t tstride, BwdWave wv, int L, int T,
                                                                            int M, int S, float* __restrict__ part) {
  __shared__ float smem[part_smem_floats<CfgNN, SMAML_BWD_PART_NCH>()];
  constexpr int G4 = 4 * H;
  const int p = wave_index(wv, (int)blockIdx.x);
  const int l = wave_sel(wv.l, p), t = wave_sel(wv.t, p), b0 = wave_sel(wv.off, p);
  const LayerOff lo = wave_sel(wv.lo, p);
  const int64_t wih_up = wave_sel(wv.wih_up, p);
  const int z = blockIdx.z;
  const int m0 = ((int)blockIdx.x - b0) * CfgNN::BM, n0 = blockIdx.y % ((H + CfgNN::BN - 1) / CfgNN::BN) * CfgNN::BN;
  const int split = blockIdx.y / ((H + CfgNN::BN - 1) / CfgNN::BN);
  const int64_t slab = (int64_t)z * T * M;
  const float* th = theta + (int64_t)z * tstride;
  const bool up = l + 1 < L, nx = t + 1 < T;
  const float* pa = dGAll + (int64_t)(l + 1) * lsz * 4 + (slab + (int64_t)t * M) * G4;
  const float* pn = dGAll + (int64_t)l * lsz * 4 + (slab + (int64_t)(t + 1) * M) * G4;
  const int ns = (up ? 1 : 0) + (nx ? 1 : 0);
  int kbeg, kend;
  split_range(ns * G4, S, split, CfgNN::BK, kbeg, kend);
  Acc<CfgNN> acc;
  acc.zero();
  if (kbeg < kend) {
    const SegKCt<2> la{{up ? pa : pn, pn}, {G4, G4}, M};
    const SegMCt<2> lb{{up ? th + wih_up : th + lo.whh, th + lo.whh}, {G4, G4}, H};
    part_mainloop<CfgNN, SMAML_BWD_PART_NCH>(la, lb, m0, n0, kbeg, kend, acc, smem);
  }
  // slab of (z, y = split * ntn + tn, x)
  constexpr int PER = CfgNN::WTM * CfgNN::WTN * 16 * CfgNN::NTH;
  store_part<CfgNN>(acc, part + (((int64_t)z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * PER);
}

template <int H, class CfgNN>
__global__ __launch_bounds__(CfgNN::NTH) void k_lstm_bwd_cell(const float* GsAll, float* dGAll,
                                                             float* __restrict__ dhAll, const float* __restrict__ CsAll,
                                                             const float* __restrict__ dHhead,
                                                             float* __restrict__ dcAll, int64_t lsz, BwdWave wv, int L,
                                                             int T, int M, int S, const float* __restrict__ part) {
  __shared__ float smem[CfgNN::BM * CfgNN::BN];
  constexpr int G4 = 4 * H;
  const int p = wave_index(wv, (int)blockIdx.x);
  const int l = wave_sel(wv.l, p), t = wave_sel(wv.t, p), b0 = wave_sel(wv.off, p);
  const int z = blockIdx.z;
  const int ntn = gridDim.y;
  const int m0 = ((int)blockIdx.x - b0) * CfgNN::BM, n0 = blockIdx.y * CfgNN::BN;
  Acc<CfgNN> acc;
  acc.zero();
  // the part kernel's grid is (x, S * ntn, z): its slab of (x, split * ntn + tn, z)
  constexpr int PER = CfgNN::WTM * CfgNN::WTN * 16 * CfgNN::NTH;
  for (int q = 0; q < S; ++q)
    add_part<CfgNN>(acc, part + (((int64_t)z * (S * ntn) + q * ntn + blockIdx.y) * gridDim.x + blockIdx.x) * PER);
  const int64_t slab = (int64_t)z * T * M;
  const float* Gz = GsAll + (int64_t)l * lsz * 4 + slab * G4;
  float* dGz = dGAll + (int64_t)l * lsz * 4 + slab * G4;
  float* dhz = dhAll ? dhAll + (int64_t)l * lsz + slab * H : nullptr;
  const float* Cz = CsAll + (int64_t)l * lsz + slab * H;
  float* dcz = dcAll + ((int64_t)l * gridDim.z + z) * M * H;
  if (l == L - 1 && t == T - 1)
    bwd_cell<H, CfgNN, true>(acc, smem, Gz, dGz, dhz, Cz, dHhead + (int64_t)z * M * H, dcz, m0, n0, t, T, M);
  else
    bwd_cell<H, CfgNN, false>(acc, smem, Gz, dGz, dhz, Cz, dHhead + (int64_t)z * M * H, dcz, m0, n0, t, T, M);
}

// The split-K BPTT step's cell kernel over 4x the threads (cf. k_lstm_fwd_cell_q): blockIdx.y =
// tn * 4 + q, each thread sums its accumulator registers 4q..4q+3 over the S partials (same order
// as k_lstm_bwd_cell) and runs the cell backward on those 4 rows of its column directly (no LDS
// transpose): all loads of a thread in flight together. Same expressions as bwd_cell_.
template <int H, class CfgNN>
__global__ __launch_bounds__(CfgNN::NTH) void k_lstm_bwd_cell_q(const float* GsAll, float* dGAll,
                                                               float* __restrict__ dhAll, const float* __restrict__ CsAll,
                                                               const float* __restrict__ dHhead,
                                                               float* __restrict__ dcAll, int64_t lsz, BwdWave wv, int L,
                                                               int T, int M, int S, const float* __restrict__ part) {
  static_assert(CfgNN::WTM == 1 && CfgNN::WTN == 1, "one 32 x 32 accumulator tile per wave");
  constexpr int G4 = 4 * H;
  constexpr int PER = 16 * CfgNN::NTH;
  const int p = wave_index(wv, (int)blockIdx.x);
  const int l = wave_sel(wv.l, p), t = wave_sel(wv.t, p), b0 = wave_sel(wv.off, p);
  const int z = blockIdx.z, tn = blockIdx.y >> 2, q = blockIdx.y & 3;
  const int ntn = gridDim.y >> 2;
  const int m0 = ((int)blockIdx.x - b0) * CfgNN::BM, n0 = tn * CfgNN::BN;
  const int tid = threadIdx.x;
  float4 a = f4zero();
  for (int sp = 0; sp < S; ++sp) {
    const float4 v =
        ld4(part + (((int64_t)z * (S * ntn) + sp * ntn + tn) * gridDim.x + blockIdx.x) * PER + 4 * (q * CfgNN::NTH + tid));
    a = make_float4(a.x + v.x, a.y + v.y, a.z + v.z, a.w + v.w);
  }
  const int64_t slab = (int64_t)z * T * M;
  const float* Gz = GsAll + (int64_t)l * lsz * 4 + slab * G4;
  float* dGz = dGAll + (int64_t)l * lsz * 4 + slab * G4;
  float* dhz = dhAll ? dhAll + (int64_t)l * lsz + slab * H : nullptr;
  const float* Cz = CsAll + (int64_t)l * lsz + slab * H;
  float* dcz = dcAll + ((int64_t)l * gridDim.z + z) * M * H;
  const float* dHz = dHhead + (int64_t)z * M * H;
  const bool first = (t == T - 1), past = t > 0, head = first && l == L - 1;
  const int j = n0 + acc_col<CfgNN>(0);
  const int rb = m0 + acc_row<CfgNN>(0, 0) + 8 * q;  // row of register 4q
  const int jc = min(j, H - 1);
  float g[4][4], cp[4], dc[4], hd[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {  // all loads first (clamped rows: valid addresses)
    const int m = min(rb + e, M - 1);
    const int64_t row = (int64_t)t * M + m;
#pragma unroll
    for (int k = 0; k < 4; ++k) g[e][k] = Gz[row * G4 + k * H + jc];
    cp[e] = past ? Cz[row * H - (int64_t)M * H + jc] : 0.f;
    dc[e] = first ? 0.f : dcz[(int64_t)m * H + jc];
    hd[e] = head ? dHz[(int64_t)m * H + jc] : 0.f;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int m = rb + e;
    if (m >= M || j >= H) continue;
    const float d = f4get(a, e) + hd[e];
    const float gi = g[e][0], gf = g[e][1], gg = g[e][2], go = g[e][3];
    const float tc = tanhf_(lstm_cell_c(gi, gf, gg, cp[e]));
    const float dct = dc[e] + d * go * (1.f - tc * tc);
    const int64_t row = (int64_t)t * M + m;
    float* gp = dGz + row * G4 + j;
    gp[0] = dct * gg * gi * (1.f - gi);
    gp[H] = dct * cp[e] * gf * (1.f - gf);
    gp[2 * H] = dct * gi * (1.f - gg * gg);
    gp[3 * H] = d * tc * go * (1.f - go);
    dcz[(int64_t)m * H + j] = dct * gf;
    if (dhz) dhz[row * H + j] = d;
  }
}
#ifndef SMAML_BWD_CELL_Q
#define SMAML_BWD_CELL_Q 1  // split-K BPTT step's cell kernel over 4x the threads (0: k_lstm_bwd_cell)
#endif

bool bwd_wave_big(const Dims& d, const Work& w, const ParamOff& po, int e) {
  BwdWave wv{};
  const int ntm = (w.M + CfgBwd::BM - 1) / CfgBwd::BM, ntn = (d.H + CfgBwd::BN - 1) / CfgBwd::BN;
  bwd_wave(d, w, po, e, ntm, false, wv);
  return (int64_t)wv.n * ntm * ntn * w.Z * (CfgBwd::BM / 64) >= w.kn.bwd_big_min;
}

void launch_lstm_bwd_wave(hipStream_t s, const Dims& d, const Work& w, int e, const float* theta, int64_t tstride,
                          const ParamOff& po, int chunk, int nch) {
  const int64_t lsz = (int64_t)w.Z * d.T * w.M * d.H;
  BwdWave wv{};
  const int ntm = (w.M + CfgBwd::BM - 1) / CfgBwd::BM, ntn = (d.H + CfgBwd::BN - 1) / CfgBwd::BN;
  bwd_wave(d, w, po, e, ntm, false, wv);
  if (wv.n == 0) return;
#define SMAML_BWD_STEP(CFG, D_)                                                                               \
  SMAML_DISPATCH_H(d.H, k_lstm_bwd_step<HT, CFG, D_><<<grid, CFG::NTH, 0, s>>>(                                  \
                            w.Gs, w.dG, w.dh, w.Cs, w.dH, w.dc, lsz, theta, tstride, wv, d.L, d.T, w.M, w.drop))
  if (nch > 1) {
    // A row chunk launches ONLY its own row tiles, always on the big tiles, whatever the diagonal's size:
    // a whole-row launch here would race the other chunks' streams (round 5's config-5 corner diagonals).
    // No other branch of this function is reachable for a chunk.
    const int lo = (int)((int64_t)ntm * chunk / nch), hi = (int)((int64_t)ntm * (chunk + 1) / nch);
    if (hi <= lo) return;
    bwd_wave(d, w, po, e, hi - lo, false, wv);
    wv.tm0 = lo;
    count_variant(w, V_BWD_BIG);
    dim3 grid(wv.off[wv.n], ntn, w.Z);
    if (w.drop.lstm()) {
      SMAML_BWD_STEP(CfgBwd, true);
    } else {
      SMAML_BWD_STEP(CfgBwd, false);
    }
    return;
  }
  // threshold in 64-row tile units (the knob predates the 128-row tile)
  const bool big = (int64_t)wv.n * ntm * ntn * w.Z * (CfgBwd::BM / 64) >= w.kn.bwd_big_min;
  if (big) {
    count_variant(w, V_BWD_BIG);
    dim3 grid(wv.off[wv.n], ntn, w.Z);
    if (w.drop.lstm()) {
      SMAML_BWD_STEP(CfgBwd, true);
    } else {
      SMAML_BWD_STEP(CfgBwd, false);
    }
  } else {
    const int ntms = (w.M + CfgNNs::BM - 1) / CfgNNs::BM, ntns = (d.H + CfgNNs::BN - 1) / CfgNNs::BN;
    bwd_wave(d, w, po, e, ntms, false, wv);
    dim3 grid(wv.off[wv.n], ntns, w.Z);
    if (!w.drop.lstm()) {
      constexpr int64_t PER = CfgNNs::WTM * CfgNNs::WTN * 16 * CfgNNs::NTH;
      const int S = small_grid_splits((int64_t)grid.x * ntns * w.Z, 8 * d.H, CfgNNs::BK,
                                      (int64_t)grid.x * ntns * w.Z * PER, w.wpart_floats, w.kn.split_max);
      if (S > 1 && small_kw_ok(d, w)) {
        launch_lstm_bwd_kw(s, d, w, e, theta, tstride, po);
        return;
      }
      if (S > 1) {
        count_variant(w, V_BWD_SPLIT);
        dim3 gp(grid.x, S * ntns, w.Z);
        SMAML_DISPATCH_H(d.H, (k_lstm_bwd_part<HT, CfgNNs><<<gp, CfgNNs::NTH, 0, s>>>(w.dG, lsz, theta, tstride, wv,
                                                                                       d.L, d.T, w.M, S, w.wpart)));
        if (SMAML_BWD_CELL_Q) {
          dim3 gq(grid.x, 4 * ntns, w.Z);
          SMAML_DISPATCH_H(d.H, (k_lstm_bwd_cell_q<HT, CfgNNs><<<gq, CfgNNs::NTH, 0, s>>>(
                                    w.Gs, w.dG, w.dh, w.Cs, w.dH, w.dc, lsz, wv, d.L, d.T, w.M, S, w.wpart)));
        } else {
          SMAML_DISPATCH_H(d.H, (k_lstm_bwd_cell<HT, CfgNNs><<<grid, CfgNNs::NTH, 0, s>>>(
                                    w.Gs, w.dG, w.dh, w.Cs, w.dH, w.dc, lsz, wv, d.L, d.T, w.M, S, w.wpart)));
        }
        return;
      }
    }
    count_variant(w, V_BWD_SMALL);
    if (w.drop.lstm()) {
      SMAML_BWD_STEP(CfgNNs, true);
    } else {
      SMAML_BWD_STEP(CfgNNs, false);
    }
  }
#undef SMAML_BWD_STEP
}

// ====================================================================================
// Weight gradients, split-K:  part[z][split][i][j] = sum_k A[k][i] * Bcat[k][j]
//   Bcat[k] = [ B1[k][0..c1) | (k >= Mshift ? B2[k - Mshift][0..c2) : 0) | 1 ]
// (the trailing column of ones is produced as column sums of A in tile column 0:
//  the bias gradient). For LSTM layer l: A = dG [T*M][4H], B1 = x_l [T*M][cin],
//  B2 = h_l (shifted one time block: h_{t-1}); for the head: A = dpred, B1 = h_T.
#ifndef SMAML_COLSUM_LDS
// Column sums of A (= the bias gradient) from the A fragments the MFMAs already hold in
// registers: lane (row r = arow + 32 i, k-half h) sums its k-values; the halves are combined
// with one cross-lane add after the mainloop (colsum_rows). No extra LDS traffic.
template <class C>
struct ColSumHook {
  float s[C::WTM];
  __device__ __forceinline__ ColSumHook() {
#pragma unroll
    for (int i = 0; i < C::WTM; ++i) s[i] = 0.f;
  }
  __device__ __forceinline__ void operator()(const float*, int) const {}
  __device__ __forceinline__ void afrag(int i, const float4& a) { s[i] += (a.x + a.y) + (a.z + a.w); }
  // staged split (C::X6S): the A float4s a thread stages always cover the same 4 gate rows
  // 4q .. 4q+3 (q = tid mod BM/4); their sums are kept here and reduced over the NTH/(BM/4) threads
  // sharing q in store().
  static constexpr int kQ = C::BM / 4, kQT = C::NTH / kQ;
  static_assert(!C::X6S || (C::NTH % kQ == 0 && !C::A_KC), "staged column sums: thread -> rows fixed");
  float4 cs = f4zero();
  template <int F4>
  __device__ __forceinline__ void stage_a(const float4 (&r)[F4]) {
#pragma unroll
    for (int i = 0; i < F4; ++i) {
      cs.x += r[i].x;
      cs.y += r[i].y;
      cs.z += r[i].z;
      cs.w += r[i].w;
    }
  }
  // lanes 0..31 own rows wm*(WTM*32) + 32 i + lane of the tile
  __device__ __forceinline__ void store(float* P, int m0, int Mrows, int ldp, int ncols, bool with_bias, float* smem) {
    if constexpr (C::X6S) {
      // the mainloop ended with a barrier: its LDS is free
      st4(smem + 4 * threadIdx.x, cs);
      __syncthreads();
      if ((int)threadIdx.x < kQ) {
        float4 v = ld4(smem + 4 * threadIdx.x);
#pragma unroll
        for (int t = 1; t < kQT; ++t) {
          const float4 u = ld4(smem + 4 * (threadIdx.x + kQ * t));
          v.x += u.x;
          v.y += u.y;
          v.z += u.z;
          v.w += u.w;
        }
        const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int row = m0 + 4 * (int)threadIdx.x + c;
          if (row < Mrows) P[(int64_t)row * ldp + ncols] = with_bias ? e[c] : 0.f;
        }
      }
      return;
    }
    const int lane = threadIdx.x & 63, wm = (threadIdx.x >> 6) / C::WAVES_N;
#pragma unroll
    for (int i = 0; i < C::WTM; ++i) {
      const float v = s[i] + __shfl_xor(s[i], 32);
      const int row = m0 + wm * (C::WTM * 32) + 32 * i + lane;
      if (lane < 32 && (threadIdx.x >> 6) % C::WAVES_N == 0 && row < Mrows)
        P[(int64_t)row * ldp + ncols] = with_bias ? v : 0.f;
    }
  }
};
#else
// A/B baseline: column sums re-read from the staged A tile in LDS once per K-tile.
template <class C>
struct ColSumHook {
  float bsum = 0.f;
  __device__ __forceinline__ void operator()(const float* as, int) {
    if (threadIdx.x < C::BM) {
      float s = bsum;
#pragma unroll 8
      for (int kk = 0; kk < C::BK; ++kk) s += as[kk * C::LDA + threadIdx.x];
      bsum = s;
    }
  }
  __device__ __forceinline__ void afrag(int, const float4&) {}
  __device__ __forceinline__ void store(float* P, int m0, int Mrows, int ldp, int ncols, bool with_bias, float*) {
    const int row = m0 + threadIdx.x;
    if (threadIdx.x < C::BM && row < Mrows) P[(int64_t)row * ldp + ncols] = with_bias ? bsum : 0.f;
  }
};
#endif

// B1 = drop(h_{l-1}) for the input weights of LSTM layer l >= 1 under dropout: row k of the
// task's [T*M][H] slab is element (task * T*M + k) * H + unit of kind 2, layer l-1.
struct WgBDrop {
  WgB b;
  XDrop d;
  __device__ __forceinline__ float4 operator()(int64_t k, int j) const {
    if (k >= b.K) return f4zero();
    if (j < b.c1) return b.B1 ? d.apply(ld4(b.B1 + k * b.c1 + j), (int)k, j) : f4zero();
    return b(k, j);
  }
};

// ---- weight-gradient mainloop with direct-to-LDS loads -----------------------------------
// k_wgrad runs ONE 8-wave workgroup per CU (207 VGPRs, 512 x 128 tile), where register staging
// leaves the MFMA pipe waiting on each K-tile's loads. Here every operand tile goes global -> LDS
// with global_load_lds_dwordx4 (no staging VGPRs, no ds_write), into a 3-stage ring, and the wait
// before each raw barrier is counted (vmcnt(5): the next tile's 5 loads per wave stay in flight
// across it). Operands outside the matrix (rows >= K, the shifted h_{t-1} rows before Mshift)
// load from a zero line. A glds wave-instruction writes 1 KB contiguously in lane order: A rows
// (512 floats = 2 KB) keep their padded LDS stride (two instructions per row), B rows (128
// floats) are unpadded (one instruction = 2 rows). Same products in the same order as the
// register-staged loop: bitwise-identical partial sums (tools/wgrad_glds_micro.hip).
#ifndef SMAML_WGRAD_GLDS
#define SMAML_WGRAD_GLDS 1
#endif
// iglp_opt strategy for the weight-gradient mainloop (staged split: none, A/B 493 -> 483 ms)
constexpr int kWgradIG = CfgTN::X6S ? -1 : SMAML_IGLP;
#ifndef SMAML_WGRAD_GLDS_IGLP
#define SMAML_WGRAD_GLDS_IGLP -1
#endif
__device__ float g_zero_line[256];  // zero-initialised module global: the source of zero rows
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;
__device__ __forceinline__ void glds16(const float* g, float* l) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)l, 16, 0, 0);
}
struct CfgTNg : CfgTN {  // unpadded B rows
  static constexpr int LDB = CfgTN::BN;
  static constexpr int B_STAGE = CfgTN::BK * CfgTN::BN;
};
constexpr int WG_GLDS_SMEM = 3 * (CfgTNg::A_STAGE + CfgTNg::B_STAGE);
constexpr bool kWgradGldsShape = CfgTN::BM == 512 && CfgTN::BN == 128 && CfgTN::BK == 16 && CfgTN::NTH == 512 &&
                                 !CfgTN::A_KC && !CfgTN::B_KC && !CfgTN::X6S;
constexpr int WG_SMEM = (SMAML_WGRAD_GLDS && kWgradGldsShape && WG_GLDS_SMEM > CfgTN::SMEM_FLOATS) ? WG_GLDS_SMEM
                                                                                                    : CfgTN::SMEM_FLOATS;

// K-tile at row k0 into one stage: per wave 4 A half-rows + 1 B instruction (2 rows).
__device__ __forceinline__ void wg_issue(const float* A, int64_t K, const WgB& b, int n0, int64_t k0, float* As,
                                         float* Bs) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int row = 2 * w + r;
    const int64_t k = k0 + row;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const float* src = k < K ? A + k * CfgTN::BM + half * 256 + 4 * lane : g_zero_line + 4 * (lane & 31);
      glds16(src, As + row * CfgTN::LDA + half * 256);
    }
  }
  const int row = 2 * w + (lane >> 5), col = 4 * (lane & 31);
  const int64_t k = k0 + row;
  const float* src;
  if (n0 < b.c1) {
    src = k < K ? b.B1 + k * b.c1 + n0 + col : g_zero_line + col;
  } else {
    const int64_t k2 = k - b.Mshift;
    src = (k < K && k2 >= 0) ? b.B2 + k2 * b.c2 + (n0 - b.c1) + col : g_zero_line + col;
  }
  glds16(src, Bs + 2 * w * CfgTN::BN);
}

template <class Hook>
__device__ __forceinline__ void wgrad_glds_loop(const float* A, int64_t K, const WgB& b, int n0, int64_t kbeg,
                                                int64_t kend, Acc<CfgTN>& acc, float* smem, Hook& hook) {
  float* As = smem;
  float* Bs = smem + 3 * CfgTNg::A_STAGE;
  const int nkt = (int)((kend - kbeg + CfgTN::BK - 1) / CfgTN::BK);
  if (nkt <= 0) return;
  wg_issue(A, K, b, n0, kbeg, As, Bs);
  if (nkt > 1) wg_issue(A, K, b, n0, kbeg + CfgTN::BK, As + CfgTNg::A_STAGE, Bs + CfgTNg::B_STAGE);
  Acc<CfgTNg>& accg = reinterpret_cast<Acc<CfgTNg>&>(acc);
  for (int kt = 0; kt < nkt; ++kt) {
    if (kt + 1 < nkt)
      asm volatile("s_waitcnt vmcnt(5)" ::: "memory");  // this tile landed; the next one may not have
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");  // every wave's share landed; stage (kt+2)%3 is free
    const int st = kt % 3;
    if (kt + 2 < nkt) {
      const int s2 = (kt + 2) % 3;
      wg_issue(A, K, b, n0, kbeg + (int64_t)(kt + 2) * CfgTN::BK, As + s2 * CfgTNg::A_STAGE,
               Bs + s2 * CfgTNg::B_STAGE);
    }
    hook(As + st * CfgTNg::A_STAGE, kt);
#if SMAML_PRIO
    __builtin_amdgcn_s_setprio(1);
#endif
    mma_tile<CfgTNg, SMAML_WGRAD_GLDS_IGLP>(As + st * CfgTNg::A_STAGE, Bs + st * CfgTNg::B_STAGE, accg, hook);
#if SMAML_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
  }
}

// Square weight-gradient tiles for the launches whose column count is a multiple of 256 (LSTM layers
// >= 1: [x | h] = 256 columns, so each workgroup covers ALL of them): 256 x 256, 8 waves of 64 x 128.
// Against the 512 x 128 tile (whose two column tiles each load and split the whole 512-row A) a
// K-tile loads and splits (256 + 256) instead of (512 + 128) rows per 256 x 128 x 2 MFMA work, 20 %
// less staging per product (micro: 196 -> 208 TF/s, profiles/r03_wgrad_tile_micro.log).
#ifndef SMAML_WGRAD_WIDE
#define SMAML_WGRAD_WIDE 1
#endif
#ifndef SMAML_TW_BN
#define SMAML_TW_BN 256  // (A/B arm: 128 with SMAML_TW_WN 1 = 256 x 128 tiles of 4 waves, two workgroups per CU)
#endif
#ifndef SMAML_TW_WN
#define SMAML_TW_WN 2
#endif
using CfgTW = GemmCfg<256, SMAML_TW_BN, 4, SMAML_TW_WN, false, false, SMAML_TN_BK, SMAML_X6_WGRAD, SMAML_TN_NST, false>;
template <class C>
constexpr int wgrad_smem_floats() {
  return std::is_same<C, CfgTN>::value ? WG_SMEM : C::SMEM_FLOATS;
}

// One weight-gradient workgroup: block L of a launch over ((ngroups + 7) / 8 * 8 * ntile) blocks.
// Pair (A2 != null): slices [nsplit1, nsplit) of each task sum a second problem of the same shape,
// A2^T [B1s | B2s] (the tangent weight gradient's dG^T [Rx | Rh] beside R(dG)^T [x | h]), into the
// same partial slabs; its slices carry no bias column (zeros).
template <class C, class LA, class LB, class Hook>
__device__ __forceinline__ void wgrad_mainloop(const LA& la, const LB& lb, int m0, int n0, int kbeg, int kend,
                                               Acc<C>& acc, float* smem, Hook& hook) {
  gemm_mainloop<C, kWgradIG>(la, lb, m0, n0, kbeg, kend, acc, smem, hook);
}

struct WgPair {
  const float* A2;
  const float *B1s, *B2s;
  int nsplit1;
};
// Layer 0's input-weight gradient over the distinct stream rows of consecutive windows (kernels.h
// XgDedup row order): B row k = the F row of compact row k (XgRowsA's mapping), A = the row sums of dG0
// (launch_dg_rowsum).
struct WgBGather {
  WgB b;
  int M, N, T;
  FastDiv ndiv;
  int compact;
  __device__ __forceinline__ float4 operator()(int64_t k, int j) const {
    if (k >= b.K || j >= b.c1) return f4zero();
    int64_t row = k;
    if (k >= M && !compact) {
      const int rr = (int)(k - M);
      const int s1 = (int)ndiv.div((uint32_t)rr);
      const int s = s1 + 1, t = min(s, T - 1);
      row = (int64_t)t * M + (int64_t)(s - t) * N + (rr - s1 * N);
    }
    return ld4(b.B1 + row * b.c1 + j);
  }
};
template <class C, bool DROP, bool GATHER = false>
__device__ __forceinline__ void wgrad_block(int L, const float* __restrict__ A, int64_t a_zstride, int Mrows, WgB lb,
                                            int64_t b1_zstride, int64_t b2_zstride, int64_t kchunk, int ntn, int ntile,
                                            int nsplit, int ngroups, float* __restrict__ part, int ldp, int with_bias,
                                            const Drop& dr, int drop_layer, float* smem, const WgPair& pr,
                                            const WgGather& ga = WgGather{}) {
  // XCD-aware: the ntile output tiles of one (split, task) group stream the same K rows of
  // A and B, so they are placed on one XCD (blocks 8 apart) to share its L2. Speed only.
  const int j = L >> 3;
  const int g = (j / ntile) * 8 + (L & 7), tile = j - (j / ntile) * ntile;
  if (g >= ngroups) return;
  const int z = g / nsplit, split = g - z * nsplit;
  const int tm = tile / ntn, tn = tile - tm * ntn;
  const bool sec = pr.A2 != nullptr && split >= pr.nsplit1;  // this slice belongs to the pair's second problem
  if (sec) {
    A = pr.A2;
    lb.B1 = pr.B1s;
    lb.B2 = pr.B2s;
  }
  if (sec) with_bias = 0;
  RowMajorMC la{A + (int64_t)z * a_zstride, lb.K, Mrows};
  WgB b = lb;
  if (b.B1) b.B1 += (int64_t)z * b1_zstride;
  if (b.B2) b.B2 += (int64_t)z * b2_zstride;
  const int64_t kbeg = (int64_t)(sec ? split - pr.nsplit1 : split) * kchunk;
  const int64_t kend = kbeg + kchunk < lb.K ? kbeg + kchunk : lb.K;
  const int m0 = tm * C::BM, n0 = tn * C::BN;
  Acc<C> acc;
  acc.zero();
  ColSumHook<C> hook;
  // k indices exceed int range only in the loaders (int64 there); the mainloop
  // passes kbeg + kt*BK as int, so K per task must stay below 2^31 (T*M*... ok).
  if constexpr (GATHER) {
    const WgBGather bg{b, ga.M, ga.N, ga.T, ga.ndiv, ga.compact};
    if (tn == 0 && with_bias) {
      wgrad_mainloop<C>(la, bg, m0, n0, (int)kbeg, (int)kend, acc, smem, hook);
    } else {
      NoHook nh;
      wgrad_mainloop<C>(la, bg, m0, n0, (int)kbeg, (int)kend, acc, smem, nh);
    }
  } else if (DROP) {
    const WgBDrop bd{b, XDrop{drop_site(dr.seed, 2, dr.step, drop_layer), dr.thr_lstm, dr.sc_lstm,
                              (uint64_t)dr.task_id[z] * (uint64_t)lb.K * lb.c1, lb.c1}};
    if (tn == 0 && with_bias) {
      wgrad_mainloop<C>(la, bd, m0, n0, (int)kbeg, (int)kend, acc, smem, hook);
    } else {
      NoHook nh;
      wgrad_mainloop<C>(la, bd, m0, n0, (int)kbeg, (int)kend, acc, smem, nh);
    }
  } else if (std::is_same<C, CfgTN>::value && SMAML_WGRAD_GLDS && kWgradGldsShape && Mrows == CfgTN::BM && lb.c1 % CfgTN::BN == 0 &&
             lb.c2 % CfgTN::BN == 0) {
    const float* Az = A + (int64_t)z * a_zstride;
    if constexpr (std::is_same<C, CfgTN>::value) {
      if (tn == 0 && with_bias) {
        wgrad_glds_loop(Az, lb.K, b, n0, kbeg, kend, acc, smem, hook);
      } else {
        NoHook nh;
        wgrad_glds_loop(Az, lb.K, b, n0, kbeg, kend, acc, smem, nh);
      }
    }
  } else if (tn == 0 && with_bias) {
    // (branch-free tile loaders for both operands measured slower here twice: with the f32 MFMA,
    // wgrad 723 -> 820 ms per meta-step, profiles/r02_ab_wgrad_gcn_tile_loaders.log; with the staged
    // bf16x6 split and 256 x 256 tiles, 498 -> 552 ms, profiles/r03_ab_wgrad_tile_loaders.log)
    wgrad_mainloop<C>(la, b, m0, n0, (int)kbeg, (int)kend, acc, smem, hook);
  } else {
    NoHook nh;
    wgrad_mainloop<C>(la, b, m0, n0, (int)kbeg, (int)kend, acc, smem, nh);
  }
  const int ncols = lb.c1 + lb.c2;
  float* P = part + ((int64_t)z * nsplit + split) * (int64_t)Mrows * ldp;
#pragma unroll
  for (int i = 0; i < C::WTM; ++i)
#pragma unroll
    for (int jj = 0; jj < C::WTN; ++jj) {
      const int c = n0 + acc_col<C>(jj);
      if (c >= ncols) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + acc_row<C>(i, r);
        if (row < Mrows) P[(int64_t)row * ldp + c] = acc.v[i][jj][r];
      }
    }
  if (tn == 0) hook.store(P, m0, Mrows, ldp, ncols, with_bias != 0, smem);
}

template <class C, bool DROP, bool GATHER = false>
__global__ __launch_bounds__(C::NTH) void k_wgrad(const float* __restrict__ A, int64_t a_zstride, int Mrows,
                                              WgB lb, int64_t b1_zstride, int64_t b2_zstride, int64_t kchunk,
                                              int ntn, int ntile, int nsplit, int ngroups, float* __restrict__ part,
                                              int ldp, int with_bias, Drop dr, int drop_layer, WgPair pr,
                                              WgGather ga) {
  __shared__ float smem[wgrad_smem_floats<C>()];
  wgrad_block<C, DROP, GATHER>((int)blockIdx.x, A, a_zstride, Mrows, lb, b1_zstride, b2_zstride, kchunk, ntn, ntile,
                               nsplit, ngroups, part, ldp, with_bias, dr, drop_layer, smem, pr, ga);
}

// Row sums of layer 0's dG over the (window, step) slots of each distinct stream row of consecutive
// windows, in the XgDedup row order (kernels.h): row r < M is slot (t = 0, m = r) itself; stream row s
// (r = M + (s - 1) N + n) sums slots (t = s - b, m = b N + n) for b = max(0, s - T + 1) .. min(B - 1, s - 1)
// in ascending b. Then dW_ih0 = S^T F_rows over (2B + T - 2) N rows instead of T B N (F2: the GCN
// features of a stream row are the same in every window). One thread per (row, 4 gate columns).
__global__ __launch_bounds__(NT) void k_dg_rowsum(const float* __restrict__ dG, int64_t a_zstride, int M, int N, int B,
                                                  int T, int G4, int rows, FastDiv ndiv, float* __restrict__ S,
                                                  int64_t s_zstride) {
  const int z = blockIdx.y;
  const int q4 = G4 / 4;
  const int64_t e = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (e >= (int64_t)rows * q4) return;
  const int r = (int)(e / q4), c = 4 * (int)(e - (int64_t)r * q4);
  const float* g = dG + (int64_t)z * a_zstride + c;
  float4 v;
  if (r < M) {
    v = ld4(g + (int64_t)r * G4);
  } else {
    const int rr = r - M;
    const int s1 = (int)ndiv.div((uint32_t)rr);
    const int s = s1 + 1, n = rr - s1 * N;
    const int b0 = max(0, s - (T - 1)), b1 = min(B - 1, s - 1);
    v = f4zero();
    for (int b = b0; b <= b1; ++b) {
      const float4 x = ld4(g + ((int64_t)(s - b) * M + (int64_t)b * N + n) * G4);
      v.x += x.x;
      v.y += x.y;
      v.z += x.z;
      v.w += x.w;
    }
  }
  st4(S + (int64_t)z * s_zstride + (int64_t)r * G4 + c, v);
}

void launch_dg_rowsum(hipStream_t s, const Dims& d, const Work& w, const float* dG0, int64_t a_zstride, float* S) {
  const int rows = (int)xg_dedup_rows(w.B, d.T, d.N);
  const int G4 = 4 * d.H;
  const int64_t n = (int64_t)rows * (G4 / 4);
  dim3 grid((unsigned)((n + NT - 1) / NT), w.Z);
  k_dg_rowsum<<<grid, NT, 0, s>>>(dG0, a_zstride, w.M, d.N, w.B, d.T, G4, rows, FastDiv((uint32_t)d.N), S,
                                  (int64_t)rows * G4);
}

// Several weight gradients in ONE launch (the LSTM layers of a small-grid backward: at batch 1 each
// layer alone fills too little of the chip and its K loop is short). Problem q owns blocks
// [blk[q], blk[q+1]) and partial slabs from part + poff[q].
template <bool DROP>
__global__ __launch_bounds__(CfgTN::NTH) void k_wgrad_multi(WgMulti mp, Drop dr) {
  __shared__ float smem[WG_SMEM];
  int q = 0;
  for (int i = 1; i < mp.n; ++i)
    if ((int)blockIdx.x >= mp.blk[i]) q = i;
  const WgradPlan& p = mp.p[q];
  WgB lb;
  lb.B1 = p.B1;
  lb.B2 = p.B2;
  lb.c1 = p.c1;
  lb.c2 = p.c2;
  lb.K = p.K;
  lb.Mshift = p.Mshift;
  if (DROP && p.drop_layer >= 0)
    wgrad_block<CfgTN, true>((int)blockIdx.x - mp.blk[q], p.A, p.a_zstride, p.Mrows, lb, p.b1_zstride, p.b2_zstride,
                      p.kchunk, p.ntn, p.ntm * p.ntn, p.nsplit, p.nsplit * p.Z, p.part, p.ldp, p.with_bias ? 1 : 0,
                      dr, p.drop_layer, smem, WgPair{});
  else
    wgrad_block<CfgTN, false>((int)blockIdx.x - mp.blk[q], p.A, p.a_zstride, p.Mrows, lb, p.b1_zstride, p.b2_zstride,
                       p.kchunk, p.ntn, p.ntm * p.ntn, p.nsplit, p.nsplit * p.Z, p.part, p.ldp, p.with_bias ? 1 : 0,
                       dr, -1, smem, WgPair{});
}

#ifndef SMAML_REDUCE_UNROLL
#define SMAML_REDUCE_UNROLL 8
#endif
__device__ __forceinline__ void wgrad_reduce_elem(const float* __restrict__ part, int nsplit, int Mrows, int ldp,
                                                  int c1, int c2, float* __restrict__ grad, int64_t P, int64_t off_w1,
                                                  int64_t off_w2, int64_t off_b1, int64_t off_b2, int accumulate,
                                                  int z, int64_t e) {
  const int64_t total = (int64_t)Mrows * ldp;
  if (e >= total) return;
  const float* p = part + (int64_t)z * nsplit * total + e;
  float v = 0.f;
  // loads issued REDUCE_UNROLL at a time, summed in split order (same result as one at a time)
  int s = 0;
  for (; s + SMAML_REDUCE_UNROLL <= nsplit; s += SMAML_REDUCE_UNROLL) {
    float x[SMAML_REDUCE_UNROLL];
#pragma unroll
    for (int u = 0; u < SMAML_REDUCE_UNROLL; ++u) x[u] = p[(int64_t)(s + u) * total];
#pragma unroll
    for (int u = 0; u < SMAML_REDUCE_UNROLL; ++u) v += x[u];
  }
  for (; s < nsplit; ++s) v += p[(int64_t)s * total];
  const int i = (int)(e / ldp), j = (int)(e - (int64_t)i * ldp);
  float* g = grad + (int64_t)z * P;
  float* dst;
  if (j < c1) {
    dst = g + off_w1 + (int64_t)i * c1 + j;
  } else if (j < c1 + c2) {
    dst = g + off_w2 + (int64_t)i * c2 + (j - c1);
  } else {
    if (accumulate || off_b1 < 0) return;  // bias written by the first (bias-carrying) pass / no bias here
    g[off_b1 + i] = v;
    if (off_b2 >= 0) g[off_b2 + i] = v;
    return;
  }
  *dst = accumulate ? *dst + v : v;
}

__global__ void k_wgrad_reduce(const float* __restrict__ part, int nsplit, int Mrows, int ldp, int c1, int c2,
                               float* __restrict__ grad, int64_t P, int64_t off_w1, int64_t off_w2,
                               int64_t off_b1, int64_t off_b2, int accumulate) {
  wgrad_reduce_elem(part, nsplit, Mrows, ldp, c1, c2, grad, P, off_w1, off_w2, off_b1, off_b2, accumulate,
                    (int)blockIdx.y, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

// Problem q's reduce owns blocks [rblk[q], rblk[q+1]) of the x dimension.
__global__ void k_wgrad_reduce_multi(WgMulti mp) {
  int q = 0;
  for (int i = 1; i < mp.n; ++i)
    if ((int)blockIdx.x >= mp.rblk[i]) q = i;
  const WgradPlan& p = mp.p[q];
  wgrad_reduce_elem(p.part, p.nsplit, p.Mrows, p.ldp, p.c1, p.c2, p.grad, p.P, p.off_w1, p.off_w2, p.off_b1, p.off_b2,
                    p.accumulate ? 1 : 0, (int)blockIdx.y,
                    ((int64_t)blockIdx.x - mp.rblk[q]) * blockDim.x + threadIdx.x);
}

void plan_wgrad(const Work& w, const float* A, int64_t a_zstride, int Mrows, const float* B1, int64_t b1_zstride,
                int c1, const float* B2, int64_t b2_zstride, int c2, int64_t K, int Mshift, float* grad, int64_t P,
                int64_t off_w1, int64_t off_w2, int64_t off_b1, int64_t off_b2, bool with_bias, bool accumulate,
                WgradPlan& p, bool multi) {
  const int ncols = c1 + c2;
  const int ldp = ncols + 1;
  const bool wide = !multi && SMAML_WGRAD_WIDE && w.kn.wgrad_wide && CfgTW::X6S && ncols % CfgTW::BN == 0 &&
                    Mrows % CfgTW::BM == 0;
  const int BMc = wide ? CfgTW::BM : CfgTN::BM, BNc = wide ? CfgTW::BN : CfgTN::BN;

  static_assert(CfgTW::BK == CfgTN::BK, "one split-K K-tile for both tiles");
  const int ntm = (Mrows + BMc - 1) / BMc;
  const int ntn = (ncols + BNc - 1) / BNc;
  const int64_t ktiles = (K + CfgTN::BK - 1) / CfgTN::BK;
  // aim for SMAML_WGRAD_THREADS threads in all, at least 8 K-tiles per split, bounded by the slab buffer
  const int nth = wide ? CfgTW::NTH : CfgTN::NTH;
  int64_t nsplit = (SMAML_WGRAD_THREADS / nth) / ((int64_t)ntm * ntn * w.Z);
  if (nsplit < 1) nsplit = 1;
  constexpr int64_t min_kt = 8;
  if (nsplit > ktiles / min_kt) nsplit = ktiles / min_kt > 0 ? ktiles / min_kt : 1;
  const int64_t per_split = (int64_t)w.Z * Mrows * ldp;
  if (nsplit * per_split > w.wpart_floats) nsplit = w.wpart_floats / per_split;
  if (nsplit < 1) nsplit = 1;
  int64_t kt_per = (ktiles + nsplit - 1) / nsplit;
  const int64_t kchunk = kt_per * CfgTN::BK;
  nsplit = (K + kchunk - 1) / kchunk;
  p.A = A;
  p.a_zstride = a_zstride;
  p.Mrows = Mrows;
  p.B1 = B1;
  p.B2 = B2;
  p.c1 = c1;
  p.c2 = c2;
  p.K = K;
  p.Mshift = Mshift;
  p.b1_zstride = b1_zstride;
  p.b2_zstride = b2_zstride;
  p.grad = grad;
  p.P = P;
  p.off_w1 = off_w1;
  p.off_w2 = off_w2;
  p.off_b1 = off_b1;
  p.off_b2 = off_b2;
  p.with_bias = with_bias;
  p.accumulate = accumulate;
  p.Z = w.Z;
  p.part = w.wpart;
  p.ldp = ldp;
  p.ntm = ntm;
  p.ntn = ntn;
  p.nsplit = (int)nsplit;
  p.kchunk = kchunk;
  p.wide = wide;
}

bool pair_wgrad(WgradPlan& p, const Work& w, const float* A2, const float* B1s, const float* B2s) {
  const int64_t ktiles = (p.K + CfgTN::BK - 1) / CfgTN::BK;
  const int64_t n1 = std::max<int64_t>(1, p.nsplit / 2);
  int64_t kt_per = (ktiles + n1 - 1) / n1;
  const int64_t kchunk = kt_per * CfgTN::BK;
  const int64_t nsplit1 = (p.K + kchunk - 1) / kchunk;
  // 2 * nsplit1 slices can exceed the planned count (a plan of one slice gives two); check them
  // against the partial-slab buffer and leave the plan unpaired if they do not fit
  if (2 * nsplit1 * p.Z * (int64_t)p.Mrows * p.ldp > w.wpart_floats) return false;
  p.kchunk = kchunk;
  p.nsplit1 = (int)nsplit1;
  p.nsplit = 2 * p.nsplit1;
  p.A2 = A2;
  p.B1s = B1s;
  p.B2s = B2s;
  return true;
}

void launch_wgrad_gemm(hipStream_t s, const WgradPlan& p) {
  WgB lb;
  lb.B1 = p.B1;
  lb.B2 = p.B2;
  lb.c1 = p.c1;
  lb.c2 = p.c2;
  lb.K = p.K;
  lb.Mshift = p.Mshift;
  const int ntile = p.ntm * p.ntn;
  const int ngroups = p.nsplit * p.Z;
  dim3 grid((unsigned)(((ngroups + 7) / 8) * 8 * ntile));
  const bool drop = p.drop_layer >= 0 && p.drop.lstm();
#define SMAML_WGRAD_LAUNCH(CFG, D_)                                                                            \
  k_wgrad<CFG, D_><<<grid, CFG::NTH, 0, s>>>(p.A, p.a_zstride, p.Mrows, lb, p.b1_zstride, p.b2_zstride, p.kchunk, \
                                             p.ntn, ntile, p.nsplit, ngroups, p.part, p.ldp, p.with_bias ? 1 : 0, \
                                             p.drop, D_ ? p.drop_layer : -1, WgPair{p.A2, p.B1s, p.B2s, p.nsplit1}, \
                                             WgGather{})
  if (p.gather.M > 0) {  // (dropout-free by construction: plan_wgrad_gather)
    const WgPair np{nullptr, nullptr, nullptr, 0};
    if (p.wide)
      k_wgrad<CfgTW, false, true><<<grid, CfgTW::NTH, 0, s>>>(p.A, p.a_zstride, p.Mrows, lb, p.b1_zstride,
                                                              p.b2_zstride, p.kchunk, p.ntn, ntile, p.nsplit, ngroups,
                                                              p.part, p.ldp, p.with_bias ? 1 : 0, p.drop, -1, np,
                                                              p.gather);
    else
      k_wgrad<CfgTN, false, true><<<grid, CfgTN::NTH, 0, s>>>(p.A, p.a_zstride, p.Mrows, lb, p.b1_zstride,
                                                              p.b2_zstride, p.kchunk, p.ntn, ntile, p.nsplit, ngroups,
                                                              p.part, p.ldp, p.with_bias ? 1 : 0, p.drop, -1, np,
                                                              p.gather);
  } else if (p.wide) {
    if (drop)
      SMAML_WGRAD_LAUNCH(CfgTW, true);
    else
      SMAML_WGRAD_LAUNCH(CfgTW, false);
  } else if (drop) {
    SMAML_WGRAD_LAUNCH(CfgTN, true);
  } else {
    SMAML_WGRAD_LAUNCH(CfgTN, false);
  }
#undef SMAML_WGRAD_LAUNCH
}

void launch_wgrad_reduce(hipStream_t s, const WgradPlan& p) {
  const int64_t total = (int64_t)p.Mrows * p.ldp;
  dim3 g2((unsigned)((total + 255) / 256), p.Z);
  k_wgrad_reduce<<<g2, 256, 0, s>>>(p.part, p.nsplit, p.Mrows, p.ldp, p.c1, p.c2, p.grad, p.P, p.off_w1,
                                    p.off_w2, p.off_b1, p.off_b2, p.accumulate ? 1 : 0);
}

void launch_wgrad(hipStream_t s, const Dims& d, const Work& w, const float* A, int64_t a_zstride,
                  int Mrows, const float* B1, int64_t b1_zstride, int c1, const float* B2,
                  int64_t b2_zstride, int c2, int64_t K, int Mshift, float* grad, int64_t P,
                  int64_t off_w1, int64_t off_w2, int64_t off_b1, int64_t off_b2, bool with_bias,
                  bool accumulate) {
  (void)d;
  WgradPlan p;
  plan_wgrad(w, A, a_zstride, Mrows, B1, b1_zstride, c1, B2, b2_zstride, c2, K, Mshift, grad, P, off_w1, off_w2,
             off_b1, off_b2, with_bias, accumulate, p);
  launch_wgrad_gemm(s, p);
  launch_wgrad_reduce(s, p);
}

// All problems share Z; each gets nsplit = (target workgroups / all tiles) slices of its K range
// (at least 8 K-tiles each), the partial slabs laid out one problem after another in w.wpart.
void launch_wgrad_multi(hipStream_t s, const Work& w, WgradPlan* ps, int n, int target_wgs) {
  int64_t tiles = 0;
  for (int q = 0; q < n; ++q) tiles += (int64_t)ps[q].ntm * ps[q].ntn * ps[q].Z;
  int64_t floats = 0;
  for (int q = 0; q < n; ++q) floats += (int64_t)ps[q].Z * ps[q].Mrows * ps[q].ldp;
  WgMulti mp{};
  mp.n = n;
  int blk = 0, rblk = 0;
  int64_t off = 0;
  for (int q = 0; q < n; ++q) {
    WgradPlan& p = ps[q];
    const int64_t ktiles = (p.K + CfgTN::BK - 1) / CfgTN::BK;
    int64_t ns = std::max<int64_t>(1, target_wgs / std::max<int64_t>(1, tiles));
    if (ns >= 8 && p.Z == 1) ns = ns / 8 * 8;  // whole octets of groups: no padding blocks past target_wgs
    ns = std::min<int64_t>(ns, std::max<int64_t>(1, ktiles / 8));
    ns = std::min<int64_t>(ns, std::max<int64_t>(1, w.wpart_floats / std::max<int64_t>(1, floats)));
    p.kchunk = ((ktiles + ns - 1) / ns) * CfgTN::BK;
    p.nsplit = (int)((p.K + p.kchunk - 1) / p.kchunk);
    p.part = w.wpart + off;
    off += (int64_t)p.nsplit * p.Z * p.Mrows * p.ldp;
    mp.p[q] = p;
    mp.blk[q] = blk;
    blk += ((p.nsplit * p.Z + 7) / 8) * 8 * p.ntm * p.ntn;
    mp.rblk[q] = rblk;
    rblk += (int)(((int64_t)p.Mrows * p.ldp + 255) / 256);
  }
  const bool drop = w.drop.lstm();
  if (drop)
    k_wgrad_multi<true><<<blk, CfgTN::NTH, 0, s>>>(mp, w.drop);
  else
    k_wgrad_multi<false><<<blk, CfgTN::NTH, 0, s>>>(mp, w.drop);
  k_wgrad_reduce_multi<<<dim3(rblk, ps[0].Z), 256, 0, s>>>(mp);
}

// ====================================================================================
// GCNConv backward helpers (the module API's STGCN / GCNConv autograd, model.py:7-52; off the hybrid
// hot path, where the GCN is frozen). Row gather: out[r] = sum over the adjacency list of row r of
// w * src[col] for r < n_gather (the ELL of A_hat for the forward aggregation, or the CSR of A_hat^T
// for the backward one), out[r] = src[r] for the other rows. One float4 of one row per thread, fixed
// summation order (deterministic).
__global__ void k_gather_rows(const float* __restrict__ src, float* __restrict__ out, int rows, int cols,
                              int n_gather, const int* __restrict__ ell_c, const float* __restrict__ ell_v,
                              const int* __restrict__ csr_p, const int* __restrict__ csr_c,
                              const float* __restrict__ csr_v) {
  const int q4 = cols / 4;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)rows * q4) return;
  const int r = (int)(i / q4), k = 4 * (int)(i - (int64_t)r * q4);
  float4 v;
  if (r < n_gather) {
    v = f4zero();
    if (csr_p) {
      for (int e = csr_p[r]; e < csr_p[r + 1]; ++e) v = fma4(csr_v[e], ld4(src + (int64_t)csr_c[e] * cols + k), v);
    } else {
#pragma unroll
      for (int e = 0; e < ELLW; ++e) {
        const float wv = ell_v[r * ELLW + e];
        if (wv != 0.f) v = fma4(wv, ld4(src + (int64_t)ell_c[r * ELLW + e] * cols + k), v);
      }
    }
  } else {
    v = ld4(src + (int64_t)r * cols + k);
  }
  st4(out + (int64_t)r * cols + k, v);
}

void launch_gather_rows(hipStream_t s, const float* src, float* out, int rows, int cols, int n_gather, const int* ell_c,
                        const float* ell_v, const int* csr_p, const int* csr_c, const float* csr_v) {
  const int64_t n = (int64_t)rows * (cols / 4);
  k_gather_rows<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(src, out, rows, cols, n_gather, ell_c, ell_v, csr_p,
                                                            csr_c, csr_v);
}

// g *= (h > 0): the ReLU derivative taken from the (post-ReLU, post-dropout) activation h
__global__ void k_relu_mask(float* __restrict__ g, const float* __restrict__ h, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    g[i] = h[i] > 0.f ? g[i] : 0.f;
}

void launch_relu_mask(hipStream_t s, float* g, const float* h, int64_t n) {
  int nb = (int)((n + 255) / 256);
  if (nb > 4096) nb = 4096;
  k_relu_mask<<<nb, 256, 0, s>>>(g, h, n);
}

// out = A . W  (A [rows][K] row-major, W [K][ncols] row-major): k_gemm_nn on one problem
void launch_gemm_nn_plain(hipStream_t s, const float* A, int rows, int K, const float* W, int ncols, float* out) {
  dim3 grid((rows + CfgNN::BM - 1) / CfgNN::BM, (ncols + CfgNN::BN - 1) / CfgNN::BN, 1);
  k_gemm_nn<<<grid, CfgNN::NTH, 0, s>>>(A, 0, rows, K, W, 0, 0, ncols, out, 0);
}

// out[z] = A[z] . W[z]^T, both operands K-contiguous ([rows][K], [ncols][K]); the batch-1 forward's
// hoisted layer-0 input projection (XG[t*M + m][n] = F[t][m] . W_ih0[n] for all T steps in one
// throughput-bound launch instead of inside every latency-bound wavefront diagonal).
#ifndef SMAML_GEMM_NT_BIG
#define SMAML_GEMM_NT_BIG 0  // k_gemm_nt tiles: 0 = CfgGateP (128 x 128, 4 waves), 1 = CfgGate (256 x 128, 8 waves)
#endif
using CfgNT2 = std::conditional_t<SMAML_GEMM_NT_BIG != 0, CfgGate, CfgGateP>;
__global__ __launch_bounds__(CfgNT2::NTH) void k_gemm_nt(const float* __restrict__ A, int64_t a_zstride, int rows,
                                                       int K, const float* __restrict__ W, int64_t w_zstride,
                                                       int ncols, float* __restrict__ out, int64_t o_zstride) {
  __shared__ float smem[CfgNT2::SMEM_FLOATS];
  const int z = blockIdx.z;
  const int m0 = blockIdx.x * CfgNT2::BM, n0 = blockIdx.y * CfgNT2::BN;
  Acc<CfgNT2> acc;
  acc.zero();
  gemm_mainloop<CfgNT2>(RowMajorKC{A + (int64_t)z * a_zstride, rows, K}, RowMajorKC{W + (int64_t)z * w_zstride, ncols, K},
                        m0, n0, 0, K, acc, smem);
  float* o = out + (int64_t)z * o_zstride;
#pragma unroll
  for (int i = 0; i < CfgNT2::WTM; ++i)
#pragma unroll
    for (int j = 0; j < CfgNT2::WTN; ++j) {
      const int c = n0 + acc_col<CfgNT2>(j);
      if (c >= ncols) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + acc_row<CfgNT2>(i, r);
        if (row < rows) o[(int64_t)row * ncols + c] = acc.v[i][j][r];
      }
    }
}

void launch_gemm_nt(hipStream_t s, const float* A, int64_t a_zstride, int rows, int K, const float* W,
                    int64_t w_zstride, int ncols, float* out, int64_t o_zstride, int Z) {
  dim3 grid((rows + CfgNT2::BM - 1) / CfgNT2::BM, (ncols + CfgNT2::BN - 1) / CfgNT2::BN, Z);
  k_gemm_nt<<<grid, CfgNT2::NTH, 0, s>>>(A, a_zstride, rows, K, W, w_zstride, ncols, out, o_zstride);
}

// ====================================================================================
// clip_grad_norm_ + SGD, per task z. Squared norm accumulated in fp64, fixed order.
__global__ void k_sqsum(const float* __restrict__ g, int64_t P, double* __restrict__ part) {
  __shared__ double red[NT / 64];
  const int z = blockIdx.y;
  const float* gz = g + (int64_t)z * P;
  const int64_t per = (P + SQB - 1) / SQB;
  const int64_t b = (int64_t)blockIdx.x * per, e = b + per < P ? b + per : P;
  double acc = 0.0;
  // (unrolled: the loads of 8 iterations in flight together; the same additions in the same order)
#pragma unroll 8
  for (int64_t i = b + threadIdx.x; i < e; i += NT) {
    const double v = gz[i];
    acc += v * v;
  }
  const double s = block_sum_d(acc, red);
  if (threadIdx.x == 0) part[(int64_t)z * SQB + blockIdx.x] = s;
}


__device__ __forceinline__ float clip_coef_from(const double* part, float max_norm, float* total_out) {
  double t = 0.0;
  for (int i = 0; i < SQB; ++i) t += part[i];
  const float total = (float)sqrt(t);
  if (total_out) *total_out = total;
  const float coef = max_norm / (total + 1e-6f);
  return coef < 1.f ? coef : 1.f;
}



// The inner SGD step as ONE kernel (train_hybrid_maml_v5.py:135-139: clip_grad_norm_ + SGD): every
// block computes the fp64 squared-norm partials of its (task, chunk) items -- the partition and order
// of k_sqsum -- then, after a grid barrier, each task's clip coefficient from its SQB partials in
// order and the SGD update of the same chunks (still in L2). `phases`: 1 = partials only, 2 = update
// only, 3 = both with the grid barrier between them (grid sized by grid_barrier_blocks; see
// grid_barrier for the bounded wait). The two-launch form (1 then 2) is bitwise equal to the fused one.
__global__ __launch_bounds__(NT) void k_inner_sgd(float* __restrict__ theta, const float* __restrict__ g, int64_t P,
                                                  int Z, double* __restrict__ part, float lr, float max_norm,
                                                  float* norm_out, float* coef_out, GridBar gb, int phases) {
  __shared__ double red[NT / 64];
  const int nit = SQB * Z;
  const int64_t per = (P + SQB - 1) / SQB;
  if (phases & 1) {
    for (int it = blockIdx.x; it < nit; it += gridDim.x) {
      const int z = it / SQB, b = it - z * SQB;
      const float* gz = g + (int64_t)z * P;
      const int64_t beg = (int64_t)b * per, end = beg + per < P ? beg + per : P;
      double acc = 0.0;
      for (int64_t i = beg + threadIdx.x; i < end; i += NT) {
        const double v = gz[i];
        acc += v * v;
      }
      const double sum = block_sum_d(acc, red);
      if (threadIdx.x == 0) part[it] = sum;
    }
  }
  if (phases == 3 && !grid_barrier(gb, gridDim.x)) return;
  if (!(phases & 2)) return;
  for (int it = blockIdx.x; it < nit; it += gridDim.x) {
    const int z = it / SQB, b = it - z * SQB;
    float total;
    const float coef = clip_coef_from(part + (int64_t)z * SQB, max_norm, &total);
    if (b == 0 && threadIdx.x == 0) {
      if (norm_out) norm_out[z] = total;
      if (coef_out) coef_out[z] = coef;
    }
    float* tz = theta + (int64_t)z * P;
    const float* gz = g + (int64_t)z * P;
    const int64_t beg = (int64_t)b * per, end = beg + per < P ? beg + per : P;
    for (int64_t i = beg + threadIdx.x; i < end; i += NT) tz[i] = fmaf(-lr, gz[i] * coef, tz[i]);
  }
}

// (queried once per (kernel, device) and cached)
int grid_barrier_capacity(const void* fn) {
  static std::mutex mu;
  static std::vector<std::pair<std::pair<const void*, int>, int>> cache;
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lk(mu);
  for (auto& e : cache)
    if (e.first.first == fn && e.first.second == dev) return e.second;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, NT, 0) != hipSuccess) return 0;
  const int cap = per_cu > 0 && cus > 0 ? per_cu * cus : 0;
  cache.push_back({{fn, dev}, cap});
  return cap;
}

int grid_barrier_blocks(const void* fn, int items, int oversize) {
  return grid_barrier_grid(grid_barrier_capacity(fn), items, oversize);
}

hipError_t launch_inner_sgd(hipStream_t s, float* theta, const float* g, int64_t P, int Z, double* part, float lr,
                            float max_norm, float* norm_out, float* coef_out, const BarPlan& bp) {
  const int items = SQB * Z;
  const int nb = bp.fused ? grid_barrier_blocks((const void*)k_inner_sgd, items, bp.oversize) : 0;
  if (nb > 0) {
    k_inner_sgd<<<nb, NT, 0, s>>>(theta, g, P, Z, part, lr, max_norm, norm_out, coef_out, bp.gb, 3);
  } else {
    const int n2 = items < 1024 ? items : 1024;
    k_inner_sgd<<<n2, NT, 0, s>>>(theta, g, P, Z, part, lr, max_norm, norm_out, coef_out, bp.gb, 1);
    k_inner_sgd<<<n2, NT, 0, s>>>(theta, g, P, Z, part, lr, max_norm, norm_out, coef_out, bp.gb, 2);
  }
  return hipGetLastError();
}

__global__ void k_sum_tasks(const float* __restrict__ g, int64_t P, int Z, float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int z = 0; z < Z; ++z) v += g[(int64_t)z * P + i];
    out[i] = v;
  }
}

void launch_sum_tasks(hipStream_t s, const float* g, int64_t P, int Z, float* out) {
  int nb = (int)((P + NT - 1) / NT);
  if (nb > 2048) nb = 2048;
  k_sum_tasks<<<nb, NT, 0, s>>>(g, P, Z, out);
}

__global__ void k_broadcast(const float* __restrict__ theta, int64_t P, float* __restrict__ out) {
  const int z = blockIdx.y;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x)
    out[(int64_t)z * P + i] = theta[i];
}

void launch_broadcast(hipStream_t s, const float* theta, int64_t P, int Z, float* out) {
  int nb = (int)((P + NT - 1) / NT);
  if (nb > 1024) nb = 1024;
  k_broadcast<<<dim3(nb, Z), NT, 0, s>>>(theta, P, out);
}

// ====================================================================================
// Outer step: clip_grad_norm_(max_norm) on the (all-reduced) meta-gradient, then
// torch.optim.AdamW (decoupled weight decay, lerp first moment).
__global__ void k_adamw(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                        float* __restrict__ v, int64_t n, const double* __restrict__ part, float lr, float b1,
                        float b2, float eps, float wd, float step, float bc2_sqrt, float max_norm,
                        float* norm_out) {
  float total;
  const float coef = clip_coef_from(part, max_norm, &total);
  if (blockIdx.x == 0 && threadIdx.x == 0 && norm_out) *norm_out = total;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i] * coef;
    float pi = p[i] * (1.f - lr * wd);
    const float mi = m[i] + (1.f - b1) * (gi - m[i]);
    const float vi = v[i] * b2 + (1.f - b2) * gi * gi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi - step * (mi / denom);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

void launch_adamw(hipStream_t s, float* p, const float* g, float* m, float* v, int64_t n, double* part,
                  float lr, float b1, float b2, float eps, float wd, float step_size, float bc2_sqrt,
                  float max_norm, float* norm_out) {
  k_sqsum<<<dim3(SQB, 1), NT, 0, s>>>(g, n, part);
  int nb = (int)((n + NT - 1) / NT);
  if (nb > 2048) nb = 2048;
  k_adamw<<<nb, NT, 0, s>>>(p, g, m, v, n, part, lr, b1, b2, eps, wd, step_size, bc2_sqrt, max_norm, norm_out);
}

// ====================================================================================
// Regional adaptation step (adapt_hybrid_v5.py:196-201): clip_grad_norm_(max_norm) then
// torch.optim.Adam with coupled L2 weight decay (g += wd * p), per-step learning rate.
// bc1 = 1 - b1^step and bc2_sqrt = sqrt(1 - b2^step) come from the host (the step is a host integer):
// a per-thread fp64 pow was most of this kernel's time at batch 1.
__global__ void k_adam_l2(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                          float* __restrict__ v, int64_t n, const double* __restrict__ part, const float* __restrict__ lr_dev,
                          double bc1, float bc2_sqrt, float b1, float b2, float eps, float wd, float max_norm,
                          const float* __restrict__ lpart, int lblocks, float inv_count, float* __restrict__ loss) {
  if (loss && blockIdx.x == 0) {  // the step's loss from the head's partials: k_loss_final's sum, same order
    __shared__ float red[NT / 64];
    float a = 0.f;
    for (int i = threadIdx.x; i < lblocks; i += NT) a += lpart[i];
    const float s = block_sum(a, red);
    if (threadIdx.x == 0) *loss = s * inv_count;
  }
  float total;
  const float coef = clip_coef_from(part, max_norm, &total);
  const float lr = *lr_dev;
  const float step_size = (float)((double)lr / bc1);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = fmaf(wd, p[i], g[i] * coef);
    const float mi = m[i] + (1.f - b1) * (gi - m[i]);
    const float vi = v[i] * b2 + (1.f - b2) * gi * gi;
    p[i] = p[i] - step_size * (mi / (sqrtf(vi) / bc2_sqrt + eps));
    m[i] = mi;
    v[i] = vi;
  }
}

// (measured: the same update as ONE grid-barrier launch -- k_sqsum's partials, a grid barrier over ~512
// blocks, the element update -- took 81 us per sample-step against 23 for these two launches,
// profiles/r04_rocprof_adapt_kw.md: 512 arrivals on one counter cost more than a launch boundary)
void launch_adam_l2(hipStream_t s, float* p, const float* g, float* m, float* v, int64_t n, double* part,
                    const float* lr_dev, int step, float b1, float b2, float eps, float wd, float max_norm,
                    const float* lpart, int lblocks, float inv_count, float* loss) {
  int nb = (int)((n + NT - 1) / NT);
  if (nb > 2048) nb = 2048;
  k_sqsum<<<dim3(SQB, 1), NT, 0, s>>>(g, n, part);
  const double bc1 = 1.0 - std::pow((double)b1, step), bc2 = 1.0 - std::pow((double)b2, step);
  k_adam_l2<<<nb, NT, 0, s>>>(p, g, m, v, n, part, lr_dev, bc1, (float)std::sqrt(bc2), b1, b2, eps, wd, max_norm,
                              lpart, lblocks, inv_count, loss);
}

}  // namespace smaml

namespace smaml {
// Product form per GEMM family as built (smaml_build_info): 0 = f32 MFMA, 1 = bf16x6 with the
// split on the MFMA fragments, 2 = bf16x6 with the split staged at the LDS store.
template <class C>
constexpr int product_form() {
  return C::X6S ? 2 : C::X6 ? 1 : 0;
}
const char* products_info() {
  static char buf[256];
  snprintf(buf, sizeof buf,
           "products(0=f32 MFMA, 1=bf16x6 fragment split, 2=bf16x6 staged split): gcn=%d gate=%d gate_dual=%d "
           "bptt=%d bptt_dual=%d wgrad=%d",
           product_form<CfgGcn>(), product_form<CfgGate>(), SMAML_X6_GATED ? (SMAML_X6_GATED == 2 ? 2 : 1) : 0,
           product_form<CfgBwd>(), SMAML_X6_BWDD ? (SMAML_X6_BWDD == 2 ? 2 : 1) : 0, product_form<CfgTN>());
  return buf;
}
}  // namespace smaml
