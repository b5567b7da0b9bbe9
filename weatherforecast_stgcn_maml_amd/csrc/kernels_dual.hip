// Second-order MAML: forward-over-reverse Hessian-vector products through the LSTM + head.
//
// For inner step k the meta-backward needs  H_k w  (H_k = Hessian of the step-k support
// loss at theta_k, w = the clip-adjusted meta-gradient direction). Every kernel here
// recomputes the primal quantity of its reference counterpart (kernels.hip) and, in the
// same launch, its directional derivative R{.} along w (Pearlmutter's R-operator):
//   k_lstm_fwd_dual    pre, R(pre) = [x|h|Rx|Rh].[U_ih|U_hh|W_ih|W_hh]^T + U_b  ->  gates, c, h and tangents
//   k_head_dual        pred, R(pred) -> dpred, R(dpred)
//   k_gemm_nn_dual     dh_T / dX and their tangents ([R(A) | A] . [W ; U])
//   k_lstm_bwd_dual    BPTT cell step and its tangent (product rule through every gate)
// The tangent weight gradient R(dW) = R(dG)^T [x|h] + dG^T [Rx|Rh] reuses k_wgrad (layers >= 1:
// one paired launch, layer 0: two accumulating passes). All contractions take f32 operands with
// f32 accumulation through gemm_core.h (f32-accurate bf16x6 products by default).
#include "kernels.h"
#include "loaders.h"

namespace smaml {

#ifndef SMAML_DUAL_BK
#define SMAML_DUAL_BK 16
#endif
// The BPTT / dX / head duals stage four operand tiles per K-tile (gemm_dual_mainloop);
// BK=16 keeps them at 54-80 KiB of LDS (two or more workgroups per CU).
using CfgGateD = GemmCfg<32 * SMAML_GATED_WM, 128 * SMAML_GATE_WN, SMAML_GATED_WM, SMAML_GATE_WN, true, true, SMAML_GATE_BK, SMAML_X6_GATED,
                         SMAML_GATE_NST>;
using CfgNTD = GemmCfg<128, 128, 2, 2, true, true, SMAML_DUAL_BK, SMAML_X6_BWDD>;
using CfgNND = GemmCfg<64, 128, 2, 2, true, false, SMAML_DUAL_BK, SMAML_X6_BWDD>;

__device__ __forceinline__ float block_sum_f(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0)
    for (int i = 0; i < NT / 64; ++i) s += red[i];
  return s;
}

// ====================================================================================
// KEPT: the primal of this step (gates, c, h) is already in Hs / Cs / Gs (kept from the inner
// step for the second-order sweep): only the tangent pass runs.
// DROP: layers >= 1 read x = drop(h_{l-1}) and R x = drop(R h_{l-1}) (the same mask).
// Tangent cell epilogue of one gate tile: R(gates), R(c), R(h) from the tangent accumulators and
// the primal gates / cell this lane has (just) written or kept. Rows are handled SMAML_FWDD_EPI_RB
// at a time with all their loads issued before their stores (a row at a time serialised one
// memory round trip per row: 16 per tile); the t = 0 case loads a valid address and selects 0, and
// the row bound is checked only in the last row tile (CHECK), so the batch's loads never branch.
#ifndef SMAML_FWDD_EPI_RB
#define SMAML_FWDD_EPI_RB 4
#endif
template <int H, bool CHECK>
__device__ __forceinline__ void fwd_dual_tangent_epi(const Acc<CfgGateD>& at, const float (&bu)[4],
                                                     const float* __restrict__ Gz, float* __restrict__ RGz,
                                                     const float* __restrict__ Cz, float* __restrict__ RCz,
                                                     float* __restrict__ RHz, int rb, int j, uint32_t tM, int M,
                                                     int t) {
  constexpr int G4 = 4 * H;
  constexpr int RB = SMAML_FWDD_EPI_RB;
  static_assert(16 % RB == 0, "row batch");
  const bool past = t > 0;
  const uint32_t pM = past ? (uint32_t)M * H : 0u;
#pragma unroll
  for (int r0 = 0; r0 < 16; r0 += RB) {
    float gi[RB], gf[RB], gg[RB], go[RB], cp[RB], rcp[RB];
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      int m = rb + racc(r0 + q);
      if (CHECK) m = min(m, M - 1);
      const uint32_t row = tM + (uint32_t)m;
      const uint32_t oh = row * H + j;
      const uint32_t og = row * G4 + j;
      gi[q] = ldb(Gz, 4u * (og));
      gf[q] = ldb(Gz, 4u * (og + H));
      gg[q] = ldb(Gz, 4u * (og + 2 * H));
      go[q] = ldb(Gz, 4u * (og + 3 * H));
      cp[q] = ldb(Cz, 4u * (oh - pM));
      rcp[q] = ldb(RCz, 4u * (oh - pM));
    }
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      const int r = r0 + q;
      const int m = rb + racc(r);
      if (CHECK && m >= M) continue;
      const uint32_t row = tM + (uint32_t)m;
      const uint32_t oh = row * H + j;
      const uint32_t og = row * G4 + j;
      const float ri = gi[q] * (1.f - gi[q]) * (at.v[0][0][r] + bu[0]);
      const float rf = gf[q] * (1.f - gf[q]) * (at.v[0][1][r] + bu[1]);
      const float rg = (1.f - gg[q] * gg[q]) * (at.v[0][2][r] + bu[2]);
      const float ro = go[q] * (1.f - go[q]) * (at.v[0][3][r] + bu[3]);
      const float cpv = past ? cp[q] : 0.f, rcpv = past ? rcp[q] : 0.f;
      const float rc = lstm_cell_rc(gi[q], gf[q], gg[q], cpv, ri, rf, rg, rcpv);
      const float tc = tanhf_(lstm_cell_c(gi[q], gf[q], gg[q], cpv));
      stb(RGz, 4u * (og), ri);
      stb(RGz, 4u * (og + H), rf);
      stb(RGz, 4u * (og + 2 * H), rg);
      stb(RGz, 4u * (og + 3 * H), ro);
      stb(RCz, 4u * (oh), rc);
      stb(RHz, 4u * (oh), ro * tc + go[q] * (1.f - tc * tc) * rc);
    }
  }
}

// The same through the transposed epilogue (loaders.h gate_epilogue_t; KEPT steps, whose primal is
// read from memory anyway): per item (row, 4 units) six 16-B loads (i, f, g, o, c_{t-1},
// R c_{t-1}) and six 16-B stores (R i, R f, R g, R o, R c, R h).
template <int H>
__device__ __forceinline__ void fwd_dual_tangent_epi_t(const Acc<CfgGateD>& at, const float (&bu)[4],
                                                       const float* __restrict__ Gz, float* __restrict__ RGz,
                                                       const float* __restrict__ Cz, float* __restrict__ RCz,
                                                       float* __restrict__ RHz, int m0, int ug, uint32_t tM, int M,
                                                       int t, float* smem) {
  constexpr int G4 = 4 * H;
  const bool full = m0 + CfgGateD::BM <= M, past = t > 0;
  const uint32_t pM = past ? (uint32_t)M * H : 0u;
  struct V {
    float4 g[4], cp, rcp;
  };
  gate_epilogue_t<CfgGateD>(
      at, bu, smem,
      [&](int ml, int u) {
        const int m = full ? m0 + ml : min(m0 + ml, M - 1);  // clamped rows: valid address, not stored
        const uint32_t jq = (uint32_t)min(ug * 32 + u, H - 4);
        const uint32_t row = tM + (uint32_t)m;
        const uint32_t og = 4u * (row * G4 + jq), oh = 4u * (row * H + jq);
        V v;
#pragma unroll
        for (int g = 0; g < 4; ++g) v.g[g] = ldo(Gz, og + 4u * g * H);
        v.cp = ldo(Cz, oh - 4u * pM);
        v.rcp = ldo(RCz, oh - 4u * pM);
        return v;
      },
      [&](int ml, int u, const float4 (&rpre)[4], const V& v) {
        if ((!full && m0 + ml >= M) || ug * 32 + u >= H) return;
        const uint32_t row = tM + (uint32_t)(m0 + ml), jq = (uint32_t)(ug * 32 + u);
        const float4 cp = sel4(past, v.cp), rcp = sel4(past, v.rcp);
        float4 ri, rf, rg, ro, rc, rh;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float gi = f4get(v.g[0], e), gf = f4get(v.g[1], e), gg = f4get(v.g[2], e), go = f4get(v.g[3], e);
          const float ri_ = gi * (1.f - gi) * f4get(rpre[0], e);
          const float rf_ = gf * (1.f - gf) * f4get(rpre[1], e);
          const float rg_ = (1.f - gg * gg) * f4get(rpre[2], e);
          const float ro_ = go * (1.f - go) * f4get(rpre[3], e);
          const float cpe = f4get(cp, e);
          const float rc_ = lstm_cell_rc(gi, gf, gg, cpe, ri_, rf_, rg_, f4get(rcp, e));
          const float tc = tanhf_(lstm_cell_c(gi, gf, gg, cpe));
          f4set(ri, e, ri_);
          f4set(rf, e, rf_);
          f4set(rg, e, rg_);
          f4set(ro, e, ro_);
          f4set(rc, e, rc_);
          f4set(rh, e, ro_ * tc + go * (1.f - tc * tc) * rc_);
        }
        const uint32_t og = 4u * (row * G4 + jq), oh = 4u * (row * H + jq);
        sto(RGz, og, ri);
        sto(RGz, og + 4u * H, rf);
        sto(RGz, og + 8u * H, rg);
        sto(RGz, og + 12u * H, ro);
        sto(RCz, oh, rc);
        sto(RHz, oh, rh);
      });
}

// IMG: the weight tiles of theta and U come from their pre-split images (launch_split_gate).
// xd.xg / xd.rxg (layer 0, set by the launcher only for this step's theta / U): layer 0's input
// projections F W_ih0^T and F U_ih0^T of the step's consecutive windows (kernels.h XgDedup) start the
// primal / tangent accumulators, whose K loops then skip the input segment (R x = 0 at layer 0).
template <int H, bool KEPT, bool DROP, bool IMG>
__global__ SMAML_GATED_ATTR __launch_bounds__(CfgGateD::NTH) void k_lstm_fwd_dual(const float* __restrict__ F,
                                                      float* __restrict__ HsAll, float* __restrict__ CsAll,
                                                      float* __restrict__ GsAll, float* __restrict__ RHsAll,
                                                      float* __restrict__ RCsAll, float* __restrict__ RGsAll,
                                                      int64_t lsz, const float* __restrict__ theta,
                                                      const float* __restrict__ U, int64_t tstride, FwdWave wv,
                                                      int T, int M, Drop dr, GateImgs gi, XgDedup xd) {
  __shared__ float smem[CfgGateD::SMEM_FLOATS];
  constexpr int G4 = 4 * H;
  int l, t, b0;
  LayerOff lo;
  const Blk bk = xcd_block();
  wave_problem(wv, bk.x, l, t, lo, b0);
  const float* X = l == 0 ? F : HsAll + (int64_t)(l - 1) * lsz;
  const float* RX = l == 0 ? nullptr : RHsAll + (int64_t)(l - 1) * lsz;
  float* Hs = HsAll + (int64_t)l * lsz;
  float* Cs = CsAll + (int64_t)l * lsz;
  float* Gs = GsAll + (int64_t)l * lsz * 4;
  float* RHs = RHsAll + (int64_t)l * lsz;
  float* RCs = RCsAll + (int64_t)l * lsz;
  float* RGs = RGsAll + (int64_t)l * lsz * 4;
  const int z = bk.z;
  const float* th = theta + (int64_t)z * tstride;
  const float* u = U + (int64_t)z * tstride;
  const int cin = lo.cin;
  const char* ith = IMG ? gi.th + (int64_t)z * gi.tstride : nullptr;
  const char* iu = IMG ? gi.u + (int64_t)z * gi.tstride : nullptr;
  int64_t io0 = 0, io1 = 0;  // layer l's image offsets (W_ih | W_hh), selected with scalar compares
  if constexpr (IMG) {
#pragma unroll
    for (int q = 0; q < MAX_LAYERS; ++q)
      if (q == l) {
        io0 = gi.off[q][0];
        io1 = gi.off[q][1];
      }
  }
  const int64_t slab = (int64_t)z * T * M;
  float* Gz = Gs + slab * G4;
  float* RGz = RGs + slab * G4;
  float* Cz = Cs + slab * H;
  float* RCz = RCs + slab * H;
  float* Hz = Hs + slab * H;
  float* RHz = RHs + slab * H;
  const float* xt = X + (slab + (int64_t)t * M) * cin;
  const float* rxt = RX ? RX + (slab + (int64_t)t * M) * cin : nullptr;
  const float* hp = t > 0 ? Hz + (int64_t)(t - 1) * M * H : nullptr;
  const float* rhp = t > 0 ? RHz + (int64_t)(t - 1) * M * H : nullptr;
  const int wh = hp ? H : 0;
  int tm, ug;
  constexpr int UPB = CfgGateD::WAVES_N;  // 32-unit groups per workgroup
  if (!gate_tile(bk.x - b0, wv.ntm ? wv.ntm : (M + CfgGateD::BM - 1) / CfgGateD::BM, (H + 32 * UPB - 1) / (32 * UPB),
                 tm, ug))
    return;
  tm += wv.tm0;
  const int m0 = tm * CfgGateD::BM, n0 = ug * CfgGateD::BN;
  XDrop xdr{};
  if (DROP && l > 0)
    xdr = XDrop{drop_site(dr.seed, 2, dr.step, l - 1), dr.thr_lstm, dr.sc_lstm,
                ((uint64_t)dr.task_id[z] * T + t) * M * H, H};

  // Register diet: the primal epilogue runs between the two passes (its accumulators die
  // there), and the tangent epilogue re-reads the gates / cell it needs from the lines this
  // lane has just written (program order: a lane sees its own stores). One accumulator set
  // is live at a time.
  const int j = (ug * UPB + (int)(threadIdx.x >> 6) % UPB) * 32 + (threadIdx.x & 31);
  const int rb = m0 + acc_row<CfgGateD>(0, 0);
  const bool full = m0 + CfgGateD::BM <= M;
  const uint32_t tM = (uint32_t)t * (uint32_t)M;
  const bool xg0 = !DROP && l == 0;  // (the XgDedup tables hold layer 0's rows; no dropout variant reads them)
  const int64_t xgo = (int64_t)z * xd.zstride + xg_dedup_row0(t, M, xd.N) * G4;
  if (!KEPT) {
    Acc<CfgGateD> ap;
    int kb = 0;
    if (xg0 && xd.xg) {
      acc_load_gates<CfgGateD, H>(ap, xd.xg + xgo, m0, ug, M);
      kb = cin;
    } else {
      ap.zero();
    }
    SegKC la{{xt, hp, nullptr, nullptr}, {cin, wh, 0, 0}, M};
    SegGateB lb{{th + lo.wih, th + lo.whh, nullptr, nullptr}, {cin, wh, 0, 0}, H};
    if (DROP && l > 0)
      gemm_mainloop<CfgGateD, SMAML_IGLP>(SegKCDrop{la, xdr}, lb, m0, n0, 0, cin + wh, ap, smem);
    else if constexpr (IMG)
      gemm_mainloop<CfgGateD, SMAML_IGLP>(SegKCt<2>{{xt, hp}, {cin, wh}, M}, SegGateImg<2>{{ith + io0, ith + io1}, {cin, wh}},
                                          m0, n0, kb, cin + wh, ap, smem);
    else
      gemm_mainloop<CfgGateD, SMAML_IGLP>(SegKCt<2>{{xt, hp}, {cin, wh}, M},
                                          SegGateBt<2>{{th + lo.wih, th + lo.whh}, {cin, wh}, H}, m0, n0, kb,
                                          cin + wh, ap, smem);
    if (j < H) {
      float bp[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) bp[g] = th[lo.bih + g * H + j] + th[lo.bhh + g * H + j];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = rb + racc(r);
        if (!full && m >= M) continue;
        const uint32_t row = tM + (uint32_t)m;
        const uint32_t oh = row * H + j;
        const uint32_t og = row * G4 + j;
        const float gi = sigmoidf_(ap.v[0][0][r] + bp[0]);
        const float gf = sigmoidf_(ap.v[0][1][r] + bp[1]);
        const float gg = tanhf_(ap.v[0][2][r] + bp[2]);
        const float go = sigmoidf_(ap.v[0][3][r] + bp[3]);
        const float cp = t > 0 ? ldb(Cz, 4u * (oh - (uint32_t)M * H)) : 0.f;
        const float c = lstm_cell_c(gi, gf, gg, cp);
        stb(Gz, 4u * (og), gi);
        stb(Gz, 4u * (og + H), gf);
        stb(Gz, 4u * (og + 2 * H), gg);
        stb(Gz, 4u * (og + 3 * H), go);
        stb(Cz, 4u * (oh), c);
        stb(Hz, 4u * (oh), go * tanhf_(c));
      }
    }
  }
  Acc<CfgGateD> at;
  int kb = 0;
  if (xg0 && xd.rxg) {
    acc_load_gates<CfgGateD, H>(at, xd.rxg + xgo, m0, ug, M);
    kb = cin;
  } else {
    at.zero();
  }
  {
    const int wrx = rxt ? cin : 0;
    SegKC la{{xt, hp, rxt, rhp}, {cin, wh, wrx, wh}, M};
    SegGateB lb{{u + lo.wih, u + lo.whh, th + lo.wih, th + lo.whh}, {cin, wh, wrx, wh}, H};
    if (DROP && l > 0)
      gemm_mainloop<CfgGateD, SMAML_IGLP>(SegKCDrop{la, xdr}, lb, m0, n0, 0, cin + wh + wrx + wh, at, smem);
    else if constexpr (IMG)
      gemm_mainloop<CfgGateD, SMAML_IGLP>(SegKCt<4>{{xt, hp, rxt, rhp}, {cin, wh, wrx, wh}, M},
                                          SegGateImg<4>{{iu + io0, iu + io1, ith + io0, ith + io1}, {cin, wh, wrx, wh}},
                                          m0, n0, kb, cin + wh + wrx + wh, at, smem);
    else
      gemm_mainloop<CfgGateD, SMAML_IGLP>(SegKCt<4>{{xt, hp, rxt, rhp}, {cin, wh, wrx, wh}, M},
                                          SegGateBt<4>{{u + lo.wih, u + lo.whh, th + lo.wih, th + lo.whh},
                                                       {cin, wh, wrx, wh}, H},
                                          m0, n0, kb, cin + wh + wrx + wh, at, smem);
  }
  if constexpr (KEPT && SMAML_FWD_EPI_T && CfgGateD::WAVES_N == 1) {
    // (KEPT: the primal gates come from memory; the non-kept path re-reads the gates this lane itself
    // stored above, which needs the accumulator-layout epilogue's lane <-> element mapping)
    float bu[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) bu[g] = j < H ? u[lo.bih + g * H + j] + u[lo.bhh + g * H + j] : 0.f;
    fwd_dual_tangent_epi_t<H>(at, bu, Gz, RGz, Cz, RCz, RHz, m0, ug, tM, M, t, smem);
    return;
  }
  if (j >= H) return;
  float bu[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) bu[g] = u[lo.bih + g * H + j] + u[lo.bhh + g * H + j];
  if (full)
    fwd_dual_tangent_epi<H, false>(at, bu, Gz, RGz, Cz, RCz, RHz, rb, j, tM, M, t);
  else
    fwd_dual_tangent_epi<H, true>(at, bu, Gz, RGz, Cz, RCz, RHz, rb, j, tM, M, t);
}

void launch_lstm_fwd_dual_wave(hipStream_t s, const Dims& d, const Work& w, int diag, const float* theta,
                               const float* U, int64_t tstride, const ParamOff& po, double* flops, int chunk, int nch) {
  const int64_t lsz = (int64_t)w.Z * d.T * w.M * d.H;
  const int ntm = (w.M + CfgGateD::BM - 1) / CfgGateD::BM;
  const int ngrp = (d.H + 32 * CfgGateD::WAVES_N - 1) / (32 * CfgGateD::WAVES_N);
  FwdWave wv{};
  const double fl = fwd_wave(d, w, po, diag, gate_blocks(ntm, ngrp), true, wv);
  if (flops) *flops = fl;
  if (wv.n == 0) return;
  if (nch > 1) {  // this launch's row tiles only (see launch_lstm_fwd_wave)
    const int lo = (int)((int64_t)ntm * chunk / nch), hi = (int)((int64_t)ntm * (chunk + 1) / nch);
    if (hi <= lo) return;
    fwd_wave(d, w, po, diag, gate_blocks(hi - lo, ngrp), true, wv);
    wv.tm0 = lo;
    wv.ntm = hi - lo;
  }
  dim3 grid(wv.off[wv.n], 1, w.Z);
  const bool kept = w.primal_kept != 0, drop = w.drop.lstm();
  count_variant(w, kept ? V_FWDD_KEPT : V_FWDD);
  const bool img = !drop && w.gimg.th && w.gimg.u && w.gimg_src == theta && w.gimg_u_src == U;
  if (img) count_variant(w, V_FWDD_IMG);
  XgDedup xd = w.xgd;  // (tables of other weights are never read)
  if (xd.src != theta || kept) xd.xg = nullptr;
  if (xd.u_src != U) xd.rxg = nullptr;
#define SMAML_FWD_DUAL(K_, D_)                                                                  \
  if (img)                                                                                      \
    SMAML_DISPATCH_H(d.H, (k_lstm_fwd_dual<HT, K_, D_, !(D_)><<<grid, CfgGateD::NTH, 0, s>>>(    \
                              w.F, w.Hs, w.Cs, w.Gs, w.RHs, w.RCs, w.RGs, lsz, theta, U, tstride, wv, \
                              d.T, w.M, w.drop, w.gimg, xd)))                                   \
  else                                                                                          \
    SMAML_DISPATCH_H(d.H, (k_lstm_fwd_dual<HT, K_, D_, false><<<grid, CfgGateD::NTH, 0, s>>>(    \
                              w.F, w.Hs, w.Cs, w.Gs, w.RHs, w.RCs, w.RGs, lsz, theta, U, tstride, wv, \
                              d.T, w.M, w.drop, w.gimg, xd)))
  if (kept && drop) {
    SMAML_FWD_DUAL(true, true);
  } else if (kept) {
    SMAML_FWD_DUAL(true, false);
  } else if (drop) {
    SMAML_FWD_DUAL(false, true);
  } else {
    SMAML_FWD_DUAL(false, false);
  }
#undef SMAML_FWD_DUAL
}

// ====================================================================================
__global__ __launch_bounds__(NT) void k_head_dual(const float* __restrict__ hT, const float* __restrict__ RhT,
                                                  int64_t zstride, const float* __restrict__ theta,
                                                  const float* __restrict__ U, int64_t tstride, int64_t wo,
                                                  int64_t bo, const float* const* __restrict__ xtab,
                                                  float* __restrict__ dpred, float* __restrict__ Rdpred, int M,
                                                  int H, int HfC, int N, int Hf, int C, int T, int cin0, int B,
                                                  float dscale) {
  __shared__ float smem[DualStage<CfgNTD>::FLOATS];
  const int z = blockIdx.z;
  const float* th = theta + (int64_t)z * tstride;
  const float* u = U + (int64_t)z * tstride;
  const float* h = hT + (int64_t)z * zstride;
  const float* rh = RhT + (int64_t)z * zstride;
  const int m0 = blockIdx.x * CfgNTD::BM;
  Acc<CfgNTD> ap, at;
  ap.zero();
  at.zero();
  {
    RowMajorKC la{h, M, H};
    RowMajorKC la2{rh, M, H};
    RowMajorKC lb{th + wo, HfC, H};
    RowMajorKC lb2{u + wo, HfC, H};
    gemm_dual_mainloop<CfgNTD>(la, la2, lb, lb2, m0, 0, H, 0, ap, at, smem);
  }
#pragma unroll
  for (int i = 0; i < CfgNTD::WTM; ++i)
#pragma unroll
    for (int jj = 0; jj < CfgNTD::WTN; ++jj) {
      const int cc = acc_col<CfgNTD>(jj);
      if (cc >= HfC) continue;
      const float bc = th[bo + cc], ubc = u[bo + cc];
      const int hh = cc / C, c = cc - hh * C;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + acc_row<CfgNTD>(i, r);
        if (m >= M) continue;
        const float p = ap.v[i][jj][r] + bc;
        const float rp = at.v[i][jj][r] + ubc;
        const int s = m / N, n = m - s * N;
        const int rr = n * Hf + hh;
        const int hp = rr / N, np = rr - hp * N;
        const float y = xtab[z * B + s][((int64_t)(T + 1 + hp) * N + np) * cin0 + c];
        const int64_t o = ((int64_t)z * M + m) * HfC + cc;
        dpred[o] = dscale * (p - y);
        Rdpred[o] = dscale * rp;
      }
    }
}

void launch_head_dual(hipStream_t s, const Dims& d, const Work& w, const float* theta, const float* U,
                      int64_t tstride, const ParamOff& po, const float* const* xtab, float dscale) {
  const int64_t lsz = (int64_t)w.Z * d.T * w.M * d.H;
  const int64_t off = (int64_t)(d.L - 1) * lsz + (int64_t)(d.T - 1) * w.M * d.H;
  if (w.drop.lstm()) {  // drop(h_T), R drop(h_T) = drop(R h_T)
    launch_drop_rows(s, w, d.H, w.Hs + off, (int64_t)d.T * w.M * d.H, w.hTd);
    launch_drop_rows(s, w, d.H, w.RHs + off, (int64_t)d.T * w.M * d.H, w.RhTd);
  }
  int64_t hz = 0;
  const float* hT = head_input(d, w, false, &hz);
  const float* RhT = head_input(d, w, true, &hz);
  dim3 grid((w.M + CfgNTD::BM - 1) / CfgNTD::BM, 1, w.Z);
  k_head_dual<<<grid, NT, 0, s>>>(hT, RhT, hz, theta, U, tstride, po.wo,
                                  po.bo, xtab, w.dpred, w.Rdpred, w.M, d.H, d.HfC, d.N, d.Hf, d.C, d.T, d.Cin0, w.B,
                                  dscale);
}

// ====================================================================================
// out = A . W ;  Rout = [RA | A] . [W ; U_W]     (W, U_W: [K][ncols] at woff in theta / U)
__global__ __launch_bounds__(NT) void k_gemm_nn_dual(const float* __restrict__ A, const float* __restrict__ RA,
                                                     int64_t a_zstride, int rows, int K,
                                                     const float* __restrict__ theta, const float* __restrict__ U,
                                                     int64_t tstride, int64_t woff, int ncols, float* __restrict__ out,
                                                     float* __restrict__ Rout, int64_t o_zstride) {
  __shared__ float smem[DualStage<CfgNND>::FLOATS];
  const int z = blockIdx.z;
  const float* a = A + (int64_t)z * a_zstride;
  const float* ra = RA + (int64_t)z * a_zstride;
  const float* W = theta + (int64_t)z * tstride + woff;
  const float* UW = U + (int64_t)z * tstride + woff;
  const int m0 = blockIdx.x * CfgNND::BM, n0 = blockIdx.y * CfgNND::BN;
  Acc<CfgNND> ap, at;
  ap.zero();
  at.zero();
  {
    RowMajorKC la{a, rows, K};
    RowMajorKC la2{ra, rows, K};
    RowMajorMC lb{W, K, ncols};
    RowMajorMC lb2{UW, K, ncols};
    gemm_dual_mainloop<CfgNND>(la, la2, lb, lb2, m0, n0, K, 0, ap, at, smem);
  }
  float* o = out + (int64_t)z * o_zstride;
  float* ro = Rout + (int64_t)z * o_zstride;
#pragma unroll
  for (int jj = 0; jj < CfgNND::WTN; ++jj) {
    const int c = n0 + acc_col<CfgNND>(jj);
    if (c >= ncols) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + acc_row<CfgNND>(0, r);
      if (m >= rows) continue;
      o[(int64_t)m * ncols + c] = ap.v[0][jj][r];
      ro[(int64_t)m * ncols + c] = at.v[0][jj][r];
    }
  }
}

void launch_head_dh_dual(hipStream_t s, const Dims& d, const Work& w, const float* theta, const float* U,
                         int64_t tstride, const ParamOff& po) {
  dim3 grid((w.M + CfgNND::BM - 1) / CfgNND::BM, (d.H + CfgNND::BN - 1) / CfgNND::BN, w.Z);
  k_gemm_nn_dual<<<grid, CfgNND::NTH, 0, s>>>(w.dpred, w.Rdpred, (int64_t)w.M * d.HfC, w.M, d.HfC, theta, U, tstride, po.wo,
                                     d.H, w.dH, w.RdH, (int64_t)w.M * d.H);
  if (w.drop.lstm()) {  // back through drop(h_T): the same mask on dh_T and R dh_T
    launch_drop_rows(s, w, d.H, w.dH, (int64_t)w.M * d.H, w.dH);
    launch_drop_rows(s, w, d.H, w.RdH, (int64_t)w.M * d.H, w.RdH);
  }
}

// ====================================================================================
#ifndef SMAML_DIAG_BWDD
#define SMAML_DIAG_BWDD 0  // timing diagnostics only (wrong results): 1 = kept tangent BPTT without its
#endif                     // epilogue, 2 = without its GEMM
using CfgNNDs = GemmCfg<64, 64, 2, 2, true, false, SMAML_DUAL_BK, SMAML_X6_BWDD>;
using CfgBwdD = GemmCfg<SMAML_BWD_BM, 128, SMAML_BWD_WM, SMAML_BWD_WN, true, false, SMAML_DUAL_BK, SMAML_X6_BWDD>;
// Kept-step epilogue in two row halves (BM*BN/2 floats of transpose LDS): with the swizzled MC weight
// images the staged stage is 48 KB, so the 128 x 128 tangent BPTT runs three workgroups per CU.
#ifndef SMAML_BWDD_HALFEPI
#define SMAML_BWDD_HALFEPI (SMAML_X6 ? 1 : 0)
#endif
#ifndef SMAML_BWDD_MIN_LDS
#define SMAML_BWDD_MIN_LDS 0  // A/B: pad the tangent BPTT's LDS to at least this many bytes (e.g. 56 KB: 2 WGs per CU)
#endif
template <class C>
constexpr int bwdd_smem_floats() {
  constexpr int E = (SMAML_BWDD_HALFEPI && C::WAVES_M == 2) ? C::BM * C::BN / 2 : C::BM * C::BN;
  constexpr int S = C::X6S ? DualStage<C>::X6S_FLOATS : DualStage<C>::FLOATS;
  constexpr int F = S > E ? S : E;
  return F > SMAML_BWDD_MIN_LDS / 4 ? F : SMAML_BWDD_MIN_LDS / 4;
}

// Tangent-only cell backward of a kept step (see kernels.hip bwd_cell_): R(dh) = the GEMM
// accumulators, transposed through LDS so each lane works on float4 groups of 4 hidden units of
// one row (16-B loads / stores); the primal cell backward is re-derived from the kept dh. Writes
// R(dG) in place over R(G) (each item's elements are read before they are written) and both
// cell-state carries.
#ifndef SMAML_NT_BWDD
#define SMAML_NT_BWDD 0  // tangent BPTT: streaming (nt) loads / stores for everything but the weights
#endif
template <bool NT>
__device__ __forceinline__ float4 ld4_(const float* p) {
  if constexpr (NT) return ld4_nt(p); else return ld4(p);
}
template <bool NT>
__device__ __forceinline__ void st4_(float* p, const float4& v) {
  if constexpr (NT) st4_nt(p, v); else st4(p, v);
}

template <int H, class C, bool HEAD, bool CHECK>
__device__ __forceinline__ void bwd_dual_kept_cell_(const float* smem, const float* Gz, float* RGz,
                                                    const float* __restrict__ dhz, const float* __restrict__ Cz,
                                                    const float* __restrict__ RCz, const float* __restrict__ dHz,
                                                    const float* __restrict__ RdHz, float* __restrict__ dcz,
                                                    float* __restrict__ rdcz, int m0, int n0, int t, int T, int M) {
  constexpr int G4 = 4 * H;
  constexpr int GPR = C::BN / 4;
  constexpr int NIT = C::BM * GPR / C::NTH;
  static_assert(NIT * C::NTH == C::BM * GPR, "epilogue items");
  const bool first = (t == T - 1), past = t > 0;
  const int64_t pM = past ? (int64_t)M * H : 0;
  const int64_t tM = (int64_t)t * M;
  struct V {  // c_t and R c_t are re-derived from the gates and c_{t-1} (lstm_cell_c / _rc)
    float4 dh, g[4], rg[4], cp, rcp, dc, rdc, rhd;
  };
  auto coords = [&](int k, int& r, int& m, int& j) {
    const int item = (int)threadIdx.x + C::NTH * k;
    r = item / GPR;
    m = m0 + r;
    j = n0 + 4 * (item % GPR);
  };
  auto load = [&](int k, V& v) {
    int r, m, j;
    coords(k, r, m, j);
    if (CHECK) {
      m = min(m, M - 1);
      j = min(j, H - 4);
    }
    const int64_t row = tM + m;
    const float* gp = Gz + row * G4 + j;
    const float* rp = RGz + row * G4 + j;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      v.g[g] = ld4_<SMAML_NT_BWDD != 0>(gp + g * H);
      v.rg[g] = ld4_<SMAML_NT_BWDD != 0>(rp + g * H);
    }
    v.dh = ld4_<SMAML_NT_BWDD != 0>(dhz + row * H + j);
    v.cp = ld4_<SMAML_NT_BWDD != 0>(Cz + row * H - pM + j);
    v.rcp = ld4_<SMAML_NT_BWDD != 0>(RCz + row * H - pM + j);
    v.dc = ld4_<SMAML_NT_BWDD != 0>(dcz + (int64_t)m * H + j);
    v.rdc = ld4_<SMAML_NT_BWDD != 0>(rdcz + (int64_t)m * H + j);
    if (HEAD) v.rhd = ld4_<SMAML_NT_BWDD != 0>(RdHz + (int64_t)m * H + j);
  };
  auto step = [&](int k, const V& v) {
    int r, m, j;
    coords(k, r, m, j);
    if (CHECK && (m >= M || j >= H)) return;
    const float4 acc = *reinterpret_cast<const float4*>(smem + r * C::BN + (j - n0));
    float4 o[4], odc, ordc;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float dh = f4get(v.dh, e);
      const float rdh = f4get(acc, e) + (HEAD ? f4get(v.rhd, e) : 0.f);
      const float gi = f4get(v.g[0], e), gf = f4get(v.g[1], e), gg = f4get(v.g[2], e), go = f4get(v.g[3], e);
      const float ri = f4get(v.rg[0], e), rf = f4get(v.rg[1], e), rgg = f4get(v.rg[2], e), ro = f4get(v.rg[3], e);
      const float cp = past ? f4get(v.cp, e) : 0.f, rcp = past ? f4get(v.rcp, e) : 0.f;
      const float c = lstm_cell_c(gi, gf, gg, cp), rc = lstm_cell_rc(gi, gf, gg, cp, ri, rf, rgg, rcp);
      const float dcin = first ? 0.f : f4get(v.dc, e), rdcin = first ? 0.f : f4get(v.rdc, e);
      const float tc = tanhf_(c);
      const float s2 = 1.f - tc * tc;
      const float rtc = s2 * rc;
      const float dct = dcin + dh * go * s2;
      const float rdct = rdcin + rdh * go * s2 + dh * ro * s2 - 2.f * dh * go * tc * rtc;
      const float si = gi * (1.f - gi), sf = gf * (1.f - gf), so = go * (1.f - go), sg = 1.f - gg * gg;
      const float o0 = rdct * gg * si + dct * rgg * si + dct * gg * (1.f - 2.f * gi) * ri;
      const float o1 = rdct * cp * sf + dct * rcp * sf + dct * cp * (1.f - 2.f * gf) * rf;
      const float o2 = rdct * gi * sg + dct * ri * sg - 2.f * dct * gi * gg * rgg;
      const float o3 = rdh * tc * so + dh * rtc * so + dh * tc * (1.f - 2.f * go) * ro;
      const float d0 = dct * gf, d1 = rdct * gf + dct * rf;
      if (e == 0) { o[0].x = o0; o[1].x = o1; o[2].x = o2; o[3].x = o3; odc.x = d0; ordc.x = d1; }
      if (e == 1) { o[0].y = o0; o[1].y = o1; o[2].y = o2; o[3].y = o3; odc.y = d0; ordc.y = d1; }
      if (e == 2) { o[0].z = o0; o[1].z = o1; o[2].z = o2; o[3].z = o3; odc.z = d0; ordc.z = d1; }
      if (e == 3) { o[0].w = o0; o[1].w = o1; o[2].w = o2; o[3].w = o3; odc.w = d0; ordc.w = d1; }
    }
    float* rp = RGz + (tM + m) * G4 + j;
#pragma unroll
    for (int g = 0; g < 4; ++g) st4_<SMAML_NT_BWDD != 0>(rp + g * H, o[g]);
    st4_<SMAML_NT_BWDD != 0>(dcz + (int64_t)m * H + j, odc);
    st4_<SMAML_NT_BWDD != 0>(rdcz + (int64_t)m * H + j, ordc);
  };
  V v;
#pragma unroll 1
  for (int k = 0; k < NIT; ++k) {
    load(k, v);
    step(k, v);
  }
}

// Tangent BPTT step, one anti-diagonal per launch (kernels.hip k_lstm_bwd_step; BwdWave):
//   dh  = A . B,   R(dh) = A2 . B + A . B2   with  A = [dG(l+1,t) | dG(l,t+1)],
//   A2 = [R dG(l+1,t) | R dG(l,t+1)],  B = [W_ih(l+1) ; W_hh(l)],  B2 = [U_ih(l+1) ; U_hh(l)]
// then the cell backward and its product-rule tangent; dG / R(dG) overwrite G / R(G) in place.
//
// KEPT: the step's primal BPTT is kept from the inner step (gates in GsAll, dG in dGAll, dh in
// dhAll): the GEMM forms only the tangent (R(dh) = A2 . B + A . B2), the primal cell backward is
// re-derived elementwise from the kept dh, and only R(dG) and the carries are written.
// Otherwise dGAll == GsAll (dG written in place over the gates) and dhAll is unused.
// DROP: as k_lstm_bwd_step (the layer-above segment masked by drop(h_l) before the recurrent one).
// Pair-segment tile order (knob bwdd_remap): the weight operands [W_ih(l+1); W_hh(l)] and U of a
// tile depend on its (task, problem) pair (per-task fast weights: 1 MB of f32 per pair), and in the
// hardware order every XCD holds tiles of ~7 pairs at once (3 workgroups x 32 CUs = 96 tiles per
// XCD, 111 row tiles per pair), more than its 4 MB L2 keeps. Here each pair's row tiles are cut in
// two segments, the segments are ordered problem-major and dealt to the XCDs round-robin, and XCD x
// (hardware id L % 8, in the order L / 8 it receives them) runs its segments one after another: ~2
// pairs' weights per XCD at a time, every XCD a similar mix of problems. 1-D grid; ids past the
// segments or past a short segment exit at once.
struct PairRemap {
  int on;
  int Z, R, seg, NS;  // tasks, row tiles per pair, tiles per segment, segments (= problems x Z x 2)
};
__device__ __forceinline__ bool remap_pair(const PairRemap& rm, int Lid, int& p, int& z, int& mb) {
  const int x = Lid & 7, j = Lid >> 3;
  const int slot = j / rm.seg, rin = j - slot * rm.seg;
  const int g = x + 8 * slot;
  if (g >= rm.NS) return false;
  p = g / (2 * rm.Z);
  z = (g >> 1) % rm.Z;
  mb = (g & 1) * rm.seg + rin;
  return mb < rm.R;
}

template <int H, class CfgNND, bool KEPT, bool DROP>
__global__ SMAML_BWDD_ATTR __launch_bounds__(CfgNND::NTH) void k_lstm_bwd_dual(const float* GsAll, float* dGAll,
                                                      const float* __restrict__ dhAll, float* __restrict__ RGsAll,
                                                      const float* __restrict__ CsAll, const float* __restrict__ RCsAll,
                                                      const float* __restrict__ dHhead, const float* __restrict__ RdHhead,
                                                      float* __restrict__ dcAll, float* __restrict__ RdcAll,
                                                      int64_t lsz, const float* __restrict__ theta,
                                                      const float* __restrict__ U, int64_t tstride, BwdWave wv, int L,
                                                      int T, int M, Drop dr, PairRemap rm) {
  __shared__ float smem[bwdd_smem_floats<CfgNND>()];
  constexpr int G4 = 4 * H;
  int mb, p, z, ny;
  if (rm.on) {  // 1-D grid, one column tile (H == BN)
    if (!remap_pair(rm, (int)blockIdx.x, p, z, mb)) return;
    ny = 0;
  } else {
    const Blk bk = xcd_block();
    p = bwd_block(wv, bk.x, mb);
    z = bk.z;
    ny = bk.y;
  }
  mb += wv.tm0;
  const int Zt = rm.on ? rm.Z : (int)gridDim.z;
  const int l = wave_sel(wv.l, p), t = wave_sel(wv.t, p);
  const LayerOff lo = wave_sel(wv.lo, p);
  const int64_t wih_up = wave_sel(wv.wih_up, p);
  const int m0 = mb * CfgNND::BM, n0 = ny * CfgNND::BN;
  const int64_t slab = (int64_t)z * T * M;
  const float* th = theta + (int64_t)z * tstride;
  const float* u = U + (int64_t)z * tstride;
  const float* Gz = GsAll + (int64_t)l * lsz * 4 + slab * G4;  // gates in
  float* dGz = dGAll + (int64_t)l * lsz * 4 + slab * G4;        // dG out (in place unless KEPT)
  float* RGz = RGsAll + (int64_t)l * lsz * 4 + slab * G4;       // R(gates) in, R(dG) out
  const float* dhz = dhAll + (int64_t)l * lsz + slab * H;
  const float* Cz = CsAll + (int64_t)l * lsz + slab * H;
  const float* RCz = RCsAll + (int64_t)l * lsz + slab * H;
  float* dcz = dcAll + ((int64_t)l * Zt + z) * M * H;
  float* rdcz = RdcAll + ((int64_t)l * Zt + z) * M * H;
  Acc<CfgNND> ap, at;
  ap.zero();
  at.zero();
  {
    const bool up = l + 1 < L, nx = t + 1 < T;
    const int64_t oa = (int64_t)(l + 1) * lsz * 4 + (slab + (int64_t)t * M) * G4;
    const int64_t on = (int64_t)(t + 1) * M * G4;
    const int ns = (up ? 1 : 0) + (nx ? 1 : 0);
    const int w0 = ns >= 1 ? G4 : 0, w1 = ns >= 2 ? G4 : 0;
    SegKC la{{up ? dGAll + oa : dGz + on, up ? dGz + on : nullptr, nullptr, nullptr}, {w0, w1, 0, 0}, M};
    SegKC la2{{up ? RGsAll + oa : RGz + on, up ? RGz + on : nullptr, nullptr, nullptr}, {w0, w1, 0, 0}, M};
    SegMC lb{{up ? th + wih_up : th + lo.whh, th + lo.whh}, {w0, w1}, H};
    SegMC lb2{{up ? u + wih_up : u + lo.whh, u + lo.whh}, {w0, w1}, H};
    if (DROP && up) {
      // layer-above segment masked by drop(h_l) (primal and tangent alike), then the recurrent one
      const XDrop xd{drop_site(dr.seed, 2, dr.step, l), dr.thr_lstm, dr.sc_lstm,
                     ((uint64_t)dr.task_id[z] * T + t) * M * H, H};
      gemm_dual_mainloop<CfgNND, !KEPT>(SegKC{{dGAll + oa, nullptr, nullptr, nullptr}, {G4, 0, 0, 0}, M},
                                        SegKC{{RGsAll + oa, nullptr, nullptr, nullptr}, {G4, 0, 0, 0}, M},
                                        SegMC{{th + wih_up, nullptr}, {G4, 0}, H},
                                        SegMC{{u + wih_up, nullptr}, {G4, 0}, H}, m0, n0, G4, 0, ap, at, smem);
      if (!KEPT) drop_acc<CfgNND>(ap, xd, m0, n0);
      drop_acc<CfgNND>(at, xd, m0, n0);
      if (nx)
        gemm_dual_mainloop<CfgNND, !KEPT>(SegKC{{dGz + on, nullptr, nullptr, nullptr}, {G4, 0, 0, 0}, M},
                                          SegKC{{RGz + on, nullptr, nullptr, nullptr}, {G4, 0, 0, 0}, M},
                                          SegMC{{th + lo.whh, nullptr}, {G4, 0}, H},
                                          SegMC{{u + lo.whh, nullptr}, {G4, 0}, H}, m0, n0, G4, 0, ap, at, smem);
    } else if (ns && SMAML_DIAG_BWDD != 2) {
      const float* a0 = up ? dGAll + oa : dGz + on;
      const float* r0 = up ? RGsAll + oa : RGz + on;
      const int64_t w0o = up ? wih_up : lo.whh;
      gemm_dual_mainloop<CfgNND, !KEPT>(SegKCt<2, SMAML_NT_BWDD != 0>{{a0, dGz + on}, {G4, G4}, M},
                                        SegKCt<2, SMAML_NT_BWDD != 0>{{r0, RGz + on}, {G4, G4}, M},
                                        SegMCt<2>{{th + w0o, th + lo.whh}, {G4, G4}, H},
                                        SegMCt<2>{{u + w0o, u + lo.whh}, {G4, G4}, H}, m0, n0, ns * G4, 0, ap, at,
                                        smem);
    }
  }
  const bool first = (t == T - 1);
  const bool head = first && l == L - 1;
  const float* dHz = dHhead + (int64_t)z * M * H;
  const float* RdHz = RdHhead + (int64_t)z * M * H;
  const bool full = m0 + CfgNND::BM <= M;
  if constexpr (KEPT) {
    constexpr bool HALF = SMAML_BWDD_HALFEPI && CfgNND::WAVES_M == 2;
    using EC = std::conditional_t<HALF, HalfRows<CfgNND>, CfgNND>;
#pragma unroll 1
    for (int hh = 0; hh < (HALF ? 2 : 1); ++hh) {
      if (hh) __syncthreads();  // the first half's readers are done with the LDS
      if constexpr (HALF)
        acc_to_lds_half<CfgNND>(at, smem, hh);
      else
        acc_to_lds<CfgNND>(at, smem);
      if (SMAML_DIAG_BWDD == 1) {  // timing diagnostic: GEMM phase only (keep the result live)
        if (t < 0) RGz[threadIdx.x] = smem[threadIdx.x];
        continue;
      }
      const int mh = m0 + hh * EC::BM;
      const bool nochk = mh + EC::BM <= M && n0 + EC::BN <= H;
#define SMAML_KEPT_EPI(HD, CK)                                                                          \
  bwd_dual_kept_cell_<H, EC, HD, CK>(smem, Gz, RGz, dhz, Cz, RCz, dHz, RdHz, dcz, rdcz, mh, n0, t, T, M)
      if (head) {
        if (nochk) SMAML_KEPT_EPI(true, false); else SMAML_KEPT_EPI(true, true);
      } else {
        if (nochk) SMAML_KEPT_EPI(false, false); else SMAML_KEPT_EPI(false, true);
      }
#undef SMAML_KEPT_EPI
    }
    return;
  }
  const uint32_t tM = (uint32_t)t * (uint32_t)M;
#pragma unroll
  for (int i = 0; i < CfgNND::WTM; ++i)
#pragma unroll
  for (int jj = 0; jj < CfgNND::WTN; ++jj) {
    const int j = n0 + acc_col<CfgNND>(jj);
    const int rb = m0 + acc_row<CfgNND>(i, 0);
    if (j >= H) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = rb + racc(r);
      if (!full && m >= M) continue;
      const uint32_t row = tM + (uint32_t)m;
      const uint32_t oh = row * H + j;
      const uint32_t og = row * G4 + j;
      const uint32_t oc = (uint32_t)m * H + j;
      const float dh = KEPT ? ldb(dhz, 4u * oh) : ap.v[i][jj][r] + (head ? ldb(dHz, 4u * oc) : 0.f);
      const float rdh = at.v[i][jj][r] + (head ? ldb(RdHz, 4u * oc) : 0.f);
      const float gi = ldb(Gz, 4u * (og)), gf = ldb(Gz, 4u * (og + H)), gg = ldb(Gz, 4u * (og + 2 * H)), go = ldb(Gz, 4u * (og + 3 * H));
      const float ri = ldb(RGz, 4u * (og)), rf = ldb(RGz, 4u * (og + H)), rgg = ldb(RGz, 4u * (og + 2 * H)), ro = ldb(RGz, 4u * (og + 3 * H));
      const float cp = t > 0 ? ldb(Cz, 4u * (oh - (uint32_t)M * H)) : 0.f;
      const float rcp = t > 0 ? ldb(RCz, 4u * (oh - (uint32_t)M * H)) : 0.f;
      const float c = lstm_cell_c(gi, gf, gg, cp), rc = lstm_cell_rc(gi, gf, gg, cp, ri, rf, rgg, rcp);
      const float dcin = first ? 0.f : ldb(dcz, 4u * (oc));
      const float rdcin = first ? 0.f : ldb(rdcz, 4u * (oc));
      const float tc = tanhf_(c);
      const float s2 = 1.f - tc * tc;
      const float rtc = s2 * rc;
      const float dct = dcin + dh * go * s2;
      const float rdct = rdcin + rdh * go * s2 + dh * ro * s2 - 2.f * dh * go * tc * rtc;
      const float si = gi * (1.f - gi), sf = gf * (1.f - gf), so = go * (1.f - go), sg = 1.f - gg * gg;
      if (!KEPT) {
        stb(dGz, 4u * (og), dct * gg * si);
        stb(dGz, 4u * (og + H), dct * cp * sf);
        stb(dGz, 4u * (og + 2 * H), dct * gi * sg);
        stb(dGz, 4u * (og + 3 * H), dh * tc * so);
      }
      stb(RGz, 4u * (og), rdct * gg * si + dct * rgg * si + dct * gg * (1.f - 2.f * gi) * ri);
      stb(RGz, 4u * (og + H), rdct * cp * sf + dct * rcp * sf + dct * cp * (1.f - 2.f * gf) * rf);
      stb(RGz, 4u * (og + 2 * H), rdct * gi * sg + dct * ri * sg - 2.f * dct * gi * gg * rgg);
      stb(RGz, 4u * (og + 3 * H), rdh * tc * so + dh * rtc * so + dh * tc * (1.f - 2.f * go) * ro);
      stb(dcz, 4u * (oc), dct * gf);
      stb(rdcz, 4u * (oc), rdct * gf + dct * rf);
    }
  }
}

template <class Cfg, bool KEPT>
static void bwd_dual_grid(hipStream_t s, const Dims& d, const Work& w, const BwdWave& wv, int ntn, const float* theta,
                          const float* U, int64_t tstride) {
  const int64_t lsz = (int64_t)w.Z * d.T * w.M * d.H;
  dim3 grid(wv.off[wv.n], ntn, w.Z);
  PairRemap rm{};
  const int R = wv.n > 0 ? wv.off[1] - wv.off[0] : 0;  // row tiles per problem
  if (w.kn.bwdd_remap && ntn == 1 && R >= 2) {
    rm.on = 1;
    rm.Z = w.Z;
    rm.R = R;
    rm.seg = (R + 1) / 2;
    rm.NS = wv.n * w.Z * 2;
    grid = dim3((unsigned)(8 * ((rm.NS + 7) / 8) * rm.seg), 1, 1);
  }
  const float* dh = KEPT ? w.dh : w.Gs;  // unread unless KEPT
  if (w.drop.lstm()) {
    SMAML_DISPATCH_H(d.H, k_lstm_bwd_dual<HT, Cfg, KEPT, true><<<grid, Cfg::NTH, 0, s>>>(
                              w.Gs, w.dG, dh, w.RGs, w.Cs, w.RCs, w.dH, w.RdH, w.dc, w.Rdc, lsz, theta, U, tstride,
                              wv, d.L, d.T, w.M, w.drop, rm));
  } else {
    SMAML_DISPATCH_H(d.H, k_lstm_bwd_dual<HT, Cfg, KEPT, false><<<grid, Cfg::NTH, 0, s>>>(
                              w.Gs, w.dG, dh, w.RGs, w.Cs, w.RCs, w.dH, w.RdH, w.dc, w.Rdc, lsz, theta, U, tstride,
                              wv, d.L, d.T, w.M, w.drop, rm));
  }
}

bool bwd_dual_wave_big(const Dims& d, const Work& w, const ParamOff& po, int e) {
  BwdWave wv{};
  const int ntm = (w.M + CfgBwdD::BM - 1) / CfgBwdD::BM, ntn = (d.H + CfgBwdD::BN - 1) / CfgBwdD::BN;
  bwd_wave(d, w, po, e, ntm, true, wv);
  return (int64_t)wv.n * ntm * ntn * w.Z * (CfgBwdD::BM / 64) >= w.kn.bwdd_big_min;
}

void launch_lstm_bwd_dual_wave(hipStream_t s, const Dims& d, const Work& w, int e, const float* theta,
                               const float* U, int64_t tstride, const ParamOff& po, int chunk, int nch) {
  BwdWave wv{};
  const int ntm = (w.M + CfgBwdD::BM - 1) / CfgBwdD::BM, ntn = (d.H + CfgBwdD::BN - 1) / CfgBwdD::BN;
  bwd_wave(d, w, po, e, ntm, true, wv);
  if (wv.n == 0) return;
  const bool kept = w.primal_kept != 0;
  if (nch > 1) {  // a row chunk: its own row tiles only, always the big tiles (see launch_lstm_bwd_wave)
    const int lo = (int)((int64_t)ntm * chunk / nch), hi = (int)((int64_t)ntm * (chunk + 1) / nch);
    if (hi <= lo) return;
    bwd_wave(d, w, po, e, hi - lo, true, wv);
    wv.tm0 = lo;
    count_variant(w, kept ? V_BWDD_BIG_KEPT : V_BWDD_BIG);
    if (kept)
      bwd_dual_grid<CfgBwdD, true>(s, d, w, wv, ntn, theta, U, tstride);
    else
      bwd_dual_grid<CfgBwdD, false>(s, d, w, wv, ntn, theta, U, tstride);
    return;
  }
  // (64-row tile units)
  const bool big = (int64_t)wv.n * ntm * ntn * w.Z * (CfgBwdD::BM / 64) >= w.kn.bwdd_big_min;
  if (big) {
    count_variant(w, kept ? V_BWDD_BIG_KEPT : V_BWDD_BIG);
    if (kept)
      bwd_dual_grid<CfgBwdD, true>(s, d, w, wv, ntn, theta, U, tstride);
    else
      bwd_dual_grid<CfgBwdD, false>(s, d, w, wv, ntn, theta, U, tstride);
  } else {
    const int ntms = (w.M + CfgNNDs::BM - 1) / CfgNNDs::BM, ntns = (d.H + CfgNNDs::BN - 1) / CfgNNDs::BN;
    bwd_wave(d, w, po, e, ntms, true, wv);
    count_variant(w, kept ? V_BWDD_SMALL_KEPT : V_BWDD_SMALL);
    if (kept)
      bwd_dual_grid<CfgNNDs, true>(s, d, w, wv, ntns, theta, U, tstride);
    else
      bwd_dual_grid<CfgNNDs, false>(s, d, w, wv, ntns, theta, U, tstride);
  }
}

// ====================================================================================
// Meta-backward bookkeeping (per task z), the derivative of clip_grad_norm_ + SGD
// (train_hybrid_maml_v5.py:135-139) through inner step k:
//   w = c_k v - [c_k < 1] * max_norm * (g_k . v) / (n (n + 1e-6)^2) * g_k,   v -= lr * H_k w
__global__ void k_axpy(float* __restrict__ V, const float* __restrict__ X, int64_t n, float alpha) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    V[i] = fmaf(alpha, X[i], V[i]);
}

// The second-order sweep's per-parameter update of one inner step as ONE kernel:
//   v += alpha * x (x = H_k w_k; skipped when x is null), dot = g . v (fp64 partials over SQB
//   fixed chunks per task, summed in chunk order), grid barrier, then
//   U = c v - [c < 1] max_norm dot / (n (n + 1e-6)^2) g
// with (g, n, c) those of the inner step the sweep visits next (round 2 ran this as two launches,
// k_axpy_dot + k_so_dir, with the same partition and order). `phases` as k_inner_sgd: 3 = one launch
// with the grid barrier, 1 then 2 = the two-launch form (bitwise equal).
__global__ __launch_bounds__(NT) void k_sweep_update(float* __restrict__ V, const float* __restrict__ X, float alpha,
                                                     const float* __restrict__ G, int64_t P, int Z,
                                                     double* __restrict__ part, const float* __restrict__ norms,
                                                     const float* __restrict__ coefs, float max_norm,
                                                     float* __restrict__ Uo, GridBar gb, int phases) {
  __shared__ double red[NT / 64];
  const int nit = SQB * Z;
  const int64_t per = (P + SQB - 1) / SQB;
  for (int it = blockIdx.x; (phases & 1) && it < nit; it += gridDim.x) {
    const int z = it / SQB, b = it - z * SQB;
    float* vz = V + (int64_t)z * P;
    const float* gz = G + (int64_t)z * P;
    const int64_t beg = (int64_t)b * per, end = beg + per < P ? beg + per : P;
    double acc = 0.0;
    if (X) {
      const float* xz = X + (int64_t)z * P;
      for (int64_t i = beg + threadIdx.x; i < end; i += NT) {
        const float v = fmaf(alpha, xz[i], vz[i]);
        vz[i] = v;
        acc += (double)gz[i] * (double)v;
      }
    } else {
      for (int64_t i = beg + threadIdx.x; i < end; i += NT) acc += (double)gz[i] * (double)vz[i];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      double sum = 0.0;
      for (int i = 0; i < NT / 64; ++i) sum += red[i];
      part[it] = sum;
    }
  }
  if (phases == 3 && !grid_barrier(gb, gridDim.x)) return;
  if (!(phases & 2)) return;
  for (int it = blockIdx.x; it < nit; it += gridDim.x) {
    const int z = it / SQB, b = it - z * SQB;
    double dot = 0.0;
    for (int i = 0; i < SQB; ++i) dot += part[(int64_t)z * SQB + i];
    const float n = norms[z], c = coefs[z];
    float beta = 0.f;
    if (c < 1.f && n > 0.f) {
      const double ne = (double)n + 1e-6;
      beta = (float)((double)max_norm * dot / ((double)n * ne * ne));
    }
    const float* vz = V + (int64_t)z * P;
    const float* gz = G + (int64_t)z * P;
    float* uz = Uo + (int64_t)z * P;
    const int64_t beg = (int64_t)b * per, end = beg + per < P ? beg + per : P;
    for (int64_t i = beg + threadIdx.x; i < end; i += NT) uz[i] = c * vz[i] - beta * gz[i];
  }
}

hipError_t launch_sweep_update(hipStream_t s, float* V, const float* X, float alpha, const float* G, int64_t P, int Z,
                               double* part, const float* norms, const float* coefs, float max_norm, float* U,
                               const BarPlan& bp) {
  const int items = SQB * Z;
  const int nb = bp.fused ? grid_barrier_blocks((const void*)k_sweep_update, items, bp.oversize) : 0;
  if (nb > 0) {
    k_sweep_update<<<nb, NT, 0, s>>>(V, X, alpha, G, P, Z, part, norms, coefs, max_norm, U, bp.gb, 3);
  } else {
    const int n2 = items < 1024 ? items : 1024;
    k_sweep_update<<<n2, NT, 0, s>>>(V, X, alpha, G, P, Z, part, norms, coefs, max_norm, U, bp.gb, 1);
    k_sweep_update<<<n2, NT, 0, s>>>(V, X, alpha, G, P, Z, part, norms, coefs, max_norm, U, bp.gb, 2);
  }
  return hipGetLastError();
}

void launch_axpy(hipStream_t s, float* V, const float* X, int64_t n, float alpha) {
  int nb = (int)((n + NT - 1) / NT);
  if (nb > 4096) nb = 4096;
  k_axpy<<<nb, NT, 0, s>>>(V, X, n, alpha);
}

}  // namespace smaml
