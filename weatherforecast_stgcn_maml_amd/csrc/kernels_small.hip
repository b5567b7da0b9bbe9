// Batch-1 wavefront steps (config 4's regional adaptation, adapt_hybrid_v5.py:186-208; eval and any
// launch too small to fill the chip): the LSTM forward step (hybrid_model.py:93-102, nn.LSTM gates
// [i,f,g,o]) and the BPTT step of one anti-diagonal, each ONE launch with the K reduction split over
// the waves of a workgroup.
//
// At M = 441 sequences a diagonal holds <= 4 problems x 14 row tiles x 4 unit groups of work, and
// its time is one tile's latency chain, not throughput. The split-K pair it replaces
// (k_lstm_*_part + k_lstm_*_cell_q, kernels.hip) spreads a tile's K over S workgroups on S CUs and
// pays a second launch plus a partial-slab round trip through L2 per diagonal. Here one workgroup owns
// a 32-row tile (forward: 8 waves, BPTT: 16); each wave accumulates one contiguous K-tile range with
// its operands loaded from global memory straight into MFMA fragments (no wave shares an operand with
// another, so there is no LDS staging and no barrier in the K loop), the partial tiles meet in LDS and
// are summed in K-range order (deterministic), and the workgroup runs the cell epilogue. The
// epilogue's own operands (bias sums, c_{t-1}; gates, carry, head dh in the BPTT) are loaded before
// the K loop, so their latency hides under it. The problem of a diagonal is the grid row (blockIdx.y).
// Config 4: 1.03 -> 0.63 ms per later-epoch sample-step with these kernels and the round-4 launch trims
// (DESIGN.md section 8).
//
// Products: bf16x6 (gemm_core.h mfma_x6, f32-accurate). Forward B operand: the pre-split gate
// images (launch_split_gate) read straight into fragments, or the f32 weights split in registers.
#include "kernels.h"
#include "loaders.h"

namespace smaml {

#ifndef SMAML_KW_PROBE
#define SMAML_KW_PROBE 0  // diagnostic builds only: per-workgroup phase timestamps (tools/kw_probe.py)
#endif
#if SMAML_KW_PROBE
// wall_clock64 at 5 points (start, K-loop loads issued, K loop done, partials in LDS, epilogue issued) of
// wave 0 of every workgroup of the launch whose id (forward diagonal, or 100 + BPTT diagonal) is the target
__device__ int g_kwp_target = -1;
__device__ unsigned long long g_kwp[1024][5];
#define KWP(id, slot)                                                                    \
  if (id == g_kwp_target && threadIdx.x == 0 && blockIdx.y * gridDim.x + blockIdx.x < 1024) \
  g_kwp[blockIdx.y * gridDim.x + blockIdx.x][slot] = wall_clock64()
// out == null: arm `target` and zero the records; else copy n workgroups' records out. Returns the wall
// clock rate in kHz (> 0) or -1.
extern "C" int smaml_kw_probe(int target, unsigned long long* out, int n) {
  int khz = 0, dev = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess)
    return -1;
  if (!out) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_kwp)) != hipSuccess || hipMemset(p, 0, sizeof(g_kwp)) != hipSuccess)
      return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_kwp_target), &target, sizeof(int)) == hipSuccess ? khz : -1;
  }
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_kwp), sizeof(unsigned long long) * 5 * (n < 1024 ? n : 1024)) ==
                 hipSuccess ? khz : -1;
}
#else
#define KWP(id, slot) (void)0
#endif

constexpr int KW_W = 8;   // forward workgroup waves / K ranges (two waves per SIMD)
constexpr int KW_CH = 2;  // forward: K-tiles per wave whose loads are in flight together (56 VGPRs each)
constexpr int KW_BCH = 8; // BPTT: the same (a K-tile's fragments are 16 VGPRs)
#ifndef SMAML_KW_BWD_WAVES
#define SMAML_KW_BWD_WAVES 16  // BPTT workgroup: 8 waves (two per SIMD) or 16 (four per SIMD, half the K range
#endif                         // each; config 4: 0.717 -> 0.698 ms per sample-step)
#ifndef SMAML_KW_FWD_WAVES
#define SMAML_KW_FWD_WAVES 8  // forward workgroup waves (8: two per SIMD; 16: four per SIMD, measured slower)
#endif
#ifndef SMAML_KW_FWD_KGROUPS
#define SMAML_KW_FWD_KGROUPS 8  // forward K ranges; the waves split the 4 gates into FWD_WAVES / FWD_KGROUPS groups
#endif
constexpr int KW_FW = SMAML_KW_FWD_WAVES;
constexpr int KW_FKG = SMAML_KW_FWD_KGROUPS;
constexpr int KW_FNG = 4 * KW_FKG / KW_FW;  // gates per forward wave
constexpr int KW_FRPT = 16 / KW_FW;         // forward epilogue accumulator rows per thread
static_assert((KW_FW == 8 || KW_FW == 16) && KW_FW % KW_FKG == 0 && KW_FNG >= 1 && KW_FNG <= 4, "forward waves");
#ifndef SMAML_KW_FWD_CH
#define SMAML_KW_FWD_CH (KW_FNG == 4 ? KW_CH : 6)  // K-tiles per load round trip (registers: A 8 + B 12 per gate)
#endif
constexpr int KW_BW = SMAML_KW_BWD_WAVES;
constexpr int KW_BRPT = 16 / KW_BW;  // epilogue accumulator rows per thread
static_assert(KW_BW == 8 || KW_BW == 16, "BPTT waves");

// Accumulator register r of lane (.., hl) holds tile row (r & 3) + 8 (r >> 2) + 4 hl; the inverse:
__device__ __forceinline__ int kw_row(int r, int hl) { return (r & 3) + 8 * (r >> 2) + 4 * hl; }

// One gate fragment (8 bf16 per plane) of a pre-split gate image: image row n = g * 32 + jj, chunk h
// (k = 8h .. 8h + 7), XOR-swizzled by (n >> 3) & 1 (k_split_gate / X6Img<128, KC, 16>).
__device__ __forceinline__ void img_frag(const char* img, int n, int h, uint4& p0, uint4& p1, uint4& p2) {
  constexpr int PLANE = 128 * 32;
  const char* q = img + n * 32 + 16 * (h ^ ((n >> 3) & 1));
  p0 = *reinterpret_cast<const uint4*>(q);
  p1 = *reinterpret_cast<const uint4*>(q + PLANE);
  p2 = *reinterpret_cast<const uint4*>(q + 2 * PLANE);
}

// Operands of one forward tile's K loop (this lane's row / unit, the two K segments [x | h_{t-1}]).
struct FwdKw {
  const float* x;    // x row ar (segment 0, width cin)
  const float* hp;   // h_{t-1} row ar (segment 1, width H)
  const float* wih;  // W_ih row (g * H + j) for g = 0 (f32 weights; + g * H * cin per gate)
  const float* whh;
  const char* img0;  // gate images of (layer, W_ih), unit group ug (IMG)
  const char* img1;  // ... W_hh
  int cin, hl, jj;
};

// N K-tiles from kt0 on: every load first (no branch between them, so all are in flight together),
// then the splits and MFMAs in K order.
template <int H, bool IMG, int N, int NG>
__device__ __forceinline__ void fwd_kw_chunk(const FwdKw& o, int kt0, int g0, f32x16 (&acc)[NG]) {
  float4 a[N][2];
  uint4 bi[N][NG][3];
  float4 bf[N][NG][2];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int k = 16 * (kt0 + i);
    const bool sx = k < o.cin;
    const int kk = sx ? k : k - o.cin;
    const float* ap = (sx ? o.x : o.hp) + kk + 8 * o.hl;
    a[i][0] = ld4(ap);
    a[i][1] = ld4(ap + 4);
    if constexpr (IMG) {
      const char* img = sx ? o.img0 + (int64_t)(kk / 16) * GATE_IMG_BYTES : o.img1 + (int64_t)(kk / 16) * GATE_IMG_BYTES;
#pragma unroll
      for (int g = 0; g < NG; ++g) img_frag(img, (g0 + g) * 32 + o.jj, o.hl, bi[i][g][0], bi[i][g][1], bi[i][g][2]);
    } else {
      const int ws = sx ? o.cin : H;
      const float* wb = (sx ? o.wih : o.whh) + kk + 8 * o.hl;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const float* wr = wb + (int64_t)(g0 + g) * H * ws;
        bf[i][g][0] = ld4(wr);
        bf[i][g][1] = ld4(wr + 4);
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);  // (keeps the scheduler from interleaving the loads with the MFMAs)
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const Split3 as = split3(a[i][0], a[i][1]);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      Split3 b;
      if constexpr (IMG) {
        b.p0 = __builtin_bit_cast(bf16x8_t, bi[i][g][0]);
        b.p1 = __builtin_bit_cast(bf16x8_t, bi[i][g][1]);
        b.p2 = __builtin_bit_cast(bf16x8_t, bi[i][g][2]);
      } else {
        b = split3(bf[i][g][0], bf[i][g][1]);
      }
      acc[g] = mfma_x6(as, b, acc[g]);
    }
  }
}

// Contiguous K-tile range [kb, ke) of K range `wave` out of NW (deterministic partition).
template <int NW = KW_W>
__device__ __forceinline__ void kw_range(int nkt, int wave, int& kb, int& ke) {
  const int per = (nkt + NW - 1) / NW;
  kb = min(nkt, wave * per);
  ke = min(nkt, kb + per);
}

// ---- forward: tile = 32 rows x 32 units (the 4 gates: 128 gate columns) ------------------------
template <int H, bool IMG>
__global__ __launch_bounds__(64 * KW_FW) void k_lstm_fwd_kw(const float* __restrict__ F, float* __restrict__ HsAll,
                                                          float* __restrict__ CsAll, float* __restrict__ GsAll,
                                                          int64_t lsz, const float* __restrict__ theta,
                                                          int64_t tstride, FwdWave wv, int T, int M, GateImgs gi,
                                                          const float* __restrict__ XG, int pid) {
  static_assert(H % 32 == 0, "32-unit groups");
  KWP(pid, 0);
  __shared__ float red[KW_FKG * 64 * 64];  // [K range][gate*16 + r][lane]
  // problem = blockIdx.y (not found from blockIdx.x by compares: its fields' kernel-argument loads then
  // depend on nothing loaded and issue with the first batch)
  const int pb = blockIdx.y;
  const int l = wave_sel(wv.l, pb), t = wave_sel(wv.t, pb);
  const LayerOff lo = wave_sel(wv.lo, pb);
  const int ntm = (M + 31) / 32;
  const int bl = (int)blockIdx.x;
  const int tm = bl % ntm, ug = bl / ntm;  // row tiles fastest (all XCDs see every unit group)
  const int z = blockIdx.z;
  const float* th = theta + (int64_t)z * tstride;
  const int cin = lo.cin;
  const int64_t slab = (int64_t)z * T * M;
  const float* X = (l == 0 ? F : HsAll + (int64_t)(l - 1) * lsz) + (slab + (int64_t)t * M) * cin;
  float* Hz = HsAll + (int64_t)l * lsz + slab * H;
  float* Cz = CsAll + (int64_t)l * lsz + slab * H;
  float* Gz = GsAll + (int64_t)l * lsz * 4 + slab * (4 * H);
  const float* Hp = Hz + (int64_t)(t > 0 ? t - 1 : 0) * M * H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hl = lane >> 5, jj = lane & 31;
  const int kg = wave % KW_FKG, g0 = (wave / KW_FKG) * KW_FNG;  // this wave's K range and first gate
  const int m0 = tm * 32, j = ug * 32 + jj;

  // layer 0 with the input projection hoisted (XG = F . W_ih0^T for all steps, run_lstm): its K loop
  // covers only the recurrent segment and the epilogue adds XG
  const bool hx = XG != nullptr && l == 0;
  // epilogue operands: this thread's elements are rows kw_row(KW_FRPT wave + q, hl), unit j
  float bs[4], cp[KW_FRPT], xg[KW_FRPT][4];
#pragma unroll
  for (int g = 0; g < 4; ++g) bs[g] = th[lo.bih + g * H + j] + th[lo.bhh + g * H + j];
#pragma unroll
  for (int q = 0; q < KW_FRPT; ++q) {
    const int m = min(m0 + kw_row(KW_FRPT * wave + q, hl), M - 1);
    const float* xr = (hx ? XG + (slab + (int64_t)t * M + m) * (4 * H) : th) + j;  // (not hx: a valid address)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float v = xr[g * H];
      xg[q][g] = hx ? v : 0.f;
    }
    const float v = Cz[((int64_t)(t > 0 ? t - 1 : 0) * M + m) * H + j];  // (t = 0: a valid address, selected out)
    cp[q] = t > 0 ? v : 0.f;
  }

  f32x16 acc[KW_FNG];
#pragma unroll
  for (int g = 0; g < KW_FNG; ++g)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[g][r] = 0.f;
  {
    const int ar = min(m0 + jj, M - 1);  // this lane's A row (clamped: rows past M are not stored)
    FwdKw o;
    o.x = X + (int64_t)ar * cin;
    o.hp = Hp + (int64_t)ar * H;
    o.wih = th + lo.wih + (int64_t)j * cin;
    o.whh = th + lo.whh + (int64_t)j * H;
    o.img0 = o.img1 = nullptr;
    if constexpr (IMG) {
      int64_t io0 = 0, io1 = 0;
#pragma unroll
      for (int q = 0; q < MAX_LAYERS; ++q)
        if (q == l) {
          io0 = gi.off[q][0];
          io1 = gi.off[q][1];
        }
      const char* ib = gi.th + (int64_t)z * gi.tstride;
      o.img0 = ib + io0 + (int64_t)ug * (cin / 16) * GATE_IMG_BYTES;
      o.img1 = ib + io1 + (int64_t)ug * (H / 16) * GATE_IMG_BYTES;
    }
    o.cin = cin;
    o.hl = hl;
    o.jj = jj;
    int kb, ke;
    kw_range<KW_FKG>(((hx ? 0 : cin) + (t > 0 ? H : 0)) / 16, kg, kb, ke);
    if (hx) {  // (K-tile indices past the input segment: the recurrent one)
      kb += cin / 16;
      ke += cin / 16;
    }
    KWP(pid, 1);
    // (uniform branches between straight-line chunks; measured: the layer-0 problem's third K-tile per
    // wave in the same round trip, its B image copied to LDS with direct-to-LDS loads, 0.712 -> 0.749 ms
    // per config-4 sample-step: the compiler waits for the copies before the register tiles' MFMAs)
    constexpr int CH = SMAML_KW_FWD_CH;
    while (ke - kb >= CH) {
      fwd_kw_chunk<H, IMG, CH, KW_FNG>(o, kb, g0, acc);
      kb += CH;
    }
    for (; kb < ke; ++kb) fwd_kw_chunk<H, IMG, 1, KW_FNG>(o, kb, g0, acc);
  }

  // partial tiles -> LDS (lane-contiguous: conflict-free), summed in wave order
  KWP(pid, 2);
#pragma unroll
  for (int g = 0; g < KW_FNG; ++g)
#pragma unroll
    for (int r = 0; r < 16; ++r) red[(kg * 64 + (g0 + g) * 16 + r) * 64 + lane] = acc[g][r];
  __syncthreads();
  KWP(pid, 3);
  const uint32_t tM = (uint32_t)t * (uint32_t)M;
#pragma unroll
  for (int q = 0; q < KW_FRPT; ++q) {
    const int r = KW_FRPT * wave + q;
    float pre[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < KW_FKG; ++w) s += red[(w * 64 + g * 16 + r) * 64 + lane];
      pre[g] = s + bs[g] + xg[q][g];
    }
    const int m = m0 + kw_row(r, hl);
    if (m >= M) continue;
    const float gi_ = sigmoidf_(pre[0]), gf = sigmoidf_(pre[1]), gg = tanhf_(pre[2]), go = sigmoidf_(pre[3]);
    const float c = lstm_cell_c(gi_, gf, gg, cp[q]);
    const float h = go * tanhf_(c);
    const uint32_t row = tM + (uint32_t)m;
    const uint32_t og = row * (4 * H) + j, oh = row * H + j;
    stb(Gz, 4u * og, gi_);
    stb(Gz, 4u * (og + H), gf);
    stb(Gz, 4u * (og + 2 * H), gg);
    stb(Gz, 4u * (og + 3 * H), go);
    stb(Cz, 4u * oh, c);
    stb(Hz, 4u * oh, h);
  }
  KWP(pid, 4);
}

// Operands of one BPTT tile's K loop: this lane's rows of the two dG segments and weight columns.
struct BwdKw {
  const float* a0;  // segment 0 (dG above, or dG next when there is no layer above): row ar, k = 8 hl
  const float* a1;  // segment 1 (dG next)
  const float* w0;  // W (k = 8 hl, unit j) of segment 0: W_ih(l+1) or W_hh(l), [4H][H]
  const float* w1;  // ... segment 1: W_hh(l)
  const char* i0;   // (IMG) segment 0's image at K-tile 0, unit tile tn, this lane's 16-B chunk
  const char* i1;   // ... segment 1
};

template <int H, bool IMG, int N>
__device__ __forceinline__ void bwd_kw_chunk(const BwdKw& o, int kt0, f32x16& acc) {
  constexpr int G4 = 4 * H;
  constexpr int KT_BYTES = (H / 32) * BWD_IMG_BYTES;  // one K-tile of an image, all unit tiles
  float4 a[N][2];
  float b[N][8];
  uint4 bi[N][3];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int k = 16 * (kt0 + i);
    const bool s1 = k >= G4;
    const int kk = s1 ? k - G4 : k;
    const float* ap = (s1 ? o.a1 : o.a0) + kk;
    a[i][0] = ld4(ap);
    a[i][1] = ld4(ap + 4);
    if constexpr (IMG) {
      const char* q = (s1 ? o.i1 : o.i0) + (kk / 16) * KT_BYTES;
      bi[i][0] = *reinterpret_cast<const uint4*>(q);
      bi[i][1] = *reinterpret_cast<const uint4*>(q + 1024);
      bi[i][2] = *reinterpret_cast<const uint4*>(q + 2048);
    } else {
      const float* wp = (s1 ? o.w1 : o.w0) + (int64_t)kk * H;
#pragma unroll
      for (int e = 0; e < 8; ++e) b[i][e] = wp[e * H];
    }
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const Split3 as = split3(a[i][0], a[i][1]);
    Split3 bs;
    if constexpr (IMG) {
      bs.p0 = __builtin_bit_cast(bf16x8_t, bi[i][0]);
      bs.p1 = __builtin_bit_cast(bf16x8_t, bi[i][1]);
      bs.p2 = __builtin_bit_cast(bf16x8_t, bi[i][2]);
    } else {
      bs = split3(make_float4(b[i][0], b[i][1], b[i][2], b[i][3]), make_float4(b[i][4], b[i][5], b[i][6], b[i][7]));
    }
    acc = mfma_x6(as, bs, acc);
  }
}

// ---- BPTT: tile = 32 rows x 32 units of dh = [dG(l+1,t) | dG(l,t+1)] . [W_ih(l+1) ; W_hh(l)] -----
template <int H, bool IMG>
__global__ __launch_bounds__(64 * KW_BW) void k_lstm_bwd_kw(const float* GsAll, float* dGAll, float* __restrict__ dhAll,
                                                          const float* __restrict__ CsAll,
                                                          const float* __restrict__ dHhead, float* __restrict__ dcAll,
                                                          int64_t lsz, const float* __restrict__ theta,
                                                          int64_t tstride, BwdWave wv, int L, int T, int M,
                                                          BwdImgs bim, int pid) {
  static_assert(H % 32 == 0, "32-unit tiles");
  KWP(pid, 0);
  constexpr int G4 = 4 * H;
  __shared__ float red[KW_BW * 16 * 64];  // [wave][r][lane]
  const int p = blockIdx.y;  // (problem per grid row, as in k_lstm_fwd_kw)
  const int l = wave_sel(wv.l, p), t = wave_sel(wv.t, p);
  const LayerOff lo = wave_sel(wv.lo, p);
  const int64_t wih_up = wave_sel(wv.wih_up, p);
  const int ntm = (M + 31) / 32;
  const int bl = (int)blockIdx.x;
  const int tm = bl % ntm, tn = bl / ntm;
  const int z = blockIdx.z;
  const int64_t slab = (int64_t)z * T * M;
  const float* th = theta + (int64_t)z * tstride;
  const float* Gz = GsAll + (int64_t)l * lsz * 4 + slab * G4;
  float* dGz = dGAll + (int64_t)l * lsz * 4 + slab * G4;
  float* dhz = dhAll ? dhAll + (int64_t)l * lsz + slab * H : nullptr;
  const float* Cz = CsAll + (int64_t)l * lsz + slab * H;
  float* dcz = dcAll + ((int64_t)l * gridDim.z + z) * M * H;
  const float* dHz = dHhead + (int64_t)z * M * H;
  const bool up = l + 1 < L, nx = t + 1 < T, first = t == T - 1, past = t > 0, head = first && l == L - 1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hl = lane >> 5, jj = lane & 31;
  const int m0 = tm * 32, j = tn * 32 + jj;

  // epilogue operands of this thread's elements (rows kw_row(KW_BRPT wave + q, hl), unit j), loaded
  // first; uniform conditions select after loads from valid addresses (no branch around a load)
  float g[KW_BRPT][4], cp[KW_BRPT], dc[KW_BRPT], hd[KW_BRPT];
#pragma unroll
  for (int q = 0; q < KW_BRPT; ++q) {
    const int m = min(m0 + kw_row(KW_BRPT * wave + q, hl), M - 1);
    const int64_t row = (int64_t)t * M + m;
#pragma unroll
    for (int k = 0; k < 4; ++k) g[q][k] = Gz[row * G4 + k * H + j];
    const float c = Cz[(past ? row - M : row) * H + j];
    const float d = dcz[(int64_t)m * H + j];
    const float h = dHz[(int64_t)m * H + j];
    cp[q] = past ? c : 0.f;
    dc[q] = first ? 0.f : d;
    hd[q] = head ? h : 0.f;
  }

  // segments [above | next] compacted (as k_lstm_bwd_step): K = ns * 4H
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  {
    const float* pa = dGAll + (int64_t)(l + 1) * lsz * 4 + (slab + (int64_t)t * M) * G4;
    const float* pn = dGz + (int64_t)(t + 1) * M * G4;
    const int ar = min(m0 + jj, M - 1);
    BwdKw o;
    o.a0 = (up ? pa : pn) + (int64_t)ar * G4 + 8 * hl;
    o.a1 = pn + (int64_t)ar * G4 + 8 * hl;
    o.w0 = (up ? th + wih_up : th + lo.whh) + (int64_t)(8 * hl) * H + j;
    o.w1 = th + lo.whh + (int64_t)(8 * hl) * H + j;
    o.i0 = o.i1 = nullptr;
    if constexpr (IMG) {
      int64_t ohh = 0, oih = 0;  // (layer l's W_hh and layer l+1's W_ih, selected with scalar compares)
#pragma unroll
      for (int q = 0; q < MAX_LAYERS; ++q) {
        if (q == l) ohh = bim.off_hh[q];
        if (q == l + 1) oih = bim.off_ih[q];
      }
      const char* ib = bim.th + (int64_t)z * bim.tstride + tn * BWD_IMG_BYTES + jj * 32 + hl * 16;
      o.i0 = ib + (up ? oih : ohh);
      o.i1 = ib + ohh;
    }
    int kb, ke;
    kw_range<KW_BW>(((up ? 1 : 0) + (nx ? 1 : 0)) * (G4 / 16), wave, kb, ke);
    KWP(pid, 1);
    while (ke - kb >= KW_BCH) {
      bwd_kw_chunk<H, IMG, KW_BCH>(o, kb, acc);
      kb += KW_BCH;
    }
    if (ke - kb >= 4) {
      bwd_kw_chunk<H, IMG, 4>(o, kb, acc);
      kb += 4;
    }
    for (; kb < ke; ++kb) bwd_kw_chunk<H, IMG, 1>(o, kb, acc);
  }

  KWP(pid, 2);
#pragma unroll
  for (int r = 0; r < 16; ++r) red[(wave * 16 + r) * 64 + lane] = acc[r];
  __syncthreads();
  KWP(pid, 3);
#pragma unroll
  for (int q = 0; q < KW_BRPT; ++q) {
    const int r = KW_BRPT * wave + q;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < KW_BW; ++w) s += red[(w * 16 + r) * 64 + lane];
    const int m = m0 + kw_row(r, hl);
    if (m >= M) continue;
    const float d = s + hd[q];
    const float gi = g[q][0], gf = g[q][1], gg = g[q][2], go = g[q][3];
    const float tc = tanhf_(lstm_cell_c(gi, gf, gg, cp[q]));
    const float dct = dc[q] + d * go * (1.f - tc * tc);
    const int64_t row = (int64_t)t * M + m;
    float* gp = dGz + row * G4 + j;
    gp[0] = dct * gg * gi * (1.f - gi);
    gp[H] = dct * cp[q] * gf * (1.f - gf);
    gp[2 * H] = dct * gi * (1.f - gg * gg);
    gp[3 * H] = d * tc * go * (1.f - go);
    dcz[(int64_t)m * H + j] = dct * gf;
    if (dhz) dhz[row * H + j] = d;
  }
  KWP(pid, 4);
}

bool small_kw_ok(const Dims& d, const Work& w) {
  if (!w.kn.small_kw || w.drop.lstm() || d.H % 32 != 0 || d.H > 256 || d.Hc % 16 != 0) return false;
  return true;
}

void launch_lstm_fwd_kw(hipStream_t s, const Dims& d, const Work& w, int diag, const float* theta, int64_t tstride,
                        const ParamOff& po) {
  const int64_t lsz = (int64_t)w.Z * d.T * w.M * d.H;
  FwdWave wv{};
  fwd_wave(d, w, po, diag, ((w.M + 31) / 32) * (d.H / 32), false, wv);
  if (wv.n == 0) return;
  const dim3 grid(((w.M + 31) / 32) * (d.H / 32), wv.n, w.Z);
  count_variant(w, V_FWD_KW);
  const float* xg = w.xg && w.xg_src == theta ? w.xg : nullptr;
  if (w.gimg.th && w.gimg_src == theta) {
    SMAML_DISPATCH_H(d.H, (k_lstm_fwd_kw<HT, true><<<grid, 64 * KW_FW, 0, s>>>(w.F, w.Hs, w.Cs, w.Gs, lsz, theta,
                                                                               tstride, wv, d.T, w.M, w.gimg, xg, diag)));
  } else {
    SMAML_DISPATCH_H(d.H, (k_lstm_fwd_kw<HT, false><<<grid, 64 * KW_FW, 0, s>>>(w.F, w.Hs, w.Cs, w.Gs, lsz, theta,
                                                                                tstride, wv, d.T, w.M, w.gimg, xg, diag)));
  }
}

void launch_lstm_bwd_kw(hipStream_t s, const Dims& d, const Work& w, int e, const float* theta, int64_t tstride,
                        const ParamOff& po) {
  const int64_t lsz = (int64_t)w.Z * d.T * w.M * d.H;
  BwdWave wv{};
  bwd_wave(d, w, po, e, ((w.M + 31) / 32) * (d.H / 32), false, wv);
  if (wv.n == 0) return;
  const dim3 grid(((w.M + 31) / 32) * (d.H / 32), wv.n, w.Z);
  count_variant(w, V_BWD_KW);
  if (w.bimg.th && w.bimg_src == theta) {
    SMAML_DISPATCH_H(d.H, (k_lstm_bwd_kw<HT, true><<<grid, 64 * KW_BW, 0, s>>>(
                              w.Gs, w.dG, w.dh, w.Cs, w.dH, w.dc, lsz, theta, tstride, wv, d.L, d.T, w.M, w.bimg, 100 + e)));
  } else {
    SMAML_DISPATCH_H(d.H, (k_lstm_bwd_kw<HT, false><<<grid, 64 * KW_BW, 0, s>>>(
                              w.Gs, w.dG, w.dh, w.Cs, w.dH, w.dc, lsz, theta, tstride, wv, d.L, d.T, w.M, w.bimg, 100 + e)));
  }
}

// ---- pre-split BPTT weight images (kernels.h BwdImgs) ----------------------------------------
int64_t bwd_img_bytes(const Dims& d, BwdImgs* bi) {
  const int64_t per = (int64_t)(4 * d.H / 16) * (d.H / 32) * BWD_IMG_BYTES;  // one [4H][H] matrix
  int64_t off = 0;
  for (int l = 0; l < d.L; ++l) {
    if (bi) bi->off_hh[l] = off;
    off += per;
    if (bi) bi->off_ih[l] = l > 0 ? off : 0;
    if (l > 0) off += per;
  }
  if (bi) bi->tstride = off;
  return off;
}

// One thread per (task, matrix, K-tile kt, unit tile tn, unit jj, half h): W[16 kt + 8 h + e][32 tn + jj],
// e = 0..7, split into three bf16 pieces, one 16-B chunk per plane.
__global__ void k_split_bwd(const float* __restrict__ theta, int64_t tstride, ParamOff po, int L, int H,
                            BwdImgs bi, int64_t nthreads) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int z = blockIdx.y;
  if (i >= nthreads) return;
  const int h = (int)(i & 1), jj = (int)((i >> 1) & 31);
  const int ntn = H / 32, nkt = 4 * H / 16;
  int64_t r = i >> 6;
  const int tn = (int)(r % ntn);
  r /= ntn;
  const int kt = (int)(r % nkt);
  const int mat = (int)(r / nkt);  // bwd_img_bytes order: W_hh(0), W_hh(1), W_ih(1), W_hh(2), W_ih(2), ...
  const int l = (mat + 1) / 2;
  const bool ih = mat > 0 && mat % 2 == 0;
  if (l >= L) return;
  const LayerOff& lo = po.lay[l];
  const float* src = theta + (int64_t)z * tstride + (ih ? lo.wih : lo.whh) + (int64_t)(16 * kt + 8 * h) * H + 32 * tn + jj;
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = src[(int64_t)e * H];
  const Split3 p = split3(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]));
  int64_t moff = 0;
#pragma unroll
  for (int q = 0; q < MAX_LAYERS; ++q)
    if (q == l) moff = ih ? bi.off_ih[q] : bi.off_hh[q];
  char* o = bi.th + (int64_t)z * bi.tstride + moff + ((int64_t)kt * ntn + tn) * BWD_IMG_BYTES + jj * 32 + h * 16;
  *reinterpret_cast<uint4*>(o) = __builtin_bit_cast(uint4, p.p0);
  *reinterpret_cast<uint4*>(o + 1024) = __builtin_bit_cast(uint4, p.p1);
  *reinterpret_cast<uint4*>(o + 2048) = __builtin_bit_cast(uint4, p.p2);
}

void launch_split_bwd(hipStream_t s, const Dims& d, const ParamOff& po, const float* theta, int64_t tstride, int Z,
                      const BwdImgs& bi) {
  const int nmat = 2 * d.L - 1;
  const int64_t threads = (int64_t)nmat * (4 * d.H / 16) * (d.H / 32) * 64;
  k_split_bwd<<<dim3((unsigned)((threads + 255) / 256), Z), 256, 0, s>>>(theta, tstride, po, d.L, d.H, bi, threads);
}

}  // namespace smaml
