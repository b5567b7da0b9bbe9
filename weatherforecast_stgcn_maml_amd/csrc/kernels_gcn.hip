// Fused GCN stack for the rows without neighbours (F3): GCNConv x4 + ReLU on the rows t >= 1 of
// every sample, where each conv is x W^T + b (hybrid_model.py:60-78 with model.py:23-26: only the
// first N rows of a T*N-row sample are covered by edge_index, every other row sees only its
// self loop, whose gcn_norm weight is 1). 23 of 24 rows take this path; the t = 0 rows keep the
// per-layer k_gcn_layer (ELL gather).
//
// Register-resident layout. One wave owns 32 data rows and ALL HC output channels of them, and
// computes out^T = W . act^T with v_mfma_f32_32x32x16_bf16 in the bf16x6 product form
// (gemm_core.h mfma_x6): the A operand is W (32 channels x 16 k per fragment) read from an LDS ring
// the workgroup's waves fill with direct-to-LDS loads of PRE-SPLIT bf16 pieces (k_gcn_wsplit, no
// VALU, no staging VGPRs); the B operand is the wave's own activations, kept as f32 in VGPRs
// between layers and split into pieces one 16-k step at a time. The accumulator of tile ci holds,
// in lane (row n = lane & 31, h = lane >> 5), register r, the channel
//   p = 32 ci + (r & 3) + 8 (r >> 2) + 4 h;
// the next layer's B fragment for k-step s = 2 ci + u needs, in lane (n, h), 8 consecutive k-values
// 16 s + 8 h + j, which are exactly registers r = 8 u + j of tile ci if the next layer's K order is
// the channel order with bits 2 and 3 swapped inside each 32-block (kappa <-> p, see kperm). The
// pre-split images of W2..W4 are stored with their columns in that order, so a layer's outputs feed
// the next layer without any cross-lane exchange or LDS round trip. Activations between the four
// layers never touch HBM: per row the kernel reads Cin0 floats and writes HC floats (the LSTM
// input F, in the time-major layout [Z][T][B*N][HC] of k_gcn_layer's remap).
//
// Consecutive windows (dedup): a row t >= 1 sees only its own input row (F3), so its features are a
// function of the stream row alone, and window b's step t is window b + 1's step t - 1. When a task's B
// windows start at consecutive stream rows (the support batches and the query batch of the reference's
// window table), the kernel computes each distinct stream row tau' = b + t in [1, B + T - 2] once --
// (B + T - 2) N rows per task instead of B (T - 1) N, 55 instead of 736 time steps at B = 32 -- and
// stores the result to every (b, t >= 1) with b + t = tau'. Same per-row arithmetic, so F is bitwise
// the per-sample result.
#include "kernels.h"
#include "loaders.h"

namespace smaml {

// Input-channel index of K position kappa (layers 2..4): bits 2 and 3 swapped inside each 32-block.
__host__ __device__ __forceinline__ int kperm(int kappa) {
  return (kappa & ~12) | ((kappa & 4) << 1) | ((kappa & 8) >> 1);
}

constexpr int GM_WAVES = 4;                        // waves (= 32-row groups) per workgroup
constexpr int GM_ROWS = 32 * GM_WAVES;             // data rows per workgroup
constexpr int GM_NSTG = 4;                         // W-image ring stages
constexpr int GM_KS1 = 2;                          // 16-k steps of layer 1 (Cin0 <= 32, zero-padded to 32)
__host__ __device__ constexpr int gm_step_bytes(int HC) { return 3 * HC * 32; }  // one 16-k step, 3 planes

// W image of one 16-k step: [plane][HC rows][16 k] bf16, 16-B chunks XOR-swizzled by row
// (X6Img<HC, true, 16>), so a lane's 8-element fragment is one conflict-free ds_read_b128.
__device__ __forceinline__ int gm_img_off(int row, int k) {
  return row * 32 + 16 * ((k >> 3) ^ ((row >> 3) & 1)) + 2 * (k & 7);
}

// Pre-split images of W1..W4, steps in layer order: layer 1 (natural K order, always GM_KS1 steps,
// zero-padded past Cin0: k_gcn_mlp walks two layer-1 steps whatever Cin0 <= 32 is), layers 2..4 (K
// order kperm). One thread per (step, row, 4 k).
__global__ void k_gcn_wsplit(const float* __restrict__ gcn, GcnWOff wo, int HC, int cin0, char* __restrict__ img) {
  constexpr int ks1 = GM_KS1;
  const int nsteps = ks1 + 3 * (HC / 16);
  const int64_t total = (int64_t)nsteps * HC * 4;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int q = (int)(i & 3), row = (int)((i >> 2) % HC), step = (int)(i / (4 * HC));
  int layer, ks;
  if (step < ks1) {
    layer = 0;
    ks = step;
  } else {
    layer = 1 + (step - ks1) / (HC / 16);
    ks = (step - ks1) % (HC / 16);
  }
  const int cin = layer == 0 ? cin0 : HC;
  const float* W = gcn + wo.w[layer];
  float v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int kap = 16 * ks + 4 * q + e;
    const int c = layer == 0 ? kap : kperm(kap);
    v[e] = c < cin ? W[(int64_t)row * cin + c] : 0.f;
  }
  uint2 p0, p1, p2;
  split4(make_float4(v[0], v[1], v[2], v[3]), p0, p1, p2);
  char* base = img + (int64_t)step * gm_step_bytes(HC) + gm_img_off(row, 4 * q);
  *reinterpret_cast<uint2*>(base) = p0;
  *reinterpret_cast<uint2*>(base + HC * 32) = p1;
  *reinterpret_cast<uint2*>(base + 2 * HC * 32) = p2;
}

typedef __attribute__((address_space(3))) void gm_lds_t;
typedef __attribute__((address_space(1))) const void gm_gbl_t;

template <int HC>
__global__ __launch_bounds__(64 * GM_WAVES) void k_gcn_mlp(GcnMlpArgs a) {
  constexpr int NT = HC / 32;  // channel tiles
  constexpr int SB = gm_step_bytes(HC);
  constexpr int CHUNKS = SB / 1024;  // 1-KB direct-to-LDS wave-instructions per step
  static_assert(SB % 1024 == 0 && CHUNKS % GM_WAVES == 0, "whole chunks per wave");
  constexpr int CPW = CHUNKS / GM_WAVES;
  constexpr int KS = HC / 16;  // steps of layers 2..4
  constexpr int NSTEPS = GM_KS1 + 3 * KS;
  __shared__ __attribute__((aligned(16))) char ring[GM_NSTG * SB];
  __shared__ __attribute__((aligned(16))) float bias_s[4][HC];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;

  // this lane's data row (t >= 1 rows of sample g: q in [N, T*N)); dedup: g is the task and
  // t = q / N the stream row tau' relative to its first window, in [1, B + T - 2]
  const int64_t r1 = (int64_t)blockIdx.x * GM_ROWS + wave * 32 + (lane & 31);
  const bool valid = r1 < a.R1;
  const uint32_t rr = valid ? (uint32_t)r1 : 0u;
  const int g = (int)a.rows_div.div(rr);
  const int q = a.N + (int)(rr - (uint32_t)g * (uint32_t)a.rows1);
  const int z = a.dedup ? g : (int)a.b_div.div((uint32_t)g), s = a.dedup ? 0 : g - z * a.B;
  const int t = (int)a.n_div.div((uint32_t)q), n = q - t * a.N;
  const float* xrow = a.xtab[a.dedup ? g * a.B : g] + (int64_t)q * a.cin0;
  // destinations: (sample boff - tt, step tt) for tt in [t_lo, t_hi]
  const int t_lo = a.dedup ? max(1, t - (a.B - 1)) : t, t_hi = a.dedup ? min(a.T - 1, t) : t;
  const int boff = s + t;
  float* frow = a.F + (((int64_t)z * a.T) * a.M + n) * HC;
  if (a.compact) {  // once, at compact row M + (t - 1) N + n (t = the stream row here): tt = t_lo only
    frow = a.F + (((int64_t)z * a.T) * a.M + a.M + (int64_t)(t - 1) * a.N + n) * HC;
  }
  uint64_t didx = 0;
  if (a.dr.gcn()) didx = (((uint64_t)a.dr.task_id[z] * a.B + s) * (uint64_t)(a.T * a.N) + (uint64_t)q) * HC;

  // layer-1 operand (k = 8 h .. 8 h + 7 and 16 + 8 h .. 16 + 8 h + 7 of the row) before any ring load,
  // so the counted waits below see only the ring's loads
  float4 x4[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int k = 16 * (e >> 1) + 8 * h + 4 * (e & 1);
    x4[e] = (valid && k < a.cin0) ? ld4(xrow + k) : f4zero();
  }
  for (int i = threadIdx.x; i < 4 * HC; i += 64 * GM_WAVES) bias_s[i / HC][i % HC] = a.gcn[a.wo.b[i / HC] + i % HC];

  // W ring: step j lands in stage j % NSTG; every wave issues CPW 1-KB chunks of it
  auto issue = [&](int j) {
    const char* src = a.wimg + (int64_t)j * SB;
    char* dst = ring + (j % GM_NSTG) * SB;
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
      const int ch = wave + GM_WAVES * c;
      __builtin_amdgcn_global_load_lds((gm_gbl_t*)(src + ch * 1024 + 16 * lane), (gm_lds_t*)(dst + ch * 1024), 16,
                                       0, 0);
    }
  };
#pragma unroll
  for (int j = 0; j < GM_NSTG - 1; ++j) issue(j);

  f32x16 acc[NT];
#pragma unroll
  for (int ci = 0; ci < NT; ++ci)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[ci][r] = 0.f;

  // one 16-k step: wait for its W image, refill the ring, the MFMAs of every channel tile against the
  // split B fragment b; the NEXT step's B fragment (nlo, nhi: registers only) is split in the same
  // block so its VALU can issue between the MFMAs
  auto step = [&](int j, Split3& b, const float4& nlo, const float4& nhi) {
    if (j + GM_NSTG - 2 < NSTEPS)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((GM_NSTG - 2) * CPW) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // step j landed for every wave; every wave is done reading stage (j - 1) % NSTG
    if (j + GM_NSTG - 1 < NSTEPS) issue(j + GM_NSTG - 1);
    const char* st = ring + (j % GM_NSTG) * SB;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ci = 0; ci < NT; ++ci) {
      const int off = gm_img_off(32 * ci + (lane & 31), 8 * h);
      Split3 af;
      af.p0 = *reinterpret_cast<const bf16x8_t*>(st + off);
      af.p1 = *reinterpret_cast<const bf16x8_t*>(st + HC * 32 + off);
      af.p2 = *reinterpret_cast<const bf16x8_t*>(st + 2 * HC * 32 + off);
      acc[ci] = mfma_x6(af, b, acc[ci]);
    }
    b = split3(nlo, nhi);
    __builtin_amdgcn_s_setprio(0);
  };
  // + bias, ReLU (every conv), dropout (conv1..conv3) -> act (the next layer's B operand), acc = 0
  float act[NT][16];
  auto epilogue = [&](int layer) {
    const bool drop = a.dr.gcn() && layer < 3;
    const uint32_t dsite = drop ? drop_site(a.dr.seed, 1, a.dr.step, layer) : 0u;
#pragma unroll
    for (int ci = 0; ci < NT; ++ci)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int p0 = 32 * ci + 8 * gq + 4 * h;
        const float4 bb = *reinterpret_cast<const float4*>(&bias_s[layer][p0]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = fmaxf(acc[ci][4 * gq + e] + f4get(bb, e), 0.f);
          if (drop) x = drop_keep(dsite, didx + p0 + e, a.dr.thr_gcn) ? x * a.dr.sc_gcn : 0.f;
          act[ci][4 * gq + e] = x;
          acc[ci][4 * gq + e] = 0.f;
        }
      }
  };

  Split3 b = split3(x4[0], x4[1]);
  step(0, b, x4[2], x4[3]);
  step(1, b, x4[2], x4[3]);  // (the split after the last step of a layer is unused)
  epilogue(0);
  auto lo4 = [&](int ks) {
    const int ci = ks >> 1, u = 8 * (ks & 1);
    return make_float4(act[ci][u], act[ci][u + 1], act[ci][u + 2], act[ci][u + 3]);
  };
  auto hi4 = [&](int ks) {
    const int ci = ks >> 1, u = 8 * (ks & 1) + 4;
    return make_float4(act[ci][u], act[ci][u + 1], act[ci][u + 2], act[ci][u + 3]);
  };
  for (int layer = 1; layer < 4; ++layer) {
    const int j0 = GM_KS1 + (layer - 1) * KS;
    b = split3(lo4(0), hi4(0));
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) step(j0 + ks, b, lo4(ks + 1 < KS ? ks + 1 : ks), hi4(ks + 1 < KS ? ks + 1 : ks));
    epilogue(layer);
  }
  if (valid) {
    for (int tt = t_lo; tt <= (a.compact ? t_lo : t_hi); ++tt) {
      float* fr = a.compact ? frow : frow + ((int64_t)tt * a.M + (int64_t)(boff - tt) * a.N) * HC;
#pragma unroll
      for (int ci = 0; ci < NT; ++ci)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq)
          st4(fr + 32 * ci + 8 * gq + 4 * h,
              make_float4(act[ci][4 * gq], act[ci][4 * gq + 1], act[ci][4 * gq + 2], act[ci][4 * gq + 3]));
    }
  }
}

void launch_gcn_wsplit(hipStream_t s, const Dims& d, const float* gcn, const GcnWOff& wo, char* img) {
  const int64_t total = (int64_t)(GM_KS1 + 3 * (d.Hc / 16)) * d.Hc * 4;
  k_gcn_wsplit<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(gcn, wo, d.Hc, d.Cin0, img);
}

int64_t gcn_wimg_bytes(const Dims& d) {
  return (int64_t)(GM_KS1 + 3 * (d.Hc / 16)) * gm_step_bytes(d.Hc);
}

// Consecutive windows on the per-layer path: C [Z][B + T - 1][N][Hc] holds each task's stream rows
// w0 .. w0 + B + T - 2 (rows without neighbours); F[z][t][b N + n] = C[z][b + t][n] for t >= 1 -- one
// workgroup per (task, t, window) N x Hc block, float4 copies.
__global__ void k_gcn_expand(const float* __restrict__ C, float* __restrict__ F, int B, int T, int64_t blk) {
  const int b = blockIdx.y % B, t = 1 + (int)(blockIdx.y / B) % (T - 1), z = blockIdx.y / (B * (T - 1));
  const float4* src = reinterpret_cast<const float4*>(C + ((int64_t)z * (B + T - 1) + b + t) * blk);
  float4* dst = reinterpret_cast<float4*>(F + (((int64_t)z * T + t) * B + b) * blk);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < blk / 4; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

// compact: per task the distinct rows s >= 1 only, one contiguous block: F[z][M + (s - 1) N ..] = C[z][s N ..]
__global__ void k_gcn_compact(const float* __restrict__ C, float* __restrict__ F, int B, int T, int64_t blk) {
  const int z = blockIdx.y;
  const int64_t n4 = (int64_t)(B + T - 2) * blk / 4;
  const float4* src = reinterpret_cast<const float4*>(C + ((int64_t)z * (B + T - 1) + 1) * blk);
  float4* dst = reinterpret_cast<float4*>(F + ((int64_t)z * T * B + B) * blk);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

void launch_gcn_expand(hipStream_t s, const Dims& d, int Z, int B, const float* C, float* F, bool compact) {
  const int64_t blk = (int64_t)d.N * d.Hc;  // floats per (task, t, window) block; Hc % 4 == 0
  if (compact) {
    const int64_t n4 = (int64_t)(B + d.T - 2) * blk / 4;
    const unsigned gx = (unsigned)std::min<int64_t>((n4 + 255) / 256, 1024);
    k_gcn_compact<<<dim3(gx, (unsigned)Z), 256, 0, s>>>(C, F, B, d.T, blk);
    return;
  }
  const unsigned gx = (unsigned)std::min<int64_t>((blk / 4 + 255) / 256, 64);
  k_gcn_expand<<<dim3(gx, (unsigned)(Z * B * (d.T - 1))), 256, 0, s>>>(C, F, B, d.T, blk);
}

bool gcn_mlp_supported(const Dims& d) { return d.Hc == 256 && d.Cin0 <= 32 && d.Cin0 % 4 == 0 && d.T > 1; }

void launch_gcn_mlp(hipStream_t s, const Dims& d, int Zb, int B, const float* const* xtab, const float* gcn,
                    const GcnWOff& wo, const char* img, float* F, const Drop* drop, bool dedup, bool compact) {
  GcnMlpArgs a{};
  a.xtab = xtab;
  a.gcn = gcn;
  a.wo = wo;
  a.wimg = img;
  a.F = F;
  a.dedup = dedup && B > 1 && !(drop && drop->gcn()) ? 1 : 0;
  a.compact = a.dedup && compact ? 1 : 0;
  a.rows1 = (a.dedup ? B + d.T - 2 : d.T - 1) * d.N;
  a.R1 = (int64_t)(a.dedup ? Zb / B : Zb) * a.rows1;
  a.rows_div = FastDiv((uint32_t)a.rows1);
  a.b_div = FastDiv((uint32_t)B);
  a.n_div = FastDiv((uint32_t)d.N);
  a.N = d.N;
  a.T = d.T;
  a.B = B;
  a.M = (int64_t)B * d.N;
  a.cin0 = d.Cin0;
  if (drop && drop->gcn()) a.dr = *drop;
  const unsigned blocks = (unsigned)((a.R1 + GM_ROWS - 1) / GM_ROWS);
  k_gcn_mlp<256><<<blocks, 64 * GM_WAVES, 0, s>>>(a);
}

}  // namespace smaml
