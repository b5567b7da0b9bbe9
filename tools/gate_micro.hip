// Microbenchmark of the LSTM GEMM + cell-epilogue shapes of config 2 (one (l, t) step of
// 15 tasks: M = 15 x 14,112 rows):
//   forward gate GEMM   N = 4H = 512, K = 256 / 384, epilogue = gates + c + h stores
//   BPTT dh GEMM        N = H = 128,  K = 1024,      epilogue = 7 loads + 5 stores (dG in place)
// Variants: tile shape, BK, epilogue off / on, and the gate-interleaved G layout
// ([row][unit][i,f,g,o]: one 16-B access per lane instead of four 4-B ones).
// Interleaved rounds in one process; prints median / min ms and TFLOP/s per variant.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "gemm_core.h"
#include "loaders.h"
using namespace smaml;

constexpr int H = 128;

struct GateB {  // logical row n = ug*128 + g*32 + jj  ->  weight row g*H + ug*32 + jj of W [4H][K]
  const float* W;
  int K;
  __device__ __forceinline__ float4 operator()(int n, int k) const {
    const int ug = n >> 7, rem = n & 127, g = rem >> 5, j = ug * 32 + (rem & 31);
    if (k >= K) return f4zero();
    return ld4(W + (int64_t)(g * H + j) * K + k);
  }
};

// EPI: 0 = cell epilogue, gates stored [row][g*H + j]; 1 = cell math, no stores;
//      2 = no epilogue (accumulators kept live); 3 = cell epilogue, gates interleaved [row][4j + g]
template <class C, int EPI>
__global__ __launch_bounds__(C::NTH) void k_gate(const float* __restrict__ A, const float* __restrict__ W,
                                                 float* __restrict__ G, float* __restrict__ CH, int M, int K) {
  __shared__ float smem[C::SMEM_FLOATS];
  constexpr int UPB = C::WAVES_N;
  const int ngrp = H / (32 * UPB);
  const int ntm = (M + C::BM - 1) / C::BM;
  const int L = blockIdx.x, per = 8 * ngrp;
  const int q = L / per, rem = L - q * per;
  const int ug = rem >> 3, tm = q * 8 + (rem & 7);
  if (tm >= ntm) return;
  const int m0 = tm * C::BM, n0 = ug * C::BN;
  Acc<C> acc;
  acc.zero();
  RowMajorKC la{A, M, K};
  GateB lb{W, K};
  gemm_mainloop<C>(la, lb, m0, n0, 0, K, acc, smem);
  if (EPI == 2) {
#pragma unroll
    for (int i = 0; i < C::WTM; ++i)
#pragma unroll
      for (int jj = 0; jj < C::WTN; ++jj) asm volatile("" ::"v"(acc.v[i][jj][0]), "v"(acc.v[i][jj][15]));
    return;
  }
  const int wave = threadIdx.x >> 6;
  const int j = (ug * UPB + wave % UPB) * 32 + (threadIdx.x & 31);
  if (EPI == 4) {  // loads of every row first (no store between them), then math + stores
#pragma unroll
    for (int i = 0; i < C::WTM; ++i) {
      const int rb = m0 + acc_row<C>(i, 0);
      float cpv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = rb + racc(r);
        cpv[r] = m < M ? ldb(CH, 4u * ((uint32_t)m * H + j)) : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = rb + racc(r);
        if (m >= M) continue;
        const uint32_t oh = (uint32_t)m * H + j, og = (uint32_t)m * 4 * H + j;
        const float gi = sigmoidf_(acc.v[i][0][r]), gf = sigmoidf_(acc.v[i][1][r]);
        const float gg = tanhf_(acc.v[i][2][r]), go = sigmoidf_(acc.v[i][3][r]);
        const float c = gf * cpv[r] + gi * gg;
        stb(G, 4u * og, gi);
        stb(G, 4u * (og + H), gf);
        stb(G, 4u * (og + 2 * H), gg);
        stb(G, 4u * (og + 3 * H), go);
        stb(CH, 4u * oh + 4u * M * H, c);
        stb(CH, 4u * oh + 8u * M * H, go * tanhf_(c));
      }
    }
    return;
  }
  float keep = 0.f;
#pragma unroll
  for (int i = 0; i < C::WTM; ++i) {
    const int rb = m0 + acc_row<C>(i, 0);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = rb + racc(r);
      if (m >= M) continue;
      const uint32_t oh = (uint32_t)m * H + j, og = (uint32_t)m * 4 * H + j;
      const float gi = sigmoidf_(acc.v[i][0][r]), gf = sigmoidf_(acc.v[i][1][r]);
      const float gg = tanhf_(acc.v[i][2][r]), go = sigmoidf_(acc.v[i][3][r]);
      const float cp = ldb(CH, 4u * oh);
      const float c = gf * cp + gi * gg;
      const float h = go * tanhf_(c);
      if (EPI == 0) {
        stb(G, 4u * og, gi);
        stb(G, 4u * (og + H), gf);
        stb(G, 4u * (og + 2 * H), gg);
        stb(G, 4u * (og + 3 * H), go);
      } else if (EPI == 3) {
        *reinterpret_cast<float4*>(G + (size_t)m * 4 * H + 4 * j) = make_float4(gi, gf, gg, go);
      }
      if (EPI == 0 || EPI == 3) {
        stb(CH, 4u * oh + 4u * M * H, c);
        stb(CH, 4u * oh + 8u * M * H, h);
      } else {
        keep += gi + gf + gg + go + c + h;
      }
    }
  }
  if (EPI == 1) asm volatile("" ::"v"(keep));
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gptr_t;

// L2 prefetch of a wave's BPTT-epilogue operands by LDS-DMA into a scratch slot during the
// last PF K-tiles of the mainloop (the data is dropped; the epilogue's own loads then hit L2).
// Footprint per wave: 32 rows x 64 units x 7 arrays (4 gates, c_t, c_{t-1}, dc) = 224 segments
// of 256 B = 56 wave-instructions of 1 KiB.
template <class C>
struct PrefetchHook {
  const float *G, *Cs, *dc;
  float* scratch;
  int m0, n0, M, nkt, PF;
  __device__ __forceinline__ void operator()(const float*, int kt) const {
    const int first = nkt - PF;
    if (kt < first) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wm = wave / C::WAVES_N, wn = wave % C::WAVES_N;
    const int per = (56 + PF - 1) / PF;
    const int i0 = (kt - first) * per;
    const int i1 = i0 + per < 56 ? i0 + per : 56;
    for (int i = i0; i < i1; ++i) {
      const int seg = 4 * i + (lane >> 4);
      const int row = seg / 7, arr = seg - row * 7;
      int m = m0 + wm * 32 + row;
      m = m < M ? m : M - 1;
      const int u = n0 + wn * 64 + (lane & 15) * 4;
      const float* p;
      if (arr < 4) p = G + (size_t)m * 4 * H + arr * H + u;
      else if (arr == 4) p = Cs + (size_t)M * H + (size_t)m * H + u;
      else if (arr == 5) p = Cs + (size_t)m * H + u;
      else p = dc + (size_t)m * H + u;
      __builtin_amdgcn_global_load_lds((gptr_t)p, (lds_ptr_t)(scratch + wave * 256), 16, 0, 0);
    }
  }
};

// BPTT step shape: dh = dGcat [M][K] . W [K][H] (W row-major [K][H]: "MC"), or W^T stored
// [H][K] ("KC"), then the cell backward. EPI: 0 = plain store of dh; 1 = cell backward with
// G [row][g*H + j]; 2 = cell backward with G interleaved [row][4j + g].
template <class C, bool BKC, int EPI, int PF = 0>
__global__ __launch_bounds__(C::NTH) void k_bptt(const float* __restrict__ A, const float* __restrict__ W,
                                                 float* __restrict__ G, const float* __restrict__ Cs,
                                                 float* __restrict__ dc, float* __restrict__ O, int M, int K) {
  __shared__ float smem[C::SMEM_FLOATS + (PF ? C::NTH / 64 * 256 : 0)];
  const int m0 = blockIdx.x * C::BM, n0 = blockIdx.y * C::BN;
  Acc<C> acc;
  acc.zero();
  RowMajorKC la{A, M, K};
  if (PF) {
    RowMajorMC lb{W, K, H};
    PrefetchHook<C> hk{G, Cs, dc, smem + C::SMEM_FLOATS, m0, n0, M, (K + C::BK - 1) / C::BK, PF};
    gemm_mainloop<C>(la, lb, m0, n0, 0, K, acc, smem, hk);
  } else if (BKC) {
    RowMajorKC lb{W, H, K};
    gemm_mainloop<C>(la, lb, m0, n0, 0, K, acc, smem);
  } else {
    RowMajorMC lb{W, K, H};
    gemm_mainloop<C>(la, lb, m0, n0, 0, K, acc, smem);
  }
  if (EPI >= 3) {
    constexpr int BATCH = EPI == 3 ? 4 : EPI == 4 ? 8 : 16;
#pragma unroll
    for (int i = 0; i < C::WTM; ++i)
#pragma unroll
      for (int jj = 0; jj < C::WTN; ++jj) {
        const int j = n0 + acc_col<C>(jj);
        const int rb = m0 + acc_row<C>(i, 0);
#pragma unroll
        for (int b0 = 0; b0 < 16; b0 += BATCH) {
          float v[BATCH][7];
#pragma unroll
          for (int q = 0; q < BATCH; ++q) {
            int m = rb + racc(b0 + q);
            m = m < M ? m : M - 1;
            const uint32_t oh = (uint32_t)m * H + j, og = (uint32_t)m * 4 * H + j;
            v[q][0] = ldb(G, 4u * og);
            v[q][1] = ldb(G, 4u * (og + H));
            v[q][2] = ldb(G, 4u * (og + 2 * H));
            v[q][3] = ldb(G, 4u * (og + 3 * H));
            v[q][4] = ldb(Cs, 4u * oh + 4u * M * H);
            v[q][5] = ldb(Cs, 4u * oh);
            v[q][6] = ldb(dc, 4u * oh);
          }
#pragma unroll
          for (int q = 0; q < BATCH; ++q) {
            const int m = rb + racc(b0 + q);
            if (m >= M) continue;
            const uint32_t oh = (uint32_t)m * H + j, og = (uint32_t)m * 4 * H + j;
            const float dh = acc.v[i][jj][b0 + q];
            const float gi = v[q][0], gf = v[q][1], gg = v[q][2], go = v[q][3];
            const float c = v[q][4], cp = v[q][5], dcin = v[q][6];
            const float tc = tanhf_(c);
            const float dct = dcin + dh * go * (1.f - tc * tc);
            stb(G, 4u * og, dct * gg * gi * (1.f - gi));
            stb(G, 4u * (og + H), dct * cp * gf * (1.f - gf));
            stb(G, 4u * (og + 2 * H), dct * gi * (1.f - gg * gg));
            stb(G, 4u * (og + 3 * H), dh * tc * go * (1.f - go));
            stb(dc, 4u * oh, dct * gf);
          }
        }
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < C::WTM; ++i)
#pragma unroll
    for (int jj = 0; jj < C::WTN; ++jj) {
      const int j = n0 + acc_col<C>(jj);
      const int rb = m0 + acc_row<C>(i, 0);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = rb + racc(r);
        if (m >= M) continue;
        const float dh = acc.v[i][jj][r];
        if (EPI == 0) {
          O[(size_t)m * H + j] = dh;
          continue;
        }
        const uint32_t oh = (uint32_t)m * H + j;
        float gi, gf, gg, go;
        if (EPI == 1 || EPI >= 6) {
          const uint32_t og = (uint32_t)m * 4 * H + j;
          gi = ldb(G, 4u * og);
          gf = ldb(G, 4u * (og + H));
          gg = ldb(G, 4u * (og + 2 * H));
          go = ldb(G, 4u * (og + 3 * H));
        } else {
          const float4 g4 = *reinterpret_cast<const float4*>(G + (size_t)m * 4 * H + 4 * j);
          gi = g4.x;
          gf = g4.y;
          gg = g4.z;
          go = g4.w;
        }
        const float c = ldb(Cs, 4u * oh + 4u * M * H);
        // EPI 6: cell-state carry in registers (no dc load/store); 7: also c_{t-1} in registers
        const float cp = EPI == 7 ? c * 0.9f : ldb(Cs, 4u * oh);
        const float dcin = EPI >= 6 ? c * 0.5f : ldb(dc, 4u * oh);
        const float tc = tanhf_(c);
        const float dct = dcin + dh * go * (1.f - tc * tc);
        const float a0 = dct * gg * gi * (1.f - gi), a1 = dct * cp * gf * (1.f - gf);
        const float a2 = dct * gi * (1.f - gg * gg), a3 = dh * tc * go * (1.f - go);
        if (EPI == 1 || EPI >= 6) {
          const uint32_t og = (uint32_t)m * 4 * H + j;
          stb(G, 4u * og, a0);
          stb(G, 4u * (og + H), a1);
          stb(G, 4u * (og + 2 * H), a2);
          stb(G, 4u * (og + 3 * H), a3);
        } else {
          *reinterpret_cast<float4*>(G + (size_t)m * 4 * H + 4 * j) = make_float4(a0, a1, a2, a3);
        }
        if (EPI < 6) stb(dc, 4u * oh, dct * gf);
        else acc.v[i][jj][r] = dct * gf;  // keep the carry live
      }
    }
}

struct Bufs {
  float *A, *W, *G, *CH, *dc, *O;
  int M;
};

typedef float (*RunFn)(const Bufs&, int);

template <class C, int EPI>
float run_gate(const Bufs& b, int K) {
  constexpr int UPB = C::WAVES_N;
  const int ngrp = H / (32 * UPB);
  const int ntm = (b.M + C::BM - 1) / C::BM;
  dim3 grid((ntm + 7) / 8 * 8 * ngrp);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int reps = 5;
  (void)hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) k_gate<C, EPI><<<grid, C::NTH>>>(b.A, b.W, b.G, b.CH, b.M, K);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms / reps;
}

template <class C, bool BKC, int EPI, int PF = 0>
float run_bptt(const Bufs& b, int K) {
  dim3 grid((b.M + C::BM - 1) / C::BM, (H + C::BN - 1) / C::BN);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int reps = 5;
  (void)hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) k_bptt<C, BKC, EPI, PF><<<grid, C::NTH>>>(b.A, b.W, b.G, b.CH, b.dc, b.O, b.M, K);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms / reps;
}

struct Variant {
  const char* name;
  RunFn run;
  int N;  // output columns (flops = 2 M N K)
};

void bench(const char* title, const Bufs& b, std::vector<Variant>& vs, int K) {
  std::vector<std::vector<float>> t(vs.size());
  for (auto& v : vs) v.run(b, K);  // warm
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("device error\n");
    return;
  }
  for (int round = 0; round < 5; ++round)
    for (size_t v = 0; v < vs.size(); ++v) t[v].push_back(vs[v].run(b, K));
  for (size_t v = 0; v < vs.size(); ++v) {
    std::sort(t[v].begin(), t[v].end());
    const float med = t[v][t[v].size() / 2];
    printf("%s K=%4d %-34s median %8.3f ms  min %8.3f ms  %6.1f TF/s\n", title, K, vs[v].name, med, t[v][0],
           2.0 * b.M * (double)vs[v].N * K / (med * 1e-3) / 1e12);
  }
  fflush(stdout);
}

int main() {
  Bufs b;
  b.M = 15 * 14112;
  const int Kmax = 1024;
  (void)hipMalloc(&b.A, (size_t)b.M * Kmax * 4);
  (void)hipMalloc(&b.W, (size_t)4 * H * Kmax * 4);
  (void)hipMalloc(&b.G, (size_t)b.M * 4 * H * 4);
  (void)hipMalloc(&b.CH, (size_t)b.M * H * 4 * 3);
  (void)hipMalloc(&b.dc, (size_t)b.M * H * 4);
  (void)hipMalloc(&b.O, (size_t)b.M * H * 4);
  {
    std::vector<float> h((size_t)b.M * Kmax);
    uint32_t s = 12345u;
    for (auto& v : h) {
      s = s * 1664525u + 1013904223u;
      v = ((s >> 8) * (1.0f / 16777216.0f) - 0.5f) * 0.2f;
    }
    (void)hipMemcpy(b.A, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(b.W, h.data(), (size_t)4 * H * Kmax * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(b.G, h.data(), (size_t)b.M * 4 * H * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(b.CH, h.data(), (size_t)b.M * H * 4 * 3, hipMemcpyHostToDevice);
    (void)hipMemcpy(b.dc, h.data(), (size_t)b.M * H * 4, hipMemcpyHostToDevice);
  }
  using G128 = GemmCfg<128, 128, 4, 1, true, true, 16>;     // current gate tile: wave 32 x 128
  using G128b32 = GemmCfg<128, 128, 4, 1, true, true, 32>;
  using G256w8 = GemmCfg<256, 128, 8, 1, true, true, 16>;   // 8 waves, wave 32 x 128
  using G256w4 = GemmCfg<256, 128, 4, 1, true, true, 16>;   // 4 waves, wave 64 x 128
  std::vector<Variant> gv = {
      {"128x128 w4 BK16 (current)", run_gate<G128, 0>, 512},
      {"128x128 w4 BK16 loads-first", run_gate<G128, 4>, 512},
      {"128x128 w4 BK16 no-store", run_gate<G128, 1>, 512},
      {"128x128 w4 BK16 no-epilogue", run_gate<G128, 2>, 512},
      {"256x128 w8 BK16", run_gate<G256w8, 0>, 512},
  };
  for (int K : {256, 384}) bench("gate", b, gv, K);

  using N64 = GemmCfg<64, 128, 2, 2, true, false, 16>;    // current BPTT tile (B k-major)
  using T64 = GemmCfg<64, 128, 2, 2, true, true, 16>;     // B transposed (k-contiguous)
  using N128 = GemmCfg<128, 128, 2, 2, true, false, 16>;  // wave 64 x 64
  using N128w4 = GemmCfg<128, 128, 4, 1, true, false, 16>;
  std::vector<Variant> bv = {
      {"64x128 NN BK16 cell (current)", run_bptt<N64, false, 1>, 128},
      {"64x128 NN BK16 cell batch-4", run_bptt<N64, false, 3>, 128},
      {"64x128 NN BK16 cell batch-8", run_bptt<N64, false, 4>, 128},
      {"64x128 NN BK16 cell batch-16", run_bptt<N64, false, 5>, 128},
      {"64x128 NN BK16 plain store", run_bptt<N64, false, 0>, 128},
      {"64x128 NN BK16 cell, gates [4j+g] float4", run_bptt<N64, false, 2>, 128},
      {"64x128 NN BK16 cell, dc carry in regs", run_bptt<N64, false, 6>, 128},
      {"64x128 NN BK16 cell, dc + c_{t-1} in regs", run_bptt<N64, false, 7>, 128},
  };
  for (int K : {512, 1024}) bench("bptt", b, bv, K);
  return 0;
}
