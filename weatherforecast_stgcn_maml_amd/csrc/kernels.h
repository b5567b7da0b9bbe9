// Internal (C++) interface between the C-ABI driver (api.cpp) and the HIP kernels
// (kernels.hip). Not part of the public boundary -- see include/smaml.h for that.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smaml {

constexpr int ELLW = 8;        // ELL width of the normalised t=0 adjacency (max in-degree 6 + self)
constexpr int MAX_LAYERS = 8;

// Every host-built plan / launch-argument struct below gives each member a default initialiser, so a
// plan a caller fills only partly can never hand a kernel an indeterminate field (round 4 found two
// faults of that class; tools/host_sanitize.cpp builds this header with -Werror=missing-field-initializers).
struct Dims {
  int N = 0;      // nodes per region (graph size)
  int T = 0;      // window (time steps)
  int Cin0 = 0;   // input channels (24)
  int Hc = 0;     // GCN hidden channels (256)
  int H = 0;      // LSTM hidden (128)
  int L = 0;      // LSTM layers (4)
  int Hf = 0;     // forecast horizon (8)
  int C = 0;      // output channels (12)
  int HfC = 0;    // head width (96)
};

struct LayerOff {
  int64_t wih = 0, whh = 0, bih = 0, bhh = 0;  // offsets into the flat trainable vector
  int cin = 0;
};

struct ParamOff {
  LayerOff lay[MAX_LAYERS] = {};
  int64_t wo = 0, bo = 0;
  int64_t P = 0;  // padded flat size (stride between tasks' fast weights)
  int64_t n_valid = 0;
};

struct GcnOff {
  int64_t w[4] = {}, b[4] = {};
  int cin[4] = {};
  int64_t total = 0;
};

// Train-mode dropout (hybrid_model.py:67,70,73 GCN outputs; nn.LSTM's inter-layer dropout :47;
// the head input :108) from counter-based masks: element idx of site (kind, step, layer) is
// kept iff (mix32(site ^ lo(idx) ^ hi(idx) * golden) >> 8) >= thr (one mixing round per
// element: the site seed is already mixed), and scaled by 1 / (1 - p). oracle/refcpu.py
// (drop_keep) restates the same function, so the masks agree bit for bit. Element indices
// (task = global task id):
//   kind 1, layer k (GCN conv k+1 output): ((task * B + s) * T*N + row) * Hc + channel
//   kind 2, layer l (LSTM layer l output fed to layer l+1): ((task * T + t) * M + m) * H + unit
//   kind 3 (head input h_T): (task * M + m) * H + unit
__host__ __device__ inline uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
__host__ __device__ inline uint32_t drop_site(uint32_t seed, int kind, int step, int layer) {
  return mix32(seed ^ mix32(((uint32_t)kind << 24) ^ ((uint32_t)step << 8) ^ (uint32_t)layer));
}
__host__ __device__ inline bool drop_keep(uint32_t site, uint64_t idx, uint32_t thr) {
  return (mix32(site ^ (uint32_t)idx ^ ((uint32_t)(idx >> 32) * 0x9E3779B9U)) >> 8) >= thr;
}
struct Drop {
  uint32_t seed = 0;
  int step = 0;                      // inner step (K = the query batch) whose forward the masks belong to
  uint32_t thr_gcn = 0, thr_lstm = 0;  // round(p * 2^24); 0 = off
  float sc_gcn = 1.f, sc_lstm = 1.f;  // 1 / (1 - p)
  const int* task_id = nullptr;      // [Z] global task id of each workspace task (device)
  __host__ __device__ bool gcn() const { return thr_gcn != 0; }
  __host__ __device__ bool lstm() const { return thr_lstm != 0; }
};

// Launch counters per kernel variant (tile configuration), read through smaml_variant_counts so
// the parity tests can assert which configurations they exercised. Order = _capi.VARIANTS.
enum Variant {
  V_FWD = 0,         // k_lstm_fwd_step (fused gate GEMM + cell)
  V_FWD_DROP,        // k_lstm_fwd_step_drop
  V_FWD_SPLIT,       // k_lstm_fwd_part + k_lstm_fwd_cell (small grids)
  V_FWD_IMG,         // k_lstm_fwd_step with pre-split weight images (also counted as V_FWD)
  V_FWDD,            // k_lstm_fwd_dual, primal recomputed
  V_FWDD_KEPT,       // k_lstm_fwd_dual, tangent only (primal kept)
  V_FWDD_IMG,        // k_lstm_fwd_dual with pre-split weight images (also counted as one of the above)
  V_BWD_BIG,         // k_lstm_bwd_step, big tiles (CfgBwd: SMAML_BWD_BM x 128, 128 x 128 in this build)
  V_BWD_SMALL,       // k_lstm_bwd_step, 64x64 tiles
  V_BWD_SPLIT,       // k_lstm_bwd_part + k_lstm_bwd_cell (small grids)
  V_BWDD_BIG,        // k_lstm_bwd_dual, big tiles (CfgBwdD, 128 x 128), primal recomputed
  V_BWDD_BIG_KEPT,   // k_lstm_bwd_dual, big tiles (CfgBwdD, 128 x 128), tangent only
  V_BWDD_SMALL,      // k_lstm_bwd_dual, 64x64 tiles, primal recomputed
  V_BWDD_SMALL_KEPT, // k_lstm_bwd_dual, 64x64 tiles, tangent only
  V_WGRAD,           // k_wgrad launches (any tile)
  V_WGRAD_WIDE,      // k_wgrad with 256 x 256 tiles (also counted as V_WGRAD)
  V_WGRAD_PAIR,      // k_wgrad summing two problems (tangent weight gradient; also counted as V_WGRAD)
  V_FWD_KW,          // k_lstm_fwd_kw (small grids: K split over the waves of one workgroup)
  V_BWD_KW,          // k_lstm_bwd_kw (same, BPTT)
  V_GCN_DEDUP,       // k_gcn_mlp once per distinct stream row of consecutive windows
  V_XG_DEDUP,        // k_xg_dedup: layer 0's input projection once per distinct stream row (big-tile forward)
  V_WGRAD_DEDUP,     // layer 0's input-weight gradient over distinct stream rows (k_dg_rowsum + gathered k_wgrad)
  V_F_COMPACT,       // GCN features stored once per distinct stream row (Work::fcompact)
  NVAR
};

// Build-time defaults of the run-time knobs below.
#ifndef SMAML_BWD_BIG_MIN
#define SMAML_BWD_BIG_MIN (3 * 256)  // BPTT launches with >= this many 64-row x 128-unit tile units use the big tiles
#endif
#ifndef SMAML_BWDD_BIG_MIN
#define SMAML_BWDD_BIG_MIN (3 * 256)
#endif
#ifndef SMAML_SPLIT_MAX
#define SMAML_SPLIT_MAX 4  // split-K ways for small-grid LSTM steps (1 = off)
#endif

// Run-time tile-selection knobs (smaml_set_option; defaults = the build-time thresholds).
struct Knobs {
  int bwd_big_min = 0;   // BPTT launches with >= this many 64-row x 128-unit tile units (a 128 x 128 big tile counts
                     // 2) use the big tiles (else 64x64 / split-K)
  int bwdd_big_min = 0;  // same, tangent BPTT
  int split_max = 1;     // split-K ways for small-grid LSTM steps (1 = off)
  int wgrad_group_max_rows = 0;  // backward with Z*M <= this: all LSTM weight gradients in one launch
  int wgrad_group_wgs = 1;       // workgroups that grouped launch aims for
  int gcn_fused = 0;             // 1: GCN rows t >= 1 through the fused four-layer kernel (k_gcn_mlp)
  int gate_img = 0;              // 1: gate GEMMs read pre-split weight images (launch_split_gate)
  int wgrad_wide = 0;            // 1: weight gradients with 256-multiple column counts on 256 x 256 tiles
  int wgrad_pair = 0;            // 1: the two passes of a tangent weight gradient (layers >= 1) as one launch
  int bwdd_remap = 0;            // 1: tangent BPTT tiles in pair-segment order per XCD (kernels_dual.hip PairRemap)
  int small_kw = 0;              // small-grid LSTM steps as one launch with the K split over waves (kernels_small.hip):
                             // 1 = on, 2 = on with pre-split BPTT weight images (launch_split_bwd), 0 = split-K pairs
  int gcn_dedup = 0;             // 1: batches of consecutive windows run the fused GCN rows once per distinct stream row
  int xg_dedup = 0;              // 1: ... and layer 0's input projection F . W_ih0^T (and its tangent) once per
                                 // distinct stream row (k_xg_dedup), added to the gate accumulators
  int wgrad_dedup = 0;           // 1: ... and layer 0's input-weight gradient (and its tangent) over the distinct
                                 // stream rows: row sums of dG0 (k_dg_rowsum) times the gathered F rows
  int bptt_streams = 1;          // > 1: the big-tile BPTT diagonals (primal and tangent) split into this many row
                                 // chunks on side streams (a chunk's rows depend on nothing else), so one
                                 // chunk's next diagonal fills the other's tail; weight gradients after the sweep
  int fwd_streams = 0;           // the same for the big-tile forward diagonals (primal and tangent); 0 = auto
  int f_compact = 0;             // 1: where every reader of a step's features goes through the distinct stream rows
                                 // (xg_dedup forwards, wgrad_dedup backwards), the GCN stores only those rows
};
#ifndef SMAML_GATE_IMG
#define SMAML_GATE_IMG 1
#endif
#ifndef SMAML_GCN_FUSED
#define SMAML_GCN_FUSED 1
#endif
#ifndef SMAML_BWDD_REMAP_DEFAULT
#define SMAML_BWDD_REMAP_DEFAULT 1  // tangent BPTT pair-segment tile order: -0.55 GB of HBM reads per launch,
#endif                              // time-neutral (3-round A/B 1785.6 -> 1784.5 ms per meta-step)
#ifndef SMAML_SMALL_KW
#define SMAML_SMALL_KW 1
#endif
#ifndef SMAML_XG_DEDUP_DEFAULT
#define SMAML_XG_DEDUP_DEFAULT 1
#endif
#ifndef SMAML_WGRAD_DEDUP_DEFAULT
#define SMAML_WGRAD_DEDUP_DEFAULT 1
#endif
#ifndef SMAML_BPTT_STREAMS_DEFAULT
#define SMAML_BPTT_STREAMS_DEFAULT 2  // A/B (profiles/r05_ab_streams*.log): config 2 1653 -> 1618 ms, config-5 share 4453 -> 4308 ms
#endif
#ifndef SMAML_F_COMPACT_DEFAULT
#define SMAML_F_COMPACT_DEFAULT 1
#endif
#ifndef SMAML_FWD_STREAMS_DEFAULT
#define SMAML_FWD_STREAMS_DEFAULT 0  // auto (api.cpp fwd_chunks): config-5 share 4308 -> 4202 ms; config 2 (not chunked) +25 ms
#endif
#ifndef SMAML_WGRAD_PAIR
#define SMAML_WGRAD_PAIR 1
#endif
#ifndef SMAML_WGRAD_GROUP_ROWS
#define SMAML_WGRAD_GROUP_ROWS 2048
#endif
#ifndef SMAML_WGRAD_GROUP_WGS
#define SMAML_WGRAD_GROUP_WGS 256
#endif

// Activations of one forward pass for Z tasks x B samples (M = B*N sequences per task).
// ---- pre-split gate-GEMM weight images (kernels.hip launch_split_gate) ----
// Per task: for layer l, segment (W_ih | W_hh), unit group ug (32 units), K-tile kt the staged-split
// LDS image (X6Img<128, KC, 16>: 3 bf16 planes x 128 rows x 16 k) of SegGateBt's 128 x 16 tile, so
// the gate GEMMs copy weight tiles into LDS with direct-to-LDS loads instead of loading and
// splitting them in every workgroup (the weights are the same for all row tiles of a launch).
constexpr int GATE_IMG_BYTES = 3 * 128 * 16 * 2;
struct GateImgs {
  char* th = nullptr;               // images of theta (launch_split_gate), null = not built
  char* u = nullptr;                // images of the tangent direction U (second-order sweep), or null
  int64_t tstride = 0;              // bytes per task
  int64_t off[MAX_LAYERS][2] = {};  // byte offset of (layer, W_ih | W_hh) in a task's images
};
// ---- pre-split BPTT weight images (kernels_small.hip launch_split_bwd; small-grid BPTT) ----
// Per task, for W_hh of every layer and W_ih of layers >= 1 (the [4H][H] matrices the BPTT step reads
// as B[k][j]): per K-tile kt (16 gate rows) and unit tile tn (32 units) three bf16 planes of
// [32 units][16 k], so a lane's MFMA B fragment (unit jj, k = 8h .. 8h + 7) is one 16-B load per plane.
constexpr int BWD_IMG_BYTES = 3 * 32 * 16 * 2;
struct BwdImgs {
  char* th = nullptr;               // null = not built
  int64_t tstride = 0;              // bytes per task
  int64_t off_hh[MAX_LAYERS] = {};  // byte offset of W_hh(l) in a task's images
  int64_t off_ih[MAX_LAYERS] = {};  // ... W_ih(l), l >= 1 (0 for l = 0: not built)
};
// Layer 0's input projection of a step whose every task reads B consecutive windows, formed once per
// distinct stream row by k_xg_dedup (launch_xg_dedup): per task [(2B + T - 2) N][4H] floats -- rows
// [0, B N) the t = 0 rows (row b N + n: their GCN features see the graph, so each window's are its own),
// then stream rows s = 1 .. B + T - 2 (row B N + (s - 1) N + n). Window b's step t >= 1 reads stream row
// b + t, i.e. row M + (t - 1) N + m with m = b N + n: one fixed shift per step, contiguous in m. The gate
// kernels start layer 0's accumulators from these rows (no bias) and run their K loop over the
// recurrent segment only.
struct XgDedup {
  const float* xg = nullptr;     // F . W_ih0^T of src, or null
  const float* rxg = nullptr;    // F . U_ih0^T of u_src (second-order sweep), or null
  const float* src = nullptr;    // the parameter vectors they were formed from (launchers check them)
  const float* u_src = nullptr;
  int64_t zstride = 0;           // floats per task
  int N = 0;
};
__host__ __device__ inline int64_t xg_dedup_rows(int B, int T, int N) { return (int64_t)(2 * B + T - 2) * N; }
// first row of step t's block of window rows in a task's XgDedup table (M = B N)
__host__ __device__ inline int64_t xg_dedup_row0(int t, int M, int N) { return t == 0 ? 0 : (int64_t)M + (int64_t)(t - 1) * N; }

struct Work {
  int Z = 0, B = 0, M = 0;
  BwdImgs bimg{};           // pre-split BPTT weight images (launch_split_bwd), small-grid BPTT only
  const float* bimg_src = nullptr; // the parameter vector bimg.th was split from
  const float* xg = nullptr;       // small-grid forward: layer 0's input projection F . W_ih0^T for all steps
                           // [Z][T][M][4H] (run_lstm), or null: the layer-0 steps form it themselves
  const float* xg_src = nullptr;   // the parameter vector xg was formed with
  XgDedup xgd{};                   // big-tile forward: layer 0's projection once per distinct stream row
  int consec = 0;                  // this step's tasks each read B consecutive windows (set by the forward)
  int fcompact = 0;                // F holds only the distinct rows of those windows, in XgDedup's row order
                                   // (rows [0, (2B + T - 2) N) of each task's slab): read through XgDedup only
  GateImgs gimg{};         // pre-split images of the weights the gate GEMMs read (launch_split_gate)
  const float* gimg_src = nullptr; // the parameter vector gimg.th was split from (kernels use it only for that one)
  const float* gimg_u_src = nullptr;// ... and gimg.u (the sweep's tangent direction)
  int64_t* vcount = nullptr;       // [NVAR] launch counters (ctx-owned; may be null)
  Knobs kn{};
  float *gcnA = nullptr, *gcnB = nullptr;    // [Z*B][T*N][Hc] ping-pong
  float* F = nullptr;              // [Z][T][M][Hc] LSTM layer-0 input
  float *Hs = nullptr, *Cs = nullptr, *Gs = nullptr;   // [L][Z][T][M][H] / [L][Z][T][M][H] / [L][Z][T][M][4H]
  float* dG = nullptr;             // BPTT output [L][Z][T][M][4H]: == Gs (in place) unless the step's
                           // primal is kept for the second-order sweep (then its own slab)
  float* dh = nullptr;             // optional: the BPTT's dh [L][Z][T][M][H] (kept for the SO sweep)
  int primal_kept = 0;       // SO sweep: Hs/Cs/Gs/dG/dh hold this step's primal (tangent-only kernels)
  float *dH = nullptr, *dc = nullptr;        // head's dh_T [Z][M][H]; cell-state carry per layer [L][Z][M][H]
                           // (the BPTT writes dG in place over Gs: [L][Z][T][M][4H])
  float *pred = nullptr, *dpred = nullptr;   // [Z][M][HfC]
  float* wpart = nullptr;          // split-K partial slabs
  int64_t wpart_floats = 0;
  float* lpart = nullptr;          // loss partials [Z][lblocks]
  int lblocks = 0;
  double* sqpart = nullptr;        // [Z][SQB]
  // second-order (tangent) buffers; null unless reserved with so = true
  float *RHs = nullptr, *RCs = nullptr, *RGs = nullptr;// like Hs, Cs, Gs
  float *RdH = nullptr, *Rdc = nullptr;      // like dH, dc (R(dG) is written in place over RGs)
  float* Rdpred = nullptr;         // like dpred
  // dropout (zero thresholds: off) and the masked head inputs drop(h_T), drop(R h_T) [Z][M][H]
  Drop drop{};
  float *hTd = nullptr, *RhTd = nullptr;
};

inline void count_variant(const Work& w, Variant v) {
  if (w.vcount) ++w.vcount[v];
}

constexpr int SQB = 64;  // blocks per task for squared-norm partials

// Grid-wide barrier of the bookkeeping kernels (k_inner_sgd, k_sweep_update). A plain launch gives NO
// co-residency guarantee, so the barrier relies on the launcher's grid sizing (grid_barrier_blocks: a
// quarter of the device's resident capacity for the kernel, so up to four such grids from processes
// sharing the GPU fit at once; blocks of ordinary kernels never wait on ours and free their slots) and
// bounds every spin: a waiter that has not seen the barrier open within `timeout` wall-clock ticks, or
// that sees another waiter's timeout, marks the error word, reports it through the pinned host flag
// and returns false; the kernel then skips its second phase and exits, so a stranded grid drains and
// the host turns the flag into SMAML_EHIP (api.cpp check_device_error) instead of hanging.
// State w[0] = arrivals at the open barrier, w[1] = generation, w[2] = error; the last arrival resets
// w[0] and bumps w[1], so nothing is mirrored on the host and a failed launch leaves no stale count.
// One barrier state per context, used by that context's stream only (launches are stream-ordered).
// Release: the block's stores are made visible before it arrives; acquire: the waiting lane's
// agent-scope load invalidates this CU's L1, so the block then reads the other blocks' results.
struct GridBar {
  unsigned* w = nullptr;     // device words [3]
  int* host_err = nullptr;   // pinned, device-mapped flag (may be null)
  uint64_t timeout = 0;      // wall_clock64 ticks a waiter spins before giving up
};
__device__ __forceinline__ bool grid_barrier(const GridBar& gb, unsigned nb) {
  __shared__ int ok_s;
  __syncthreads();
  if (threadIdx.x == 0) {
    int ok = 1;
    unsigned* cnt = gb.w;
    unsigned* gen = gb.w + 1;
    unsigned* err = gb.w + 2;
    const unsigned g0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == nb - 1) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gen, g0 + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const uint64_t t0 = wall_clock64();
      while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g0) {
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
            wall_clock64() - t0 > gb.timeout) {
          __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (gb.host_err) __hip_atomic_store(gb.host_err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    ok_s = ok;
  }
  __syncthreads();
  return ok_s != 0;
}
// Launch plan of a bookkeeping kernel over `items` (task, chunk) items: `fused` = one launch with the
// grid barrier (nb blocks, each looping over items), else the two phases as two launches of the same
// kernel (same partition and summation order: bitwise-equal results).
struct BarPlan {
  GridBar gb{};
  int fused = 0;     // 1: grid-barrier launch
  int oversize = 0;  // debug: > 0 launches oversize x the resident capacity + 1 blocks (never co-resident)
};
// Grid of a grid-barrier launch over `items` items given the kernel's resident capacity `cap` (blocks
// the device holds at once): min(items, cap / 4) -- a quarter, so up to four processes sharing the GPU
// each fit one such grid beside the others (ordinary kernels drain and free their slots); the kernels
// loop over their items, so any grid size is correct. 0 = capacity unknown (the caller runs the
// two-launch form). `oversize` > 0 (debug knob) returns cap * oversize + 1 blocks, a grid that can
// never be co-resident, to exercise the bounded wait.
inline int grid_barrier_grid(int cap, int items, int oversize) {
  if (cap <= 0 || items <= 0) return 0;
  if (oversize > 0) return cap * oversize + 1;
  const int q = cap / 4 > 0 ? cap / 4 : 1;
  return items < q ? items : q;
}
// grid_barrier_grid with the capacity of `fn` on the current device
// (hipOccupancyMaxActiveBlocksPerMultiprocessor x CUs at NT threads)
int grid_barrier_blocks(const void* fn, int items, int oversize);
int grid_barrier_capacity(const void* fn);  // resident blocks of fn on the current device (0: unknown)
#ifndef SMAML_WGRAD_MAXSPLIT
#define SMAML_WGRAD_MAXSPLIT 128  // split-K slices per weight gradient (partial-slab capacity)
#endif

// One anti-diagonal of the (layer, step) grid of the LSTM forward: the problems (l, t) with
// l + t = diag are independent ((l, t) reads only (l-1, t) and (l, t-1), both on the previous
// diagonal), so they share one launch: T + L - 1 launches per sweep instead of T * L, each up
// to L times wider (fills the chip when a rank holds few tasks). Problem p owns blocks
// [off[p], off[p+1]) (multiples of 8, keeping the XCD-aware gate tile mapping).
struct FwdWave {
  int n = 0;
  int l[MAX_LAYERS] = {}, t[MAX_LAYERS] = {}, off[MAX_LAYERS + 1] = {};
  LayerOff lo[MAX_LAYERS] = {};
  int tm0 = 0, ntm = 0;  // big-tile gate kernels: row tiles [tm0, tm0 + ntm) (ntm 0 = all of them)
};
// Backward counterpart: problems (l, t) with (L-1-l) + (T-1-t) = e. Step (l, t) forms
//   dh = [dG(l+1, t) | dG(l, t+1)] . [W_ih(l+1) ; W_hh(l)]   (one K = 8H GEMM; the dX of the
// layer above is fused here instead of a separate GEMM), reading only the previous diagonal.
struct BwdWave {
  int n = 0;
  int l[MAX_LAYERS] = {}, t[MAX_LAYERS] = {}, off[MAX_LAYERS + 1] = {};
  LayerOff lo[MAX_LAYERS] = {};
  int64_t wih_up[MAX_LAYERS] = {};  // W_ih offset of layer l+1 (unused at the top layer)
  int tm0 = 0;  // big-tile kernels: first row tile of this launch (row chunks on separate streams)
};
double bwd_wave(const Dims& d, const Work& w, const ParamOff& po, int e, int blocks_per_problem, bool dual,
                BwdWave& wv);
// Fills wv for diagonal diag; returns its algorithmic flops (dual: primal + tangent GEMMs).
double fwd_wave(const Dims& d, const Work& w, const ParamOff& po, int diag, int blocks_per_problem, bool dual,
                FwdWave& wv);

const char* products_info();  // product form per GEMM family as built (kernels.hip)

// ---- launchers (kernels.hip) ----
// drop_rps: rows per sample of the dropout element index (default rows_per_sample; the t = 0 path of
// run_gcn runs N-row "samples" but indexes masks as the T*N-row samples they belong to)
void launch_gcn_layer(hipStream_t s, const Dims& d, int layer, int Zb, int B, const float* const* xtab,
                      const float* src, float* dst, bool remap_lstm, bool relu, const float* W,
                      const float* b, int cin, int cout, const int* ell_c, const float* ell_v, int rows_per_sample,
                      int ell_rows, const Drop* drop = nullptr, int drop_rps = 0);

// Exact unsigned division by a run-time invariant d for n < 2^31 (one 64-bit multiply):
// m = ceil(2^(32+s) / d), s = ceil(log2 d)  =>  n / d == (n * m) >> (32 + s).
struct FastDiv {
  uint64_t m = 0;
  uint32_t s = 0;
  uint32_t d = 0;
  FastDiv() = default;
  __host__ explicit FastDiv(uint32_t dd) : d(dd) {
    s = 0;
    while ((1ull << s) < dd) ++s;
    m = (uint64_t)((((unsigned __int128)1 << (32 + s)) + dd - 1) / dd);
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    return (uint32_t)(((unsigned __int128)n * m) >> (32 + s));
  }
};

int64_t gate_img_bytes(const Dims& d, GateImgs* layout);  // bytes per task; fills off[] / tstride
void launch_split_gate(hipStream_t s, const Dims& d, const ParamOff& po, const float* theta, int64_t tstride, int Z,
                       const GateImgs& gi, char* dst);

// ---- fused GCN stack for the rows t >= 1 (kernels_gcn.hip) ----
struct GcnWOff {  // offsets of conv{1..4}.lin.weight / conv{1..4}.bias in the GCN parameter vector
  int64_t w[4] = {}, b[4] = {};
};
struct GcnMlpArgs {
  const float* const* xtab = nullptr;  // [Z*B] sample window pointers ([T*N][Cin0] each)
  const float* gcn = nullptr;          // GCN parameter vector (biases)
  GcnWOff wo{};
  const char* wimg = nullptr;          // pre-split W images (launch_gcn_wsplit)
  float* F = nullptr;                  // [Z][T][B*N][Hc]
  int64_t R1 = 0, M = 0;               // rows t >= 1 over all samples; B*N
  FastDiv rows_div{}, b_div{}, n_div{};
  int rows1 = 0, N = 0, T = 0, B = 0, cin0 = 0;
  int compact = 0;                     // dedup: store each distinct row ONCE, at its compact row (XgDedup order)
  int dedup = 0;                       // 1: every task's B windows are consecutive; rows1 = (B + T - 2) * N distinct
                             // time steps per task, each row written to every (sample, t >= 1) holding it
  Drop dr{};
};
bool gcn_mlp_supported(const Dims& d);
// compact: only the distinct rows, F[z][M + (s - 1) N + n] = C[z][s][n] for s >= 1 (XgDedup order)
void launch_gcn_expand(hipStream_t s, const Dims& d, int Z, int B, const float* C, float* F, bool compact = false);
int64_t gcn_wimg_bytes(const Dims& d);
void launch_gcn_wsplit(hipStream_t s, const Dims& d, const float* gcn, const GcnWOff& wo, char* img);
// dedup: the B windows of every task start at consecutive stream rows (xtab[z*B + b] = xtab[z*B] + b
// time steps) and there is no GCN dropout -- see k_gcn_mlp
void launch_gcn_mlp(hipStream_t s, const Dims& d, int Zb, int B, const float* const* xtab, const float* gcn,
                    const GcnWOff& wo, const char* img, float* F, const Drop* drop, bool dedup = false,
                    bool compact = false);
// out[z] = layer-0 input projection of every distinct stream row of task z's consecutive windows
// (XgDedup layout) with the gate weights W_ih0 of `params` (theta or the tangent direction U); the
// weights come from the pre-split images `img` when given (w.gimg.th / .u), else from `params`; F is
// read in XgDedup order when w.fcompact, else at each stream row's (window, step) slot
void launch_xg_dedup(hipStream_t s, const Dims& d, const Work& w, const float* params, int64_t tstride,
                     const ParamOff& po, const char* img, int64_t img_tstride, int64_t img_off, float* out);
// chunk / nch: row chunks as in launch_lstm_bwd_wave (nch > 1: every diagonal on the big tiles)
void launch_lstm_fwd_wave(hipStream_t s, const Dims& d, const Work& w, int diag, const float* theta,
                          int64_t tstride, const ParamOff& po, double* flops, int chunk = 0, int nch = 1);
void launch_head_loss(hipStream_t s, const Dims& d, const Work& w, const float* theta, int64_t tstride,
                      const ParamOff& po, const float* const* xtab, float dscale, bool want_loss);
void launch_head_loss_y(hipStream_t s, const Dims& d, const Work& w, const float* hT, const float* theta,
                        const ParamOff& po, const float* const* ytab, float* pred, float* dpred, float dscale);
void launch_loss_final(hipStream_t s, const Work& w, float inv_count, float* out);
#ifndef SMAML_HEAD_SMALL_M
#define SMAML_HEAD_SMALL_M 2048  // rows per task up to which the head runs as a SIMT kernel
#endif
#define SMAML_HEAD_MAX_H 128  // (SIMT head: H <= this, H * 8 threads per weight-gradient workgroup)
bool head_small(const Dims& d, int M);
int head_lblocks(const Dims& d, int M);  // loss partials per task written by the head launch
// head weight gradient (dWo, dbo) for head_small() sizes; overwrites
// theta != null: the same launch also writes the top layer's dh_T = dpred . Wo into w.dH (no LSTM dropout)
void launch_head_wgrad_small(hipStream_t s, const Dims& d, const Work& w, const float* dpred, const float* hT,
                             int64_t hz, float* grad, int64_t P, int64_t wo, int64_t bo, const float* theta,
                             int64_t tstride);
// dst[z] = drop(src[z]) with the head-input mask ([M][H] rows per task; src == dst allowed)
void launch_drop_rows(hipStream_t s, const Work& w, int H, const float* src, int64_t src_zstride, float* dst);
// x[i] = drop(x[i]) in place with the GCN-output masks (kind 1, `layer`, step 0, task 0, sample 0):
// STGCN.forward's train-mode dropout after conv layer+1 of one sample (model.py:33-42)
void launch_dropout_inplace(hipStream_t s, float* x, int64_t n, float p, uint32_t seed, int layer);
// rows the head reads: h_T (or R h_T) of the top layer, or their dropout-masked copies
const float* head_input(const Dims& d, const Work& w, bool tangent, int64_t* zstride);
void launch_head_dh(hipStream_t s, const Dims& d, const Work& w, const float* theta, int64_t tstride,
                    const ParamOff& po);
// chunk / nch: the launch covers row tiles [chunk ntm / nch, (chunk + 1) ntm / nch) of every problem on the
// big tiles whatever the size (the BPTT of a row touches only that row's slabs, so row chunks on separate
// streams are independent -- as long as EVERY diagonal is chunked the same way)
void launch_lstm_bwd_wave(hipStream_t s, const Dims& d, const Work& w, int e, const float* theta, int64_t tstride,
                          const ParamOff& po, int chunk = 0, int nch = 1);
// the unchunked launch of diagonal e would run the big tiles (primal / tangent BPTT)
bool bwd_wave_big(const Dims& d, const Work& w, const ParamOff& po, int e);
bool bwd_dual_wave_big(const Dims& d, const Work& w, const ParamOff& po, int e);
// kernels_small.hip: the small-grid (batch-1) forward / BPTT diagonal as one launch with the K
// reduction split over the waves of a workgroup (used where the split-K pair would run)
bool small_kw_ok(const Dims& d, const Work& w);
// launch_lstm_fwd_wave runs diagonal `diag` as the kw kernel (the only forward form that reads w.xg)
bool fwd_wave_kw(const Dims& d, const Work& w, const ParamOff& po, int diag);
// ... as the big-tile k_lstm_fwd_step (the only primal form that reads w.xgd)
bool fwd_wave_big(const Dims& d, const Work& w, const ParamOff& po, int diag);
int64_t bwd_img_bytes(const Dims& d, BwdImgs* bi);  // per task; fills bi's offsets / tstride
void launch_split_bwd(hipStream_t s, const Dims& d, const ParamOff& po, const float* theta, int64_t tstride, int Z,
                      const BwdImgs& bi);
void launch_lstm_fwd_kw(hipStream_t s, const Dims& d, const Work& w, int diag, const float* theta, int64_t tstride,
                        const ParamOff& po);
void launch_lstm_bwd_kw(hipStream_t s, const Dims& d, const Work& w, int e, const float* theta, int64_t tstride,
                        const ParamOff& po);
void launch_wgrad(hipStream_t s, const Dims& d, const Work& w, const float* A, int64_t a_zstride,
                  int Mrows, const float* B1, int64_t b1_zstride, int c1, const float* B2,
                  int64_t b2_zstride, int c2, int64_t K, int Mshift, float* grad, int64_t P,
                  int64_t off_w1, int64_t off_w2, int64_t off_b1, int64_t off_b2, bool with_bias = true,
                  bool accumulate = false);
// B-row gather of layer 0's input-weight gradient over distinct stream rows (WgBGather): M > 0 = on
struct WgGather {
  int M = 0, N = 0, T = 0;
  FastDiv ndiv{};
  int compact = 0;  // F is compact (Work::fcompact): row k is F's row k
};
// launch_wgrad split in its two launches (the GEMM into split-K partial slabs, then the
// fixed-order reduce into the flat gradient), so each can be timed on its own.
struct WgradPlan {
  const float* A = nullptr;
  int64_t a_zstride = 0;
  int Mrows = 0;
  const float *B1 = nullptr, *B2 = nullptr;
  int c1 = 0, c2 = 0;
  int64_t K = 0, Mshift = 0;
  int64_t b1_zstride = 0, b2_zstride = 0;
  float* grad = nullptr;
  int64_t P = 0, off_w1 = -1, off_w2 = -1, off_b1 = -1, off_b2 = -1;
  bool with_bias = false, accumulate = false;
  int Z = 0;
  float* part = nullptr;
  int ldp = 0, ntm = 0, ntn = 0, nsplit = 0;
  int64_t kchunk = 0;
  Drop drop{};          // B1 = drop(h_{drop_layer}) when drop_layer >= 0 and LSTM dropout is on
  int drop_layer = -1;  // (defaults: no dropout -- launch_wgrad's callers never set these)
  bool wide = false;    // 256 x 256 tiles (CfgTW) instead of 512 x 128 (kernels.hip plan_wgrad)
  // pair (pair_wgrad): slices [nsplit1, nsplit) sum A2^T [B1s | B2s] (same shape and strides) into
  // the same gradient; A2 == nullptr: one problem
  const float* A2 = nullptr;
  const float *B1s = nullptr, *B2s = nullptr;
  int nsplit1 = 0;
  WgGather gather{};  // M > 0: B1 rows through XgDedup's compact-row -> F-row map (no B2, no dropout)
};
// Turn a planned weight gradient into a pair with a second problem of the same shape (each problem
// gets about half of the planned slices; one launch, one reduce, no accumulate pass). Returns false
// (plan unchanged) when the pair's slices would not fit the partial-slab buffer w.wpart.
bool pair_wgrad(WgradPlan& p, const Work& w, const float* A2, const float* B1s, const float* B2s);
void plan_wgrad(const Work& w, const float* A, int64_t a_zstride, int Mrows, const float* B1, int64_t b1_zstride,
                int c1, const float* B2, int64_t b2_zstride, int c2, int64_t K, int Mshift, float* grad, int64_t P,
                int64_t off_w1, int64_t off_w2, int64_t off_b1, int64_t off_b2, bool with_bias, bool accumulate,
                WgradPlan& p, bool multi = false);
// Several plans (same Z) in one GEMM launch + one reduce launch; their nsplit / kchunk / part are
// re-planned for about target_wgs workgroups in total (partial slabs must fit w.wpart).
struct WgMulti {
  int n = 0;
  int blk[MAX_LAYERS] = {}, rblk[MAX_LAYERS] = {};
  WgradPlan p[MAX_LAYERS] = {};
};
void launch_wgrad_multi(hipStream_t s, const Work& w, WgradPlan* ps, int n, int target_wgs);
void launch_wgrad_gemm(hipStream_t s, const WgradPlan& p);
// S[z] = row sums of layer 0's dG slab (dG0 = [T][M][4H] per task, a_zstride floats apart) over the
// (window, step) slots of each distinct stream row, in XgDedup's row order ([(2B + T - 2) N][4H] per task)
void launch_dg_rowsum(hipStream_t s, const Dims& d, const Work& w, const float* dG0, int64_t a_zstride, float* S);
void launch_wgrad_reduce(hipStream_t s, const WgradPlan& p);
// clip_grad_norm_ + SGD of every task as one grid-barrier kernel (k_inner_sgd), or its two phases as
// two launches (BarPlan)
hipError_t launch_inner_sgd(hipStream_t s, float* theta, const float* g, int64_t P, int Z, double* part, float lr,
                            float max_norm, float* norm_out, float* coef_out, const BarPlan& bp);
// second-order sweep bookkeeping as one grid-barrier kernel (k_sweep_update): v += alpha x (x may be
// null), U = clip-adjusted direction of (G, norms, coefs) at v
hipError_t launch_sweep_update(hipStream_t s, float* V, const float* X, float alpha, const float* G, int64_t P, int Z,
                               double* part, const float* norms, const float* coefs, float max_norm, float* U,
                               const BarPlan& bp);
// ---- GCNConv backward helpers (module API autograd; kernels.hip) ----
// out[r] = sum_adj w * src[col] for r < n_gather (ELL when csr_p is null, else CSR), src[r] otherwise
void launch_gather_rows(hipStream_t s, const float* src, float* out, int rows, int cols, int n_gather, const int* ell_c,
                        const float* ell_v, const int* csr_p, const int* csr_c, const float* csr_v);
void launch_relu_mask(hipStream_t s, float* g, const float* h, int64_t n);  // g *= (h > 0)
void launch_gemm_nn_plain(hipStream_t s, const float* A, int rows, int K, const float* W, int ncols, float* out);
// out[z] = A[z] . W[z]^T (both K-contiguous), Z problems with the given element strides
void launch_gemm_nt(hipStream_t s, const float* A, int64_t a_zstride, int rows, int K, const float* W,
                    int64_t w_zstride, int ncols, float* out, int64_t o_zstride, int Z);
void launch_sum_tasks(hipStream_t s, const float* g, int64_t P, int Z, float* out);
void launch_broadcast(hipStream_t s, const float* theta, int64_t P, int Z, float* out);
void launch_adamw(hipStream_t s, float* p, const float* g, float* m, float* v, int64_t n, double* part,
                  float lr, float b1, float b2, float eps, float wd, float step_size, float bc2_sqrt,
                  float max_norm, float* norm_out);

// loss != null: block 0 also writes the step's loss from the head's partials (launch_loss_final's sum)
void launch_adam_l2(hipStream_t s, float* p, const float* g, float* m, float* v, int64_t n, double* part,
                    const float* lr_dev, int step, float b1, float b2, float eps, float wd, float max_norm,
                    const float* lpart, int lblocks, float inv_count, float* loss);

// ---- second-order launchers (kernels_dual.hip) ----
void launch_lstm_fwd_dual_wave(hipStream_t s, const Dims& d, const Work& w, int diag, const float* theta,
                               const float* U, int64_t tstride, const ParamOff& po, double* flops, int chunk = 0,
                               int nch = 1);
void launch_head_dual(hipStream_t s, const Dims& d, const Work& w, const float* theta, const float* U,
                      int64_t tstride, const ParamOff& po, const float* const* xtab, float dscale);
void launch_head_dh_dual(hipStream_t s, const Dims& d, const Work& w, const float* theta, const float* U,
                         int64_t tstride, const ParamOff& po);
void launch_lstm_bwd_dual_wave(hipStream_t s, const Dims& d, const Work& w, int e, const float* theta,
                               const float* U, int64_t tstride, const ParamOff& po, int chunk = 0, int nch = 1);
void launch_axpy(hipStream_t s, float* V, const float* X, int64_t n, float alpha);

}  // namespace smaml
