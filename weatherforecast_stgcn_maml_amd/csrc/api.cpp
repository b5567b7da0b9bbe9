// C ABI (include/smaml.h) and the host-side driver of the STGCN-LSTM MAML hot path.
//
// The inner loop (train_hybrid_maml_v5.py:110-141) and the meta-step
// (train_hybrid_maml_v5.py:144-184) run here in C++: Python calls one entry point per
// meta-step and never sees an inner step. Everything for all tasks of the meta-batch
// is batched into each launch (blockIdx.z = task, per-task fast weights).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <dlfcn.h>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "kernels.h"
#include "smaml.h"

using namespace smaml;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(x)                                                                              \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) return fail(SMAML_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define TRY(x)                \
  do {                        \
    int r_ = (x);             \
    if (r_ != SMAML_OK) return r_; \
  } while (0)

constexpr int64_t PAD = 64;  // floats: every tensor offset is 256-B aligned

int64_t pad_up(int64_t x) { return (x + PAD - 1) / PAD * PAD; }

struct Spec {
  int64_t off, size;
};

int check_dims(const smaml_dims* d) {
  if (!d) return fail(SMAML_EINVAL, "dims is NULL");
  if (d->num_nodes <= 0 || d->window_size <= 0 || d->lstm_num_layers <= 0 ||
      d->lstm_num_layers > MAX_LAYERS || d->forecast_horizon <= 0 || d->output_channels <= 0)
    return fail(SMAML_EINVAL, "non-positive dimension");
  if (d->input_channels % 4 || d->hidden_channels % 4)
    return fail(SMAML_EINVAL, "input/hidden channels must be multiples of 4");
  if (d->lstm_hidden_size != 32 && d->lstm_hidden_size != 64 && d->lstm_hidden_size != 128 &&
      d->lstm_hidden_size != 256)
    return fail(SMAML_EINVAL, "lstm_hidden_size must be 32, 64, 128 or 256");
  if (d->forecast_horizon * d->output_channels > 128)
    return fail(SMAML_EINVAL, "forecast_horizon*output_channels must be <= 128");
  if (d->output_channels > d->input_channels)
    return fail(SMAML_EINVAL, "output_channels must not exceed input_channels (targets come from inputs)");
  return SMAML_OK;
}

void layout(const smaml_dims& d, int which, std::vector<Spec>& specs, int64_t& total) {
  specs.clear();
  int64_t off = 0;
  auto add = [&](int64_t n) {
    specs.push_back({off, n});
    off = pad_up(off + n);
  };
  const int64_t H = d.lstm_hidden_size, G = 4 * H;
  if (which == 0) {
    for (int l = 0; l < d.lstm_num_layers; ++l) {
      const int64_t cin = l == 0 ? d.hidden_channels : H;
      add(G * cin);  // weight_ih_l
      add(G * H);    // weight_hh_l
      add(G);        // bias_ih_l
      add(G);        // bias_hh_l
    }
    add((int64_t)d.forecast_horizon * d.output_channels * H);  // output_layer.weight
    add((int64_t)d.forecast_horizon * d.output_channels);      // output_layer.bias
  } else {
    int64_t cin = d.input_channels;
    for (int k = 0; k < 4; ++k) {
      add(d.hidden_channels);        // convK.bias
      add(d.hidden_channels * cin);  // convK.lin.weight
      cin = d.hidden_channels;
    }
  }
  total = off;
}

int build_ell(const int64_t* ei, int64_t E, int N, std::vector<int32_t>& cols, std::vector<float>& vals) {
  cols.assign((size_t)N * ELLW, 0);
  vals.assign((size_t)N * ELLW, 0.f);
  std::vector<float> deg(N, 1.f);  // self loop (add_remaining_self_loops, fill 1)
  const int64_t* src = ei;
  const int64_t* dst = ei + E;
  for (int64_t e = 0; e < E; ++e) {
    if (src[e] < 0 || src[e] >= N || dst[e] < 0 || dst[e] >= N)
      return fail(SMAML_EINVAL, "edge_index references a node outside [0, num_nodes)");
    if (src[e] != dst[e]) deg[dst[e]] += 1.f;
  }
  std::vector<float> dinv(N);
  for (int i = 0; i < N; ++i) dinv[i] = 1.f / std::sqrt(deg[i]);
  std::vector<int> fill(N, 0);
  for (int64_t e = 0; e < E; ++e) {
    const int64_t s = src[e], t = dst[e];
    if (s == t) continue;
    if (fill[t] >= ELLW - 1) return fail(SMAML_EINVAL, "node in-degree exceeds the ELL width (7)");
    cols[(size_t)t * ELLW + fill[t]] = (int32_t)s;
    vals[(size_t)t * ELLW + fill[t]] = dinv[s] * dinv[t];
    ++fill[t];
  }
  for (int i = 0; i < N; ++i) {
    for (int j = fill[i]; j < ELLW; ++j) cols[(size_t)i * ELLW + j] = i;
    vals[(size_t)i * ELLW + fill[i]] = dinv[i] * dinv[i];
  }
  return SMAML_OK;
}

// one kernel per timing category (bench roofline = one kernel's launches)
// (the *_WALL categories: the wall time of a sweep whose diagonals ran as concurrent row chunks on side
// streams -- events on the caller's stream around the fork / join -- beside the per-chunk kernel times)
enum Cat { C_GCN = 0, C_FWD, C_FWD_DUAL, C_HEAD, C_HEAD_DH, C_BWD, C_BWD_DUAL, C_WGRAD, C_WGRAD_RED, C_MISC, C_XG, C_DGSUM,
           C_FWD_WALL, C_FWD_DUAL_WALL, C_BWD_WALL, C_BWD_DUAL_WALL, NCAT };

// Live per-category kernel timing with HIP events on the launch stream (bench roofline).
struct Timer {
  bool on = false;
  struct Rec {
    int cat;
    hipEvent_t a, b;
    double flops;
  };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  double ms[NCAT] = {};
  double flops[NCAT] = {};
  int64_t count[NCAT] = {};
  hipEvent_t get() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
};

// Pinned host staging ring for small host -> device uploads (window pointer tables, task ids):
// each upload takes the next slot, waits only for that slot's previous copy (event), then issues
// an async copy on the caller's stream -- no stream drain, the queue keeps running.
struct Staging {
  static constexpr int NSLOT = 4;
  char* host[NSLOT] = {};
  hipEvent_t evt[NSLOT] = {};
  int64_t cap = 0;  // bytes per slot
  int next = 0;
  int upload(hipStream_t s, void* dev, const void* src, int64_t bytes) {
    if (bytes > cap) {
      TRY(release());
      const int64_t c = std::max<int64_t>(bytes, 8192);
      for (int i = 0; i < NSLOT; ++i) {
        HIP_TRY(hipHostMalloc((void**)&host[i], c, hipHostMallocDefault));
        HIP_TRY(hipEventCreateWithFlags(&evt[i], hipEventDisableTiming));
      }
      cap = c;
    }
    const int i = next;
    next = (next + 1) % NSLOT;
    HIP_TRY(hipEventSynchronize(evt[i]));  // this slot's previous copy has been consumed
    std::memcpy(host[i], src, bytes);
    HIP_TRY(hipMemcpyAsync(dev, host[i], bytes, hipMemcpyHostToDevice, s));
    HIP_TRY(hipEventRecord(evt[i], s));
    return SMAML_OK;
  }
  int release() {
    for (int i = 0; i < NSLOT; ++i) {
      if (evt[i]) {
        HIP_TRY(hipEventSynchronize(evt[i]));
        HIP_TRY(hipEventDestroy(evt[i]));
      }
      if (host[i]) HIP_TRY(hipHostFree(host[i]));
      evt[i] = nullptr;
      host[i] = nullptr;
    }
    cap = 0;
    return SMAML_OK;
  }
};

}  // namespace

// The build-time defaults of the run-time knobs, by name (kernels.h Knobs; smaml_set_option changes them).
static Knobs default_knobs() {
  Knobs k;
  k.bwd_big_min = SMAML_BWD_BIG_MIN;
  k.bwdd_big_min = SMAML_BWDD_BIG_MIN;
  k.split_max = SMAML_SPLIT_MAX;
  k.wgrad_group_max_rows = SMAML_WGRAD_GROUP_ROWS;
  k.wgrad_group_wgs = SMAML_WGRAD_GROUP_WGS;
  k.gcn_fused = SMAML_GCN_FUSED;
  k.gate_img = SMAML_GATE_IMG;
  k.wgrad_wide = 1;
  k.wgrad_pair = SMAML_WGRAD_PAIR;
  k.bwdd_remap = SMAML_BWDD_REMAP_DEFAULT;
  k.small_kw = SMAML_SMALL_KW;
  k.gcn_dedup = 1;
  k.xg_dedup = SMAML_XG_DEDUP_DEFAULT;
  k.wgrad_dedup = SMAML_WGRAD_DEDUP_DEFAULT;
  k.bptt_streams = SMAML_BPTT_STREAMS_DEFAULT;
  k.fwd_streams = SMAML_FWD_STREAMS_DEFAULT;
  k.f_compact = SMAML_F_COMPACT_DEFAULT;
  return k;
}

// Host-timed phases of one smaml_adapt_steps call (smaml_adapt_phases): workspace reserve, feature-cache
// allocation, the batched cache fill, the step loop. The last two are enqueue times unless the option
// adapt_phase_sync is on (then each ends with a stream sync and includes the GPU time).
enum { AD_RESERVE = 0, AD_ALLOC, AD_FILL, AD_STEPS, AD_NPH };
struct AdPhases {
  double ms[AD_NPH] = {};
  int64_t filled = 0;  // windows computed by a per-step GCN pass (not the batched fill)
};

struct smaml_ctx {
  smaml_dims dims{};
  Dims d{};
  ParamOff po{};
  GcnOff go{};
  int device = 0;
  int32_t* ell_c = nullptr;
  float* ell_v = nullptr;
  // A_hat^T as CSR (GCNConv backward's aggregation of the t = 0 rows; built with the ELL)
  int32_t *tr_p = nullptr, *tr_c = nullptr;
  float* tr_v = nullptr;
  int64_t tr_nnz_cap = 0;
  float* bw_scratch = nullptr;  // GCNConv backward: [rows][max(cin, cout)] x 2
  int64_t bw_scratch_cap = 0;
  const float* gcn = nullptr;
  // workspace
  char* arena = nullptr;
  int64_t arena_bytes = 0;
  int zb_cap = 0, z_cap = 0;
  Work w{};
  float* fast = nullptr;
  float* grad = nullptr;
  float* scratch_loss = nullptr;  // [(steps+1)*Z] fallback when the caller passes no buffer
  int64_t scratch_loss_cap = 0;
  // device pointer table for sample windows (uploaded through the pinned staging ring)
  const float** xtab = nullptr;  // never index directly: xtab_at (the table moves when it grows)
  int64_t xtab_cap = 0;
  int64_t xtab_n = 0;  // entries of the last upload_xtab
  Staging stage;
  // kernel-variant launch counters and run-time tile knobs (smaml_variant_counts / smaml_set_option)
  int64_t vcount[NVAR] = {};
  Knobs kn = default_knobs();
  int n_cu = 256;  // compute units of the device (smaml_create)
  int keep_max = -1;  // cap on kept second-order steps (-1: SMAML_KEEP env or all that fit)
  // tasks
  std::vector<const float*> feats;
  std::vector<int> t_total;
  Timer tm;
  // second-order state
  bool so_cap = false;
  float *so_u = nullptr, *so_hu = nullptr;
  float *so_theta = nullptr, *so_grad = nullptr, *so_norm = nullptr, *so_coef = nullptr;
  int64_t so_store_cap = 0, so_nc_cap = 0;
  float* so_F = nullptr;  // [K][Z][T][M][Hc] GCN features of every inner step (null: recompute)
  int64_t so_F_cap = 0;
  std::vector<int8_t> so_fc;  // per inner step: whether run_gcn wrote its so_F slot compact (Work::fcompact)
  float* F_main = nullptr;  // the workspace's own F buffer
  // batch-1 adaptation: GCN features per window of task 0 (the frozen GCN stack without dropout
  // is a pure function of the window, F2), filled on first use and reused by later epochs.
  // Invalidated by smaml_set_graph / _set_gcn_params / _set_tasks.
  char* gcn_wimg = nullptr;   // pre-split GCN weight images of the fused t >= 1 GCN (kernels_gcn.hip)
  char* gimg_buf = nullptr;   // pre-split gate-GEMM weight images (prep_gate_images)
  int64_t gimg_cap = 0;
  char* bimg_buf = nullptr;   // pre-split BPTT weight images (prep_bwd_images; small-grid BPTT)
  int64_t bimg_cap = 0;
  float* xg_buf = nullptr;    // small-grid forward: layer 0's hoisted input projection (run_lstm)
  int64_t xg_cap = 0;
  float* xgd_buf = nullptr;   // big-tile forward: layer 0's projection per distinct stream row (prep_xg_dedup)
  int64_t xgd_cap = 0;
  // grid-barrier state of the bookkeeping kernels (kernels.h GridBar): device words [3], the pinned
  // device-mapped error flag a timed-out waiter sets, the wait bound and the launch form
  unsigned* bar = nullptr;
  int* bar_err_host = nullptr;
  int* bar_err_dev = nullptr;
  int64_t bar_timeout_us = 4000000;  // smaml_set_option("barrier_timeout_us")
  int bar_fused = 1;                 // smaml_set_option("grid_barrier"): 0 = two launches per kernel
  int bar_oversize = 0;              // smaml_set_option("barrier_oversize"): debug, never co-resident
  uint64_t wall_khz = 0;             // wall_clock64 rate
  float* ad_F = nullptr;
  int64_t ad_cap = 0;              // windows the cache holds
  std::vector<uint8_t> ad_valid;   // per window start
  int ad_gcn_batch = 32;           // windows per GCN pass when filling the cache (<= 1: one per step)
  int ad_phase_sync = 0;           // smaml_set_option("adapt_phase_sync"): sync at the phase boundaries
  AdPhases ad_ph;                  // host-timed phases of the last smaml_adapt_steps (smaml_adapt_phases)
  float *Hs_main = nullptr, *Cs_main = nullptr, *Gs_main = nullptr;  // the workspace's own activations
  // primal of the last inner steps kept for the second-order sweep (ensure_keep): slot 0 adds
  // dG + dh to the workspace's Hs/Cs/Gs, slot i >= 1 holds Hs/Cs/Gs/dG/dh of its own
  std::vector<float*> keep_mem;
  int keep_n = 0;
  int64_t keep_rows = 0;  // rows * L the slots were sized for
  int keep_tried_K = -1;
  int keep_want = 0;  // slots the current second-order meta-step may use (<= keep_n)
  int keep_last = 0;  // slots the last second-order meta-step used
  // train-mode dropout (smaml_set_dropout / smaml_set_task_ids); p = 0: off
  float p_gcn = 0.f, p_lstm = 0.f;
  uint32_t drop_seed = 0;
  std::vector<int32_t> task_ids;  // global id of each task of smaml_set_tasks (default: its index)
  int* task_id_dev = nullptr;     // [z_cap] (arena)
  int64_t keep_tried_rows = -1;
  // activations of the last smaml_forward / smaml_lstm_forward (single task, act_B samples);
  // -1 once anything else has used the workspace (the backward consumes them: dG in place)
  int act_B = -1;
  // side streams of the row-chunked BPTT (knob bptt_streams) and their fork / join events
  hipStream_t cs[4] = {};
  hipEvent_t fork_ev = nullptr, join_ev[4] = {};
  // RCCL communicator (smaml_comm_init), opaque; created non-blocking when the library allows it
  void* comm = nullptr;
  int comm_nb = 0;
  int64_t comm_timeout_ms = 120000;  // smaml_set_option("comm_timeout_ms")
};

namespace {

int ensure_device(smaml_ctx* c) {
  HIP_TRY(hipSetDevice(c->device));
  return SMAML_OK;
}

int free_keep(smaml_ctx* c) {
  if (c->keep_mem.empty()) return SMAML_OK;
  HIP_TRY(hipDeviceSynchronize());
  for (float* p : c->keep_mem) HIP_TRY(hipFree(p));
  c->keep_mem.clear();
  c->keep_n = 0;
  c->keep_rows = 0;
  c->keep_tried_K = -1;
  c->keep_tried_rows = -1;
  return SMAML_OK;
}

static void ad_cache_drop(smaml_ctx* c);

int reserve(smaml_ctx* c, int Z, int B, bool so = false) {
  const int zb = Z * B;
  // per-task activation slabs are addressed with 32-bit offsets inside the kernels
  if ((int64_t)c->d.T * B * c->d.N * 4 * c->d.H >= (1ll << 31))
    return fail(SMAML_EINVAL, "batch too large: T*B*N*4H must stay below 2^31 per task");
  so = so || c->so_cap;
  if (zb <= c->zb_cap && Z <= c->z_cap && so == c->so_cap) return SMAML_OK;
  ad_cache_drop(c);  // a growing workspace takes precedence over the adaptation feature cache
  const int zbc = std::max(zb, c->zb_cap), zc = std::max(Z, c->z_cap);
  const Dims& d = c->d;
  const int64_t rows = (int64_t)zbc * d.T * d.N;
  const int64_t G = 4 * d.H;
  const int64_t seq = (int64_t)zbc * d.N;
  int max_cin = std::max(d.Hc, d.H);
  const int64_t wpart = std::max<int64_t>((int64_t)zc * G * (max_cin + d.H + 1) * SMAML_WGRAD_MAXSPLIT, 1 << 24);
  // loss partials per task: head_lblocks(M) for every per-task row count M <= seq
  const int64_t lblk =
      (int64_t)zc * (std::max<int64_t>(head_lblocks(d, (int)std::min<int64_t>(seq, SMAML_HEAD_SMALL_M)),
                                       (seq + 127) / 128) + 1);
  std::vector<std::pair<void**, int64_t>> parts;  // (dst, bytes)
  Work w{};
  parts.push_back({(void**)&w.F, rows * d.Hc * 4});
  parts.push_back({(void**)&w.Hs, rows * d.L * d.H * 4});
  parts.push_back({(void**)&w.Cs, rows * d.L * d.H * 4});
  parts.push_back({(void**)&w.Gs, rows * d.L * G * 4});  // gates, then dG in place (BPTT)
  parts.push_back({(void**)&w.dH, seq * d.H * 4});
  parts.push_back({(void**)&w.dc, seq * d.L * d.H * 4});
  parts.push_back({(void**)&w.gcnA, rows * d.Hc * 4});
  parts.push_back({(void**)&w.gcnB, rows * d.Hc * 4});
  parts.push_back({(void**)&w.pred, seq * d.HfC * 4});
  parts.push_back({(void**)&w.dpred, seq * d.HfC * 4});
  parts.push_back({(void**)&w.wpart, wpart * 4});
  parts.push_back({(void**)&w.lpart, lblk * 4});
  parts.push_back({(void**)&w.sqpart, (int64_t)(zc + 1) * SQB * 8});
  parts.push_back({(void**)&w.hTd, seq * d.H * 4});
  int* task_id_dev = nullptr;
  parts.push_back({(void**)&task_id_dev, (int64_t)zc * 4});
  float *fast = nullptr, *grad = nullptr;
  parts.push_back({(void**)&fast, (int64_t)zc * c->po.P * 4});
  parts.push_back({(void**)&grad, (int64_t)zc * c->po.P * 4});
  float *so_u = nullptr, *so_hu = nullptr;
  if (so) {
    parts.push_back({(void**)&w.RHs, rows * d.L * d.H * 4});
    parts.push_back({(void**)&w.RCs, rows * d.L * d.H * 4});
    parts.push_back({(void**)&w.RGs, rows * d.L * G * 4});
    parts.push_back({(void**)&w.RdH, seq * d.H * 4});
    parts.push_back({(void**)&w.Rdc, seq * d.L * d.H * 4});
    parts.push_back({(void**)&w.Rdpred, seq * d.HfC * 4});
    parts.push_back({(void**)&w.RhTd, seq * d.H * 4});
    parts.push_back({(void**)&so_u, (int64_t)zc * c->po.P * 4});
    parts.push_back({(void**)&so_hu, (int64_t)zc * c->po.P * 4});
  }
  int64_t total = 0;
  for (auto& p : parts) total += (p.second + 255) / 256 * 256;
  c->act_B = -1;
  TRY(free_keep(c));
  if (c->arena) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipFree(c->arena));
    c->arena = nullptr;
    c->arena_bytes = 0;
  }
  char* arena = nullptr;
  if (hipMalloc((void**)&arena, total) != hipSuccess) {
    (void)hipGetLastError();
    return fail(SMAML_ENOMEM, "hipMalloc of " + std::to_string(total) + " B workspace failed");
  }
  int64_t off = 0;
  for (auto& p : parts) {
    *p.first = arena + off;
    off += (p.second + 255) / 256 * 256;
  }
  w.wpart_floats = wpart;
  HIP_TRY(hipMemset(grad, 0, (size_t)zc * c->po.P * 4));
  HIP_TRY(hipMemset(fast, 0, (size_t)zc * c->po.P * 4));
  c->arena = arena;
  c->arena_bytes = total;
  c->w = w;
  c->task_id_dev = task_id_dev;
  c->fast = fast;
  c->grad = grad;
  c->zb_cap = zbc;
  c->z_cap = zc;
  c->so_cap = so;
  c->F_main = w.F;
  c->Hs_main = w.Hs;
  c->Cs_main = w.Cs;
  c->Gs_main = w.Gs;
  c->w.dG = w.Gs;
  c->so_u = so_u;
  c->so_hu = so_hu;
  if (so_hu) HIP_TRY(hipMemset(so_hu, 0, (size_t)zc * c->po.P * 4));
  return SMAML_OK;
}

// Per-step stores of the second-order sweep: theta_k and g_k [K][Z][P], |g_k| and the
// clip coefficient [K][Z].
int ensure_so_store(smaml_ctx* c, int K, int Z, int B) {
  // GCN features of each inner step, kept for the second-order sweep (weight-independent, F2).
  // Best effort: without room the sweep recomputes them.
  const int64_t fneed = (int64_t)K * Z * B * c->d.T * c->d.N * c->d.Hc;
  if (fneed > c->so_F_cap) {
    if (c->so_F) {
      HIP_TRY(hipDeviceSynchronize());
      HIP_TRY(hipFree(c->so_F));
      c->so_F = nullptr;
      c->so_F_cap = 0;
    }
    size_t freeb = 0, totb = 0;
    HIP_TRY(hipMemGetInfo(&freeb, &totb));
    if ((int64_t)freeb > fneed * 4 + (4ll << 30) && hipMalloc((void**)&c->so_F, fneed * 4) == hipSuccess) {
      c->so_F_cap = fneed;
    } else {
      (void)hipGetLastError();
      c->so_F = nullptr;
    }
  }
  const int64_t need = (int64_t)K * Z * c->po.P;
  if (need <= c->so_store_cap && (int64_t)K * Z <= c->so_nc_cap) return SMAML_OK;
  if (c->so_theta) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipFree(c->so_theta));
    HIP_TRY(hipFree(c->so_grad));
    HIP_TRY(hipFree(c->so_norm));
    HIP_TRY(hipFree(c->so_coef));
  }
  HIP_TRY(hipMalloc((void**)&c->so_theta, need * 4));
  HIP_TRY(hipMalloc((void**)&c->so_grad, need * 4));
  HIP_TRY(hipMalloc((void**)&c->so_norm, (int64_t)K * Z * 4));
  HIP_TRY(hipMalloc((void**)&c->so_coef, (int64_t)K * Z * 4));
  c->so_store_cap = need;
  c->so_nc_cap = (int64_t)K * Z;
  return SMAML_OK;
}

// Primal activations of the last inner steps, kept for the second-order sweep so that its
// dual kernels run tangent-only for those steps (no primal recompute of the forward or the
// BPTT GEMMs). Slot 0 (step K-1) keeps the workspace's own Hs/Cs/Gs -- the query then runs in
// the tangent buffers -- and adds dG + dh; slot i >= 1 (step K-1-i) holds its own
// Hs/Cs/Gs/dG/dh. Best effort: as many slots as fit in free HBM with a margin, capped by the
// SMAML_KEEP environment variable (0 disables). Needs the GCN feature cache (so_F).
int ensure_keep(smaml_ctx* c, int K, int Z, int B) {
  const Dims& d = c->d;
  int want = c->so_F ? K : 0;
  if (c->keep_max >= 0)
    want = std::min(want, c->keep_max);
  else if (const char* e = std::getenv("SMAML_KEEP"))
    want = std::min(want, std::max(0, std::atoi(e)));
  const int64_t rowsL = (int64_t)Z * B * d.T * d.N * d.L;
  c->keep_want = want;
  if (want <= c->keep_n && rowsL <= c->keep_rows) return SMAML_OK;
  // already as many as fit for a group at least this large: keep those slots (unequal task groups, e.g.
  // 8 + 7, would otherwise free and re-allocate every slot at every group change, seconds per meta-step)
  if (rowsL <= c->keep_rows && want <= c->keep_tried_K && rowsL <= c->keep_tried_rows) return SMAML_OK;
  TRY(free_keep(c));
  c->keep_tried_K = want;
  c->keep_tried_rows = rowsL;
  const int64_t margin = 8ll << 30;
  for (int i = 0; i < want; ++i) {
    const int64_t bytes = rowsL * (i == 0 ? 5 : 11) * d.H * 4;  // [dG | dh] or [Hs | Cs | Gs | dG | dh]
    size_t freeb = 0, totb = 0;
    HIP_TRY(hipMemGetInfo(&freeb, &totb));
    float* p = nullptr;
    if ((int64_t)freeb < bytes + margin || hipMalloc((void**)&p, bytes) != hipSuccess) {
      (void)hipGetLastError();
      break;
    }
    c->keep_mem.push_back(p);
  }
  c->keep_n = (int)c->keep_mem.size();
  c->keep_rows = rowsL;
  return SMAML_OK;
}

// Points the workspace's primal activation buffers at the workspace's own (slot < 0), at a
// kept slot, or (query, when slot 0 holds the workspace's own) at the tangent buffers.
enum { SET_MAIN = -1, SET_QUERY = -2 };
void use_primal(smaml_ctx* c, int slot) {
  Work& w = c->w;
  const int64_t rowsL = (int64_t)w.Z * w.B * c->d.T * c->d.N * c->d.L;
  const int64_t H = c->d.H;
  w.dh = nullptr;
  if (slot == SET_QUERY) {
    w.Hs = w.RHs;
    w.Cs = w.RCs;
    w.Gs = w.dG = w.RGs;
  } else if (slot < 0) {
    w.Hs = c->Hs_main;
    w.Cs = c->Cs_main;
    w.Gs = w.dG = c->Gs_main;
  } else if (slot == 0) {
    w.Hs = c->Hs_main;
    w.Cs = c->Cs_main;
    w.Gs = c->Gs_main;
    w.dG = c->keep_mem[0];
    w.dh = c->keep_mem[0] + rowsL * 4 * H;
  } else {
    float* p = c->keep_mem[slot];
    w.Hs = p;
    w.Cs = p + rowsL * H;
    w.Gs = p + rowsL * 2 * H;
    w.dG = p + rowsL * 6 * H;
    w.dh = p + rowsL * 10 * H;
  }
}

// Dropout masks of one forward pass (inner step / query `step`) for the Z tasks of the workspace.
int upload_task_ids(smaml_ctx* c, hipStream_t s, int Z) {
  std::vector<int32_t> ids(Z);
  for (int z = 0; z < Z; ++z) ids[z] = z < (int)c->task_ids.size() ? c->task_ids[z] : z;
  return c->stage.upload(s, c->task_id_dev, ids.data(), (int64_t)Z * 4);  // pinned ring: no stream drain
}

void set_step_drop(smaml_ctx* c, int step) {
  Drop dr{};
  auto thr = [](float p) { return (uint32_t)std::min<double>(std::llround((double)p * 16777216.0), 16777216.0); };
  dr.seed = c->drop_seed;
  dr.step = step;
  dr.thr_gcn = thr(c->p_gcn);
  dr.thr_lstm = thr(c->p_lstm);
  dr.sc_gcn = 1.f / (1.f - c->p_gcn);
  dr.sc_lstm = 1.f / (1.f - c->p_lstm);
  dr.task_id = c->task_id_dev;
  c->w.drop = dr;
}

int ensure_xtab(smaml_ctx* c, int64_t n) {
  if (n <= c->xtab_cap) return SMAML_OK;
  if (c->xtab) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipFree((void*)c->xtab));
  }
  const int64_t cap = std::max<int64_t>(n, 1024);
  c->xtab_n = 0;
  HIP_TRY(hipMalloc((void**)&c->xtab, cap * sizeof(float*)));
  c->xtab_cap = cap;
  return SMAML_OK;
}

int upload_xtab(smaml_ctx* c, hipStream_t s, const float* const* ptrs, int64_t n) {
  TRY(ensure_xtab(c, n));
  c->xtab_n = 0;
  TRY(c->stage.upload(s, (void*)c->xtab, ptrs, n * (int64_t)sizeof(float*)));
  c->xtab_n = n;
  return SMAML_OK;
}

// Device address of entry i of the window table. The only way table pointers are formed: after the
// upload_xtab that wrote entry i (ensure_xtab may move the table, so a pointer taken before an upload
// could dangle -- the fault class of round 4's first gcn_dedup run).
int xtab_at(const smaml_ctx* c, int64_t i, const float* const** out) {
  if (!c->xtab || i < 0 || i >= c->xtab_n)
    return fail(SMAML_EINVAL, "internal: window-table entry " + std::to_string(i) + " read before its upload (" +
                                  std::to_string(c->xtab_n) + " uploaded)");
  *out = c->xtab + i;
  return SMAML_OK;
}

void set_work(smaml_ctx* c, int Z, int B) {
  c->act_B = -1;  // any new use of the workspace ends the validity of saved activations
  c->w.Z = Z;
  c->w.B = B;
  c->w.M = B * c->d.N;
  c->w.lblocks = head_lblocks(c->d, c->w.M);
  c->w.F = c->F_main;
  c->w.primal_kept = 0;
  c->w.consec = 0;
  c->w.fcompact = 0;
  c->w.drop = Drop{};  // dropout only inside smaml_meta_step / smaml_adapt_steps (set_step_drop)
  c->w.vcount = c->vcount;
  c->w.kn = c->kn;
  if (c->Hs_main) use_primal(c, SET_MAIN);
}

#define TIMED(c, s, cat, fl, stmt)                              \
  do {                                                           \
    if ((c)->tm.on) {                                            \
      hipEvent_t a_ = (c)->tm.get(), b_ = (c)->tm.get();         \
      (void)hipEventRecord(a_, s);                               \
      stmt;                                                      \
      (void)hipEventRecord(b_, s);                               \
      (c)->tm.recs.push_back({cat, a_, b_, (double)(fl)});       \
    } else {                                                     \
      stmt;                                                      \
    }                                                            \
  } while (0)

// Weight gradient = split-K GEMM (C_WGRAD) + fixed-order reduce (C_WGRAD_RED).
int fork_streams(smaml_ctx* c, hipStream_t s, int n);

// One weight gradient's split-K GEMM + reduce, in order on s.
void wgrad_run(smaml_ctx* c, hipStream_t s, double fl, WgradPlan& p) {
  TIMED(c, s, C_WGRAD, fl, launch_wgrad_gemm(s, p));
  TIMED(c, s, C_WGRAD_RED, 0, launch_wgrad_reduce(s, p));
}

void timed_wgrad(smaml_ctx* c, hipStream_t s, double fl, const float* A, int64_t a_zstride, int Mrows,
                 const float* B1, int64_t b1_zstride, int c1, const float* B2, int64_t b2_zstride, int c2, int64_t K,
                 int Mshift, float* grad, int64_t P, int64_t off_w1, int64_t off_w2, int64_t off_b1, int64_t off_b2,
                 bool with_bias = true, bool accumulate = false, int drop_layer = -1) {
  WgradPlan p;
  plan_wgrad(c->w, A, a_zstride, Mrows, B1, b1_zstride, c1, B2, b2_zstride, c2, K, Mshift, grad, P, off_w1, off_w2,
             off_b1, off_b2, with_bias, accumulate, p);
  p.drop = c->w.drop;  // B1 = drop(h_{drop_layer}) under LSTM dropout (input weights of layer >= 1)
  p.drop_layer = drop_layer;
  count_variant(c->w, V_WGRAD);
  if (p.wide) count_variant(c->w, V_WGRAD_WIDE);
  wgrad_run(c, s, fl, p);
}

// Tangent weight gradient of one LSTM layer as ONE split-K launch + ONE reduce:
//   R(dW) = R(dG)^T [x | h_{t-1}] + dG^T [Rx | Rh_{t-1}]   (both problems 4H x (cin + H)).
bool timed_wgrad_pair(smaml_ctx* c, hipStream_t s, double fl, const float* RdG, const float* dG, int64_t a_zstride,
                      int Mrows, const float* X, const float* RX, int64_t b1_zstride, int c1, const float* Hh,
                      const float* RHh, int64_t b2_zstride, int c2, int64_t K, int Mshift, float* grad, int64_t P,
                      int64_t off_w1, int64_t off_w2, int64_t off_b1, int64_t off_b2, int drop_layer) {
  WgradPlan p;
  plan_wgrad(c->w, RdG, a_zstride, Mrows, X, b1_zstride, c1, Hh, b2_zstride, c2, K, Mshift, grad, P, off_w1, off_w2,
             off_b1, off_b2, true, false, p);
  if (!pair_wgrad(p, c->w, dG, RX, RHh)) return false;  // the caller runs the two accumulating passes
  p.drop = c->w.drop;
  p.drop_layer = drop_layer;
  count_variant(c->w, V_WGRAD);
  if (p.wide) count_variant(c->w, V_WGRAD_WIDE);
  count_variant(c->w, V_WGRAD_PAIR);
  wgrad_run(c, s, fl, p);
  return true;
}

// Row chunks of a forward sweep (knob fwd_streams; 0 = auto: two when one problem's big-tile gate launch
// fills at most one round of the device's workgroup slots, e.g. config 5's one-task groups, where the
// chunks fill each other's tails; at config 2 a diagonal is ~9 rounds and chunking measured slower).
int fwd_chunks(const smaml_ctx* c) {
  const Work& w = c->w;
  // (only where the full diagonal runs the big tiles anyway; every chunked diagonal does)
  if ((int64_t)w.Z * w.M <= c->kn.wgrad_group_max_rows || !fwd_wave_big(c->d, w, c->po, std::min(c->d.L, c->d.T) - 1))
    return 1;
  if (c->kn.fwd_streams > 0) return c->kn.fwd_streams;
  const int64_t wgs = (int64_t)(w.M + 255) / 256 * ((c->d.H + 31) / 32) * w.Z;  // 256-row x 32-unit gate tiles
  return wgs <= 2LL * c->n_cu ? 2 : 1;
}

// Side streams for row chunks of the BPTT (knob bptt_streams): each waits for the work already on s.
int fork_streams(smaml_ctx* c, hipStream_t s, int n) {
  if (!c->fork_ev) HIP_TRY(hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(c->fork_ev, s));
  for (int i = 0; i < n; ++i) {
    if (!c->cs[i]) HIP_TRY(hipStreamCreateWithFlags(&c->cs[i], hipStreamNonBlocking));
    if (!c->join_ev[i]) HIP_TRY(hipEventCreateWithFlags(&c->join_ev[i], hipEventDisableTiming));
    HIP_TRY(hipStreamWaitEvent(c->cs[i], c->fork_ev, 0));
  }
  return SMAML_OK;
}
// the workspace as chunk ci's launches see it: launch counters once per diagonal (chunk 0's)
Work chunk_work(const Work& w, int ci) {
  Work q = w;
  if (ci > 0) q.vcount = nullptr;
  return q;
}

// a timing record of category cat from event a (recorded on s before a fork) to now on s (after the join)
void time_wall(smaml_ctx* c, hipStream_t s, hipEvent_t a, int cat, double fl) {
  if (!a) return;
  hipEvent_t b = c->tm.get();
  (void)hipEventRecord(b, s);
  c->tm.recs.push_back({cat, a, b, fl});
}

// s waits for everything issued on the side streams
int join_streams(smaml_ctx* c, hipStream_t s, int n) {
  for (int i = 0; i < n; ++i) {
    HIP_TRY(hipEventRecord(c->join_ev[i], c->cs[i]));
    HIP_TRY(hipStreamWaitEvent(s, c->join_ev[i], 0));
  }
  return SMAML_OK;
}

// The XgDedup-row-order scratch (k_xg_dedup tables / k_dg_rowsum sums) with room for `floats`, or null.
float* xgd_scratch(smaml_ctx* c, int64_t floats) {
  if (floats > c->xgd_cap) {
    if (c->xgd_buf) (void)hipFree(c->xgd_buf);
    c->xgd_buf = nullptr;
    c->xgd_cap = 0;
    if (hipMalloc((void**)&c->xgd_buf, floats * 4) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    c->xgd_cap = floats;
  }
  return c->xgd_buf;
}

// Whether this step's layer-0 input-weight gradient runs over distinct stream rows (wgrad_dedup).
bool wgrad_dedup_ok(const smaml_ctx* c) {
  const Work& w = c->w;
  return w.consec && c->kn.wgrad_dedup && w.B > 1 && !w.drop.gcn() && !w.drop.lstm();
}

// dW_ih0 (or its tangent) = S^T F_rows over the distinct stream rows of the step's consecutive windows:
// S = row sums of dGl (layer 0's dG or R(dG), k_dg_rowsum, in the scratch), then ONE gathered split-K
// GEMM into grad's W_ih0 block (no bias; written, not accumulated). False: no scratch (the caller runs
// the full-row form).
bool timed_wgrad_ih0_dedup(smaml_ctx* c, hipStream_t s, const float* dGl, float* grad) {
  const Dims& d = c->d;
  Work& w = c->w;
  const int64_t rows = xg_dedup_rows(w.B, d.T, d.N), TM = (int64_t)d.T * w.M;
  float* S = xgd_scratch(c, rows * 4 * d.H * w.Z);
  if (!S) return false;
  const LayerOff& lo = c->po.lay[0];
  TIMED(c, s, C_DGSUM, 0, launch_dg_rowsum(s, d, w, dGl, TM * 4 * d.H, S));
  WgradPlan p;
  plan_wgrad(w, S, rows * 4 * d.H, 4 * d.H, w.F, TM * lo.cin, lo.cin, nullptr, 0, 0, rows, 0, grad, c->po.P, lo.wih, -1,
             -1, -1, false, false, p);
  p.gather = WgGather{w.M, d.N, d.T, FastDiv((uint32_t)d.N), w.fcompact};
  count_variant(w, V_WGRAD);
  count_variant(w, V_WGRAD_DEDUP);
  if (p.wide) count_variant(w, V_WGRAD_WIDE);
  wgrad_run(c, s, 2.0 * w.Z * rows * 4 * d.H * lo.cin, p);
  return true;
}

// Whether a consecutive-window step's features may be stored compact (Work::fcompact, the distinct rows
// only, XgDedup order): every reader of F must then take those rows -- the forwards' layer-0 gates through
// the k_xg_dedup tables (every layer-0 diagonal on the big tiles; the tangent forward always reads them),
// the backwards' dW_ih0 through the gathered form (not the grouped small-grid launch) -- with the
// scratch for both tables reserved here, so neither reader can miss it later. Deterministic in the
// step's state; the tangent sweep reuses the flag recorded when a step's so_F slot was written (so_fc).
bool f_compact_ok(smaml_ctx* c, bool consec) {
  const Dims& d = c->d;
  const Work& w = c->w;
  const Knobs& kn = c->kn;
  if (!consec || !kn.f_compact || !kn.gcn_dedup || !kn.xg_dedup || !kn.wgrad_dedup || w.B <= 1 || w.drop.gcn() ||
      w.drop.lstm() || (int64_t)w.Z * w.M <= kn.wgrad_group_max_rows)
    return false;
  for (int diag = 0; diag < d.T; ++diag)
    if (!fwd_wave_big(d, w, c->po, diag)) return false;
  return xgd_scratch(c, 2 * xg_dedup_rows(w.B, d.T, d.N) * 4 * d.H * w.Z) != nullptr;
}

// GCN x4 (no_grad, F2): sample windows -> w.F [Z][T][M][Hc]. With the fused kernel (Hc = 256): the
// rows t >= 1 (no neighbours, F3) run all four convs in one launch (k_gcn_mlp, activations kept in
// registers), the t = 0 rows (ELL gather) four per-layer launches over N-row blocks.
// first_tab (device, [Z]: each task's first window pointer), given when every task's B windows start at
// consecutive stream rows (the caller checked the window table): the rows t >= 1 are then computed
// once per distinct stream row -- by the fused kernel (k_gcn_mlp dedup), or, on the per-layer path,
// as one (B + T - 1) N-row pseudo-sample per task without neighbours, expanded into F afterwards.
int run_gcn(smaml_ctx* c, hipStream_t s, const float* const* xtab_dev, const float* const* first_tab = nullptr) {
  const bool consec = first_tab != nullptr;
  const Dims& d = c->d;
  Work& w = c->w;
  w.fcompact = f_compact_ok(c, consec) ? 1 : 0;
  if (w.fcompact) count_variant(w, V_F_COMPACT);
  const int rps = d.T * d.N;
  const int zb = w.Z * w.B;
  const float* src = nullptr;
  float* bufs[2] = {w.gcnA, w.gcnB};
  if (gcn_mlp_supported(d) && c->kn.gcn_fused) {
    if (!c->gcn_wimg) HIP_TRY(hipMalloc((void**)&c->gcn_wimg, gcn_wimg_bytes(d)));
    GcnWOff wo;
    for (int k = 0; k < 4; ++k) {
      wo.w[k] = c->go.w[k];
      wo.b[k] = c->go.b[k];
    }
    // the GCN parameters may change between calls (smaml_set_gcn_params keeps the pointer): re-split
    TIMED(c, s, C_MISC, 0, launch_gcn_wsplit(s, d, c->gcn, wo, c->gcn_wimg));
    const bool dedup = consec && c->kn.gcn_dedup && w.B > 1 && !w.drop.gcn();
    if (dedup) count_variant(w, V_GCN_DEDUP);
    const double rows1 = dedup ? (double)w.Z * (w.B + d.T - 2) * d.N : (double)zb * (d.T - 1) * d.N;
    TIMED(c, s, C_GCN, 2.0 * rows1 * d.Hc * (d.Cin0 + 3.0 * d.Hc),
          launch_gcn_mlp(s, d, zb, w.B, xtab_dev, c->gcn, wo, c->gcn_wimg, w.F, &w.drop, dedup, w.fcompact));
    for (int k = 0; k < 4; ++k) {  // t = 0 rows: N-row blocks, masks indexed as rows of T*N-row samples
      const bool last = k == 3;
      float* dst = last ? w.F : bufs[k & 1];
      TIMED(c, s, C_GCN, 2.0 * zb * d.N * c->go.cin[k] * d.Hc,
            launch_gcn_layer(s, d, k, zb, w.B, k == 0 ? xtab_dev : nullptr, src, dst, last, true,
                             c->gcn + c->go.w[k], c->gcn + c->go.b[k], c->go.cin[k], d.Hc, c->ell_c, c->ell_v,
                             d.N, d.N, &w.drop, rps));
      src = dst;
    }
    HIP_TRY(hipGetLastError());
    return SMAML_OK;
  }
  if (consec && c->kn.gcn_dedup && w.B > 1 && !w.drop.gcn()) {
    count_variant(w, V_GCN_DEDUP);
    const int rpsC = (w.B + d.T - 1) * d.N;  // stream rows w0 .. w0 + B + T - 2 of each task
    for (int k = 0; k < 4; ++k) {
      float* dst = bufs[k & 1];
      TIMED(c, s, C_GCN, 2.0 * w.Z * rpsC * c->go.cin[k] * d.Hc,
            launch_gcn_layer(s, d, k, w.Z, 1, k == 0 ? first_tab : nullptr, src, dst, false, true,
                             c->gcn + c->go.w[k], c->gcn + c->go.b[k], c->go.cin[k], d.Hc, c->ell_c, c->ell_v,
                             rpsC, 0, nullptr));
      src = dst;
    }
    TIMED(c, s, C_GCN, 0, launch_gcn_expand(s, d, w.Z, w.B, src, w.F, w.fcompact));
    src = nullptr;
    for (int k = 0; k < 4; ++k) {  // t = 0 rows: N-row blocks with the ELL gather, as on the fused path
      const bool last = k == 3;
      float* dst = last ? w.F : bufs[k & 1];
      TIMED(c, s, C_GCN, 2.0 * zb * d.N * c->go.cin[k] * d.Hc,
            launch_gcn_layer(s, d, k, zb, w.B, k == 0 ? xtab_dev : nullptr, src, dst, last, true,
                             c->gcn + c->go.w[k], c->gcn + c->go.b[k], c->go.cin[k], d.Hc, c->ell_c, c->ell_v,
                             d.N, d.N, &w.drop, rps));
      src = dst;
    }
    HIP_TRY(hipGetLastError());
    return SMAML_OK;
  }
  for (int k = 0; k < 4; ++k) {
    const bool last = k == 3;
    float* dst = last ? w.F : bufs[k & 1];
    TIMED(c, s, C_GCN, 2.0 * zb * rps * c->go.cin[k] * d.Hc,
          launch_gcn_layer(s, d, k, zb, w.B, k == 0 ? xtab_dev : nullptr, src, dst, last, true,
                           c->gcn + c->go.w[k], c->gcn + c->go.b[k], c->go.cin[k], d.Hc, c->ell_c, c->ell_v,
                           rps, d.N, &w.drop));
    src = dst;
  }
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

// Pre-split images of theta's gate-GEMM weights for this forward (launch_split_gate; the fast
// weights change every inner step, so every forward re-splits them: a few microseconds).
int prep_gate_images(smaml_ctx* c, hipStream_t s, const float* theta, int64_t tstride, const float* U = nullptr) {
  const Dims& d = c->d;
  Work& w = c->w;
  w.gimg = GateImgs{};
  w.gimg_src = nullptr;
  w.gimg_u_src = nullptr;
  if (!c->kn.gate_img || w.drop.lstm()) return SMAML_OK;  // (the dropout kernels load f32 weights)
  GateImgs gi{};
  const int64_t per = gate_img_bytes(d, &gi) * w.Z;
  const int64_t need = per * (U ? 2 : 1);
  if (need > c->gimg_cap) {
    if (c->gimg_buf) HIP_TRY(hipFree(c->gimg_buf));
    c->gimg_buf = nullptr;
    c->gimg_cap = 0;
    if (hipMalloc((void**)&c->gimg_buf, need) != hipSuccess) {
      (void)hipGetLastError();
      return SMAML_OK;  // no room: the kernels load and split the f32 weights themselves
    }
    c->gimg_cap = need;
  }
  gi.th = c->gimg_buf;
  TIMED(c, s, C_MISC, 0, launch_split_gate(s, d, c->po, theta, tstride, w.Z, gi, gi.th));
  if (U) {
    gi.u = c->gimg_buf + per;
    TIMED(c, s, C_MISC, 0, launch_split_gate(s, d, c->po, U, tstride, w.Z, gi, gi.u));
  }
  w.gimg = gi;
  w.gimg_src = theta;
  w.gimg_u_src = U;
  return SMAML_OK;
}

// Pre-split images of theta's BPTT weights for this backward (launch_split_bwd) when the small-grid
// BPTT steps will read them (small_kw 2, batch-1 sizes); like the gate images, re-split every call.
int prep_bwd_images(smaml_ctx* c, hipStream_t s, const float* theta, int64_t tstride) {
  const Dims& d = c->d;
  Work& w = c->w;
  w.bimg = BwdImgs{};
  w.bimg_src = nullptr;
  if (c->kn.small_kw != 2 || !small_kw_ok(d, w) || (int64_t)w.Z * w.M > c->kn.wgrad_group_max_rows) return SMAML_OK;
  BwdImgs bi{};
  const int64_t need = bwd_img_bytes(d, &bi) * w.Z;
  if (need > c->bimg_cap) {
    if (c->bimg_buf) HIP_TRY(hipFree(c->bimg_buf));
    c->bimg_buf = nullptr;
    c->bimg_cap = 0;
    if (hipMalloc((void**)&c->bimg_buf, need) != hipSuccess) {
      (void)hipGetLastError();
      return SMAML_OK;  // no room: the BPTT steps load and split the f32 weights themselves
    }
    c->bimg_cap = need;
  }
  bi.th = c->bimg_buf;
  TIMED(c, s, C_MISC, 0, launch_split_bwd(s, d, c->po, theta, tstride, w.Z, bi));
  w.bimg = bi;
  w.bimg_src = theta;
  return SMAML_OK;
}

// Layer 0's input projection of a step whose every task reads B consecutive windows, once per distinct
// stream row (kernels.h XgDedup, k_xg_dedup): the XG table of theta (want_xg) and / or of the sweep's
// tangent direction U, into w.xgd. Returns whether the tables were formed (no room, dropout, a batch of
// one or the option off: the gate kernels form the projection in their own K loops).
bool prep_xg_dedup(smaml_ctx* c, hipStream_t s, bool consec, const float* theta, const float* U, int64_t tstride,
                   bool want_xg) {
  const Dims& d = c->d;
  Work& w = c->w;
  w.xgd = XgDedup{};
  if (!consec || !c->kn.xg_dedup || w.B <= 1 || w.drop.gcn() || w.drop.lstm() || (!want_xg && !U)) return false;
  const int64_t per = xg_dedup_rows(w.B, d.T, d.N) * 4 * d.H;
  const int64_t need = per * w.Z * ((want_xg ? 1 : 0) + (U ? 1 : 0));
  if (need > c->xgd_cap) {
    if (c->xgd_buf) HIP_TRY(hipFree(c->xgd_buf));
    c->xgd_buf = nullptr;
    c->xgd_cap = 0;
    if (hipMalloc((void**)&c->xgd_buf, need * 4) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    c->xgd_cap = need;
  }
  XgDedup xd{};
  xd.zstride = per;
  xd.N = d.N;
  w.xgd = xd;  // (zstride read by the launcher)
  const double fl = 2.0 * w.Z * xg_dedup_rows(w.B, d.T, d.N) * 4 * d.H * c->po.lay[0].cin;
  float* dst = c->xgd_buf;
  if (want_xg) {
    const bool img = w.gimg.th && w.gimg_src == theta;
    TIMED(c, s, C_XG, fl,
          launch_xg_dedup(s, d, w, theta, tstride, c->po, img ? w.gimg.th : nullptr, w.gimg.tstride,
                          w.gimg.off[0][0], dst));
    xd.xg = dst;
    xd.src = theta;
    dst += per * w.Z;
  }
  if (U) {
    const bool img = w.gimg.u && w.gimg_u_src == U;
    TIMED(c, s, C_XG, fl,
          launch_xg_dedup(s, d, w, U, tstride, c->po, img ? w.gimg.u : nullptr, w.gimg.tstride, w.gimg.off[0][0],
                          dst));
    xd.rxg = dst;
    xd.u_src = U;
  }
  w.xgd = xd;
  return true;
}

// LSTM forward over all layers and time steps from w.F (anti-diagonal wavefront). consec: every task
// of this step reads B consecutive windows (layer 0's projection may then run once per stream row).
int run_lstm(smaml_ctx* c, hipStream_t s, const float* theta, int64_t tstride, bool consec = false) {
  const Dims& d = c->d;
  Work& w = c->w;
  TRY(prep_gate_images(c, s, theta, tstride));
  // big-tile steps (the meta-step's batches): the XG table when every layer-0 diagonal runs big tiles
  bool xgd_ok = consec;
  for (int diag = 0; xgd_ok && diag < d.T; ++diag) xgd_ok = fwd_wave_big(d, w, c->po, diag);
  const bool use_xgd = xgd_ok && prep_xg_dedup(c, s, true, theta, nullptr, tstride, true);
  if (w.fcompact && !use_xgd) return fail(SMAML_ESTATE, "compact features without the layer-0 projection table");
  // Batch-1 sizes (the small-grid steps): layer 0's input projection F . W_ih0^T does not depend on the
  // recurrence, so it runs for all T steps as one throughput-bound GEMM before the wavefront and the
  // layer-0 steps' latency-bound K loops cover only the recurrent segment (kernels_small.hip).
  w.xg = nullptr;
  w.xg_src = nullptr;
  // only the kw kernel reads the hoisted projection: hoist when every diagonal with a layer-0 step takes it
  bool hoist = small_kw_ok(d, w) && (int64_t)w.Z * w.M <= c->kn.wgrad_group_max_rows;
  for (int diag = 0; hoist && diag < d.T; ++diag) hoist = fwd_wave_kw(d, w, c->po, diag);
  if (hoist) {
    const int64_t per = (int64_t)d.T * w.M * 4 * d.H, need = per * w.Z;
    if (need > c->xg_cap) {
      if (c->xg_buf) HIP_TRY(hipFree(c->xg_buf));
      c->xg_buf = nullptr;
      c->xg_cap = 0;
      if (hipMalloc((void**)&c->xg_buf, need * 4) == hipSuccess)
        c->xg_cap = need;
      else
        (void)hipGetLastError();  // no room: the layer-0 steps form the projection themselves
    }
    if (c->xg_buf) {
      TIMED(c, s, C_XG, 2.0 * w.Z * d.T * w.M * 4 * d.H * d.Hc,
            launch_gemm_nt(s, w.F, (int64_t)d.T * w.M * d.Hc, d.T * w.M, d.Hc, theta + c->po.lay[0].wih, tstride,
                           4 * d.H, c->xg_buf, per, w.Z));
      w.xg = c->xg_buf;
      w.xg_src = theta;
    }
  }
  // row chunks on side streams (fwd_chunks; big sizes only, where every diagonal runs the big tiles)
  const int nch = w.xg ? 1 : fwd_chunks(c);
  hipEvent_t wa = nullptr;
  if (nch > 1 && c->tm.on) (void)hipEventRecord(wa = c->tm.get(), s);
  if (nch > 1) TRY(fork_streams(c, s, nch));
  double wfl = 0.0;
  for (int diag = 0; diag < d.T + d.L - 1; ++diag) {
    FwdWave wv{};
    double fl = fwd_wave(d, w, c->po, diag, 0, false, wv);
    if ((w.xg && fwd_wave_kw(d, w, c->po, diag)) || use_xgd)  // (the projection's flops are counted above)
      for (int q = 0; q < wv.n; ++q)
        if (wv.l[q] == 0) fl -= 2.0 * w.Z * w.M * 4 * d.H * wv.lo[q].cin;
    wfl += fl;
    if (nch > 1) {
      for (int ci = 0; ci < nch; ++ci)
        TIMED(c, c->cs[ci], C_FWD, fl / nch,
              launch_lstm_fwd_wave(c->cs[ci], d, chunk_work(w, ci), diag, theta, tstride, c->po, nullptr, ci, nch));
    } else {
      TIMED(c, s, C_FWD, fl, launch_lstm_fwd_wave(s, d, w, diag, theta, tstride, c->po, nullptr));
    }
  }
  if (nch > 1) {
    TRY(join_streams(c, s, nch));
    time_wall(c, s, wa, C_FWD_WALL, wfl);
  }
  w.xg = nullptr;
  w.xg_src = nullptr;
  w.xgd = XgDedup{};
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

static void ad_cache_drop(smaml_ctx* c) {
  if (c->ad_F) (void)hipFree(c->ad_F);
  c->ad_F = nullptr;
  c->ad_cap = 0;
  c->ad_valid.clear();
}

// New graph / GCN parameters / tasks: every cached window is stale, but the slots stay allocated (a
// re-allocation can cost seconds when the driver has to clear released VRAM, see ad_prepare).
static void ad_cache_invalidate(smaml_ctx* c) { std::fill(c->ad_valid.begin(), c->ad_valid.end(), (uint8_t)0); }

int run_forward(smaml_ctx* c, hipStream_t s, const float* theta, int64_t tstride, const float* const* xtab_dev,
                const float* const* first_tab = nullptr) {
  TRY(run_gcn(c, s, xtab_dev, first_tab));
  c->w.consec = first_tab != nullptr;  // (read by the backward of these activations)
  return run_lstm(c, s, theta, tstride, first_tab != nullptr);
}

int run_bptt(smaml_ctx* c, hipStream_t s, const float* theta, int64_t tstride, float* grad);

// Backward from dpred (already written by k_head_loss) into grad [Z][P].
int run_backward(smaml_ctx* c, hipStream_t s, const float* theta, int64_t tstride, float* grad) {
  const Dims& d = c->d;
  Work& w = c->w;
  const ParamOff& po = c->po;
  const int64_t TM = (int64_t)d.T * w.M;
  const int64_t lsz = (int64_t)w.Z * TM * d.H;
  // batch-1 sizes without LSTM dropout: dh_T comes from the head's weight-gradient launch
  const bool dh_fused = head_small(d, w.M) && !w.drop.lstm();
  if (!dh_fused) TIMED(c, s, C_HEAD_DH, 2.0 * w.Z * w.M * d.HfC * d.H, launch_head_dh(s, d, w, theta, tstride, po));
  int64_t hz = 0;
  const float* hT = head_input(d, w, false, &hz);  // h_T, or drop(h_T) under dropout
  if (head_small(d, w.M)) {
    TIMED(c, s, C_WGRAD, (dh_fused ? 4.0 : 2.0) * w.Z * w.M * d.HfC * d.H,
          launch_head_wgrad_small(s, d, w, w.dpred, hT, hz, grad, po.P, po.wo, po.bo, dh_fused ? theta : nullptr,
                                  tstride));
    return run_bptt(c, s, theta, tstride, grad);
  }
  timed_wgrad(c, s, 2.0 * w.Z * w.M * d.HfC * d.H, w.dpred, (int64_t)w.M * d.HfC, d.HfC, hT, hz, d.H, nullptr, 0, 0,
                     w.M, 0, grad, po.P, po.wo, -1, po.bo, -1);
  return run_bptt(c, s, theta, tstride, grad);
}

// BPTT + LSTM weight gradients from the top layer's dh_T in w.dH [Z][M][H].
int run_bptt(smaml_ctx* c, hipStream_t s, const float* theta, int64_t tstride, float* grad) {
  const Dims& d = c->d;
  Work& w = c->w;
  const ParamOff& po = c->po;
  const int64_t TM = (int64_t)d.T * w.M;
  const int64_t lsz = (int64_t)w.Z * TM * d.H;
  // BPTT as reverse anti-diagonals; layer l's weight gradient as soon as its t = 0 step is done,
  // or, for small grids (batch-1 adaptation), all layers' in one launch after the sweep
  const bool grouped = (int64_t)w.Z * w.M <= c->kn.wgrad_group_max_rows;
  TRY(prep_bwd_images(c, s, theta, tstride));
  WgradPlan plans[MAX_LAYERS];
  double gfl = 0.0;
  auto layer_wgrad = [&](int l) {
    const LayerOff& lo = po.lay[l];
    const float* X = l == 0 ? w.F : w.Hs + (int64_t)(l - 1) * lsz;
    if (grouped) {
      WgradPlan& p = plans[l];
      plan_wgrad(w, w.dG + (int64_t)l * lsz * 4, TM * 4 * d.H, 4 * d.H, X, TM * lo.cin, lo.cin,
                 w.Hs + (int64_t)l * lsz, TM * d.H, d.H, TM, w.M, grad, po.P, lo.wih, lo.whh, lo.bih, lo.bhh, true,
                 false, p, true);
      p.drop = w.drop;
      p.drop_layer = l - 1;
      gfl += 2.0 * w.Z * TM * 4 * d.H * (lo.cin + d.H);
      return;
    }
    if (l == 0 && wgrad_dedup_ok(c) && timed_wgrad_ih0_dedup(c, s, w.dG, grad)) {
      // W_hh0 and the bias over every row (h_{t-1} differs per window): [0 | h_{t-1}], no input columns
      timed_wgrad(c, s, 2.0 * w.Z * TM * 4 * d.H * d.H, w.dG, TM * 4 * d.H, 4 * d.H, nullptr, 0, 0, w.Hs, TM * d.H,
                  d.H, TM, w.M, grad, po.P, -1, lo.whh, lo.bih, lo.bhh, true, false, -1);
      return;
    }
    timed_wgrad(c, s, 2.0 * w.Z * TM * 4 * d.H * (lo.cin + d.H), w.dG + (int64_t)l * lsz * 4, TM * 4 * d.H, 4 * d.H, X,
                TM * lo.cin, lo.cin, w.Hs + (int64_t)l * lsz, TM * d.H, d.H, TM, w.M, grad, po.P, lo.wih, lo.whh,
                lo.bih, lo.bhh, true, false, l - 1);
  };
  // after a chunked sweep: layers L-1 .. 0 on the caller's stream
  auto after_sweep_wgrads = [&]() {
    for (int l = d.L - 1; l >= 0; --l) layer_wgrad(l);
  };
  // row chunks on side streams (knob bptt_streams): every diagonal's big-tile launch split by rows, the
  // weight gradients after the sweep on the caller's stream
  // (chunked only where a full diagonal runs the big tiles anyway: tile-forcing knobs keep their meaning)
  const int nch = grouped || !bwd_wave_big(d, w, po, std::min(d.L, d.T) - 1) ? 1 : c->kn.bptt_streams;
  hipEvent_t wa = nullptr;
  if (nch > 1 && c->tm.on) (void)hipEventRecord(wa = c->tm.get(), s);
  if (nch > 1) TRY(fork_streams(c, s, nch));
  double wfl = 0.0;
  for (int e = 0; e < d.T + d.L - 1; ++e) {
    BwdWave wv{};
    const double fl = bwd_wave(d, w, po, e, 0, false, wv);
    wfl += fl;
    if (nch > 1) {
      for (int ci = 0; ci < nch; ++ci)
        TIMED(c, c->cs[ci], C_BWD, fl / nch, launch_lstm_bwd_wave(c->cs[ci], d, chunk_work(w, ci), e, theta, tstride, po, ci, nch));
    } else {
      TIMED(c, s, C_BWD, fl, launch_lstm_bwd_wave(s, d, w, e, theta, tstride, po));
    }
    const int l = d.L - 1 - (e - (d.T - 1));
    if (e < d.T - 1 || l < 0) continue;
    if (nch <= 1) layer_wgrad(l);
  }
  if (nch > 1) {
    TRY(join_streams(c, s, nch));
    time_wall(c, s, wa, C_BWD_WALL, wfl);
    after_sweep_wgrads();
  }
  if (grouped) TIMED(c, s, C_WGRAD, gfl, launch_wgrad_multi(s, w, plans, d.L, c->kn.wgrad_group_wgs));
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

// Primal recompute + tangent along U (second-order sweep), GCN features recomputed.
// gcn_cached: w.F is the step's so_F slot, written by the inner loop's GCN in the layout fcompact_rec
// recorded then (not re-derived: f_compact_ok allocates, so a later call could decide differently).
int run_forward_dual(smaml_ctx* c, hipStream_t s, const float* theta, const float* U, int64_t tstride,
                     const float* const* xtab_dev, bool gcn_cached, const float* const* first_tab, int fcompact_rec) {
  const Dims& d = c->d;
  Work& w = c->w;
  if (!gcn_cached) TRY(run_gcn(c, s, xtab_dev, first_tab));
  else w.fcompact = fcompact_rec;
  w.consec = first_tab != nullptr;
  TRY(prep_gate_images(c, s, theta, tstride, U));
  // layer 0's tangent projection F U_ih0^T (and, unless the primal is kept, F W_ih0^T) once per stream row
  const bool use_xgd = prep_xg_dedup(c, s, first_tab != nullptr, theta, U, tstride, !w.primal_kept);
  if (w.fcompact && !use_xgd) return fail(SMAML_ESTATE, "compact features without the layer-0 projection tables");
  const int nch = fwd_chunks(c);  // (row chunks on side streams)
  hipEvent_t wa = nullptr;
  if (nch > 1 && c->tm.on) (void)hipEventRecord(wa = c->tm.get(), s);
  if (nch > 1) TRY(fork_streams(c, s, nch));
  double wfl = 0.0;
  for (int diag = 0; diag < d.T + d.L - 1; ++diag) {
    FwdWave wv{};
    double fl = fwd_wave(d, w, c->po, diag, 0, true, wv);
    if (w.primal_kept) fl -= fwd_wave(d, w, c->po, diag, 0, false, wv);  // tangent pass only
    if (use_xgd)  // (counted in C_XG)
      for (int q = 0; q < wv.n; ++q)
        if (wv.l[q] == 0) fl -= (w.primal_kept ? 1.0 : 2.0) * 2.0 * w.Z * w.M * 4 * d.H * wv.lo[q].cin;
    wfl += fl;
    if (nch > 1) {
      for (int ci = 0; ci < nch; ++ci)
        TIMED(c, c->cs[ci], C_FWD_DUAL, fl / nch,
              launch_lstm_fwd_dual_wave(c->cs[ci], d, chunk_work(w, ci), diag, theta, U, tstride, c->po, nullptr, ci, nch));
    } else {
      TIMED(c, s, C_FWD_DUAL, fl, launch_lstm_fwd_dual_wave(s, d, w, diag, theta, U, tstride, c->po, nullptr));
    }
  }
  if (nch > 1) {
    TRY(join_streams(c, s, nch));
    time_wall(c, s, wa, C_FWD_DUAL_WALL, wfl);
  }
  w.xgd = XgDedup{};
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

// Tangent of the backward pass: HU[z] = H_z U[z] (primal weight grads are not formed).
int run_backward_dual(smaml_ctx* c, hipStream_t s, const float* theta, const float* U, int64_t tstride, float* HU) {
  const Dims& d = c->d;
  Work& w = c->w;
  const ParamOff& po = c->po;
  const int64_t TM = (int64_t)d.T * w.M;
  const int64_t lsz = (int64_t)w.Z * TM * d.H;
  TIMED(c, s, C_HEAD_DH, 3.0 * 2.0 * w.Z * w.M * d.HfC * d.H, launch_head_dh_dual(s, d, w, theta, U, tstride, po));
  int64_t hz = 0;
  const float* hT = head_input(d, w, false, &hz);
  const float* RhT = head_input(d, w, true, &hz);
  timed_wgrad(c, s, 2.0 * w.Z * w.M * d.HfC * d.H, w.Rdpred, (int64_t)w.M * d.HfC, d.HfC, hT, hz, d.H, nullptr, 0, 0,
                     w.M, 0, HU, po.P, po.wo, -1, po.bo, -1, true, false);
  timed_wgrad(c, s, 2.0 * w.Z * w.M * d.HfC * d.H, w.dpred, (int64_t)w.M * d.HfC, d.HfC, RhT, hz, d.H, nullptr, 0, 0,
                     w.M, 0, HU, po.P, po.wo, -1, po.bo, -1, false, true);
  auto layer_wgrad = [&](int l) {
    const LayerOff& lo = po.lay[l];
    const float* X = l == 0 ? w.F : w.Hs + (int64_t)(l - 1) * lsz;
    const float* RX = l == 0 ? nullptr : w.RHs + (int64_t)(l - 1) * lsz;
    const float* dGl = w.dG + (int64_t)l * lsz * 4;
    const float* RdGl = w.RGs + (int64_t)l * lsz * 4;
    if (l == 0 && wgrad_dedup_ok(c) && timed_wgrad_ih0_dedup(c, s, RdGl, HU)) {
      // R(dW_ih0) = R(dG0)^T F (R x = 0 at layer 0) over distinct stream rows above; R(dW_hh0) =
      // R(dG0)^T h + dG0^T R h and R(db) as one paired launch over every row
      const double flp = 2.0 * 2.0 * w.Z * TM * 4 * d.H * d.H;
      if (!(c->kn.wgrad_pair && timed_wgrad_pair(c, s, flp, RdGl, dGl, TM * 4 * d.H, 4 * d.H, nullptr, nullptr, 0, 0,
                                                 w.Hs, w.RHs, TM * d.H, d.H, TM, w.M, HU, po.P, -1, lo.whh, lo.bih,
                                                 lo.bhh, -1))) {
        timed_wgrad(c, s, flp / 2, RdGl, TM * 4 * d.H, 4 * d.H, nullptr, 0, 0, w.Hs, TM * d.H, d.H, TM, w.M, HU, po.P,
                    -1, lo.whh, lo.bih, lo.bhh, true, false, -1);
        timed_wgrad(c, s, flp / 2, dGl, TM * 4 * d.H, 4 * d.H, nullptr, 0, 0, w.RHs, TM * d.H, d.H, TM, w.M, HU, po.P,
                    -1, lo.whh, lo.bih, lo.bhh, false, true, -1);
      }
      return;
    }
    if (l > 0 && c->kn.wgrad_pair &&  // both passes 4H x (cin + H): one launch
        timed_wgrad_pair(c, s, 2.0 * 2.0 * w.Z * TM * 4 * d.H * (lo.cin + d.H), RdGl, dGl, TM * 4 * d.H, 4 * d.H, X,
                         RX, TM * lo.cin, lo.cin, w.Hs + (int64_t)l * lsz, w.RHs + (int64_t)l * lsz, TM * d.H, d.H,
                         TM, w.M, HU, po.P, lo.wih, lo.whh, lo.bih, lo.bhh, l - 1))
      return;
    timed_wgrad(c, s, 2.0 * w.Z * TM * 4 * d.H * (lo.cin + d.H), RdGl, TM * 4 * d.H, 4 * d.H, X, TM * lo.cin, lo.cin,
                w.Hs + (int64_t)l * lsz, TM * d.H, d.H, TM, w.M, HU, po.P, lo.wih, lo.whh, lo.bih, lo.bhh, true, false,
                l - 1);
    timed_wgrad(c, s, 2.0 * w.Z * TM * 4 * d.H * ((l > 0 ? lo.cin : 0) + d.H), dGl, TM * 4 * d.H, 4 * d.H, RX,
                TM * lo.cin, l > 0 ? lo.cin : 0, w.RHs + (int64_t)l * lsz, TM * d.H, d.H, TM, w.M, HU, po.P, lo.wih,
                lo.whh, lo.bih, lo.bhh, false, true, l - 1);
  };
  // after a chunked sweep: layers L-1 .. 0 on the caller's stream
  auto after_sweep_wgrads = [&]() {
    for (int l = d.L - 1; l >= 0; --l) layer_wgrad(l);
  };
  const int nch = (int64_t)w.Z * w.M <= c->kn.wgrad_group_max_rows || !bwd_dual_wave_big(d, w, po, std::min(d.L, d.T) - 1)
                      ? 1
                      : c->kn.bptt_streams;
  hipEvent_t wa = nullptr;
  if (nch > 1 && c->tm.on) (void)hipEventRecord(wa = c->tm.get(), s);
  if (nch > 1) TRY(fork_streams(c, s, nch));
  double wfl = 0.0;
  for (int e = 0; e < d.T + d.L - 1; ++e) {
    BwdWave wv{};
    const double fl = bwd_wave(d, w, po, e, 0, true, wv) * (w.primal_kept ? 2.0 / 3.0 : 1.0);
    wfl += fl;
    if (nch > 1) {
      for (int ci = 0; ci < nch; ++ci)
        TIMED(c, c->cs[ci], C_BWD_DUAL, fl / nch,
              launch_lstm_bwd_dual_wave(c->cs[ci], d, chunk_work(w, ci), e, theta, U, tstride, po, ci, nch));
    } else {
      TIMED(c, s, C_BWD_DUAL, fl, launch_lstm_bwd_dual_wave(s, d, w, e, theta, U, tstride, po));
    }
    const int l = d.L - 1 - (e - (d.T - 1));
    if (e < d.T - 1 || l < 0) continue;
    if (nch <= 1) layer_wgrad(l);
  }
  if (nch > 1) {
    TRY(join_streams(c, s, nch));
    time_wall(c, s, wa, C_BWD_DUAL_WALL, wfl);
    after_sweep_wgrads();
  }
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

int require_ready(smaml_ctx* c) {
  if (!c) return fail(SMAML_EINVAL, "ctx is NULL");
  if (!c->ell_c) return fail(SMAML_ESTATE, "smaml_set_graph not called");
  if (!c->gcn) return fail(SMAML_ESTATE, "smaml_set_gcn_params not called");
  return SMAML_OK;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// the bookkeeping kernels' grid-barrier state (zeroed once; self-resetting, see kernels.h GridBar)
int ensure_bar(smaml_ctx* c) {
  if (c->bar) return SMAML_OK;
  int khz = 0;
  HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device));
  c->wall_khz = khz > 0 ? (uint64_t)khz : 100000;
  HIP_TRY(hipHostMalloc((void**)&c->bar_err_host, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
  *(volatile int*)c->bar_err_host = 0;
  HIP_TRY(hipHostGetDevicePointer((void**)&c->bar_err_dev, c->bar_err_host, 0));
  HIP_TRY(hipMalloc((void**)&c->bar, 4 * sizeof(unsigned)));
  HIP_TRY(hipMemset(c->bar, 0, 4 * sizeof(unsigned)));
  HIP_TRY(hipDeviceSynchronize());
  return SMAML_OK;
}

BarPlan bar_plan(const smaml_ctx* c) {
  BarPlan bp{};
  bp.gb.w = c->bar;
  bp.gb.host_err = c->bar_err_dev;
  bp.gb.timeout = (uint64_t)c->bar_timeout_us * c->wall_khz / 1000;
  bp.fused = c->bar_fused;
  bp.oversize = c->bar_oversize;
  return bp;
}

// A grid-barrier wait that timed out (kernels.h grid_barrier) raised the pinned flag: drain the device,
// reset the barrier state and report it. No host sync unless the flag is up.
int check_device_error(smaml_ctx* c) {
  if (!c->bar_err_host || *(volatile int*)c->bar_err_host == 0) return SMAML_OK;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemset(c->bar, 0, 4 * sizeof(unsigned)));
  HIP_TRY(hipDeviceSynchronize());
  *(volatile int*)c->bar_err_host = 0;
  return fail(SMAML_EHIP,
              "a grid-barrier kernel (k_inner_sgd / k_sweep_update) timed out waiting for its grid: the grid was "
              "not co-resident (another process holding the GPU, or the barrier_oversize debug knob); its "
              "results are invalid");
}

}  // namespace

// =====================================================================================
extern "C" {

const char* smaml_last_error(void) { return g_err.c_str(); }

int32_t smaml_abi_version(void) { return 7; }

const char* smaml_build_info(void) { return smaml::products_info(); }

int smaml_param_layout(const smaml_dims* dims, int32_t which, int64_t* offsets, int64_t* sizes, int32_t cap,
                       int32_t* count, int64_t* total) {
  TRY(check_dims(dims));
  if (which != 0 && which != 1) return fail(SMAML_EINVAL, "which must be 0 (trainable) or 1 (gcn)");
  std::vector<Spec> sp;
  int64_t tot = 0;
  layout(*dims, which, sp, tot);
  if (count) *count = (int32_t)sp.size();
  if (total) *total = tot;
  for (int i = 0; i < (int)sp.size() && i < cap; ++i) {
    if (offsets) offsets[i] = sp[i].off;
    if (sizes) sizes[i] = sp[i].size;
  }
  return SMAML_OK;
}

int smaml_graph_ell(const int64_t* edge_index_host, int64_t num_edges, int32_t num_nodes, int32_t* cols_host,
                    float* vals_host) {
  if (!edge_index_host || !cols_host || !vals_host || num_nodes <= 0 || num_edges < 0)
    return fail(SMAML_EINVAL, "bad arguments to smaml_graph_ell");
  std::vector<int32_t> cols;
  std::vector<float> vals;
  TRY(build_ell(edge_index_host, num_edges, num_nodes, cols, vals));
  std::memcpy(cols_host, cols.data(), cols.size() * 4);
  std::memcpy(vals_host, vals.data(), vals.size() * 4);
  return SMAML_OK;
}

int smaml_create(const smaml_dims* dims, int32_t device, smaml_ctx** out) {
  if (!out) return fail(SMAML_EINVAL, "out is NULL");
  *out = nullptr;
  TRY(check_dims(dims));
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(SMAML_EINVAL, "device ordinal out of range");
  smaml_ctx* c = new smaml_ctx();
  c->dims = *dims;
  c->device = device;
  Dims& d = c->d;
  d.N = dims->num_nodes;
  d.T = dims->window_size;
  d.Cin0 = dims->input_channels;
  d.Hc = dims->hidden_channels;
  d.H = dims->lstm_hidden_size;
  d.L = dims->lstm_num_layers;
  d.Hf = dims->forecast_horizon;
  d.C = dims->output_channels;
  d.HfC = d.Hf * d.C;
  std::vector<Spec> sp;
  int64_t tot = 0;
  layout(*dims, 0, sp, tot);
  for (int l = 0; l < d.L; ++l) {
    c->po.lay[l].wih = sp[4 * l].off;
    c->po.lay[l].whh = sp[4 * l + 1].off;
    c->po.lay[l].bih = sp[4 * l + 2].off;
    c->po.lay[l].bhh = sp[4 * l + 3].off;
    c->po.lay[l].cin = l == 0 ? d.Hc : d.H;
  }
  c->po.wo = sp[4 * d.L].off;
  c->po.bo = sp[4 * d.L + 1].off;
  c->po.P = tot;
  int64_t nv = 0;
  for (auto& x : sp) nv += x.size;
  c->po.n_valid = nv;
  layout(*dims, 1, sp, tot);
  for (int k = 0; k < 4; ++k) {
    c->go.b[k] = sp[2 * k].off;
    c->go.w[k] = sp[2 * k + 1].off;
    c->go.cin[k] = k == 0 ? d.Cin0 : d.Hc;
  }
  c->go.total = tot;
  if (const char* e = std::getenv("SMAML_BWD_BIG_MIN")) c->kn.bwd_big_min = std::atoi(e);
  if (const char* e = std::getenv("SMAML_BWDD_BIG_MIN")) c->kn.bwdd_big_min = std::atoi(e);
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    delete c;
    return fail(SMAML_EHIP, std::string("context init: ") + hipGetErrorString(e));
  }
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0) c->n_cu = ncu;
  *out = c;
  return SMAML_OK;
}

int smaml_destroy(smaml_ctx* c) {
  if (!c) return SMAML_OK;
  (void)hipSetDevice(c->device);
  if (c->comm) (void)smaml_comm_destroy(c);
  (void)hipDeviceSynchronize();
  if (c->arena) (void)hipFree(c->arena);
  if (c->ell_c) (void)hipFree(c->ell_c);
  if (c->ell_v) (void)hipFree(c->ell_v);
  if (c->tr_p) (void)hipFree(c->tr_p);
  if (c->tr_c) (void)hipFree(c->tr_c);
  if (c->tr_v) (void)hipFree(c->tr_v);
  if (c->bw_scratch) (void)hipFree(c->bw_scratch);
  if (c->xtab) (void)hipFree((void*)c->xtab);
  (void)c->stage.release();
  if (c->scratch_loss) (void)hipFree(c->scratch_loss);
  if (c->so_theta) (void)hipFree(c->so_theta);
  if (c->so_grad) (void)hipFree(c->so_grad);
  if (c->so_norm) (void)hipFree(c->so_norm);
  if (c->so_coef) (void)hipFree(c->so_coef);
  if (c->so_F) (void)hipFree(c->so_F);
  if (c->gcn_wimg) (void)hipFree(c->gcn_wimg);
  if (c->gimg_buf) (void)hipFree(c->gimg_buf);
  if (c->bimg_buf) (void)hipFree(c->bimg_buf);
  if (c->xg_buf) (void)hipFree(c->xg_buf);
  if (c->xgd_buf) (void)hipFree(c->xgd_buf);
  if (c->bar) (void)hipFree(c->bar);
  for (int i = 0; i < 4; ++i) {
    if (c->cs[i]) (void)hipStreamDestroy(c->cs[i]);
    if (c->join_ev[i]) (void)hipEventDestroy(c->join_ev[i]);
  }
  if (c->fork_ev) (void)hipEventDestroy(c->fork_ev);
  if (c->bar_err_host) (void)hipHostFree(c->bar_err_host);
  ad_cache_drop(c);
  for (float* p : c->keep_mem) (void)hipFree(p);
  for (auto& r : c->tm.recs) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  for (auto e : c->tm.pool) (void)hipEventDestroy(e);
  delete c;
  return SMAML_OK;
}

int smaml_set_graph(smaml_ctx* c, const int64_t* edge_index_host, int64_t num_edges) {
  if (!c || !edge_index_host) return fail(SMAML_EINVAL, "NULL argument");
  TRY(ensure_device(c));
  std::vector<int32_t> cols;
  std::vector<float> vals;
  TRY(build_ell(edge_index_host, num_edges, c->d.N, cols, vals));
  ad_cache_invalidate(c);
  if (!c->ell_c) {
    HIP_TRY(hipMalloc((void**)&c->ell_c, cols.size() * 4));
    HIP_TRY(hipMalloc((void**)&c->ell_v, vals.size() * 4));
  }
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(c->ell_c, cols.data(), cols.size() * 4, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(c->ell_v, vals.data(), vals.size() * 4, hipMemcpyHostToDevice));
  // A_hat^T as CSR: entry (t, e) of the ELL (row t gathers column cols[t][e] with weight vals[t][e])
  // becomes row cols[t][e] of the transpose, in ascending t (fixed order)
  const int N = c->d.N;
  std::vector<int32_t> tp(N + 1, 0), tc;
  std::vector<float> tv;
  for (int t = 0; t < N; ++t)
    for (int e = 0; e < ELLW; ++e)
      if (vals[(size_t)t * ELLW + e] != 0.f) ++tp[cols[(size_t)t * ELLW + e] + 1];
  for (int i = 0; i < N; ++i) tp[i + 1] += tp[i];
  tc.resize(tp[N]);
  tv.resize(tp[N]);
  std::vector<int32_t> pos(tp.begin(), tp.end() - 1);
  for (int t = 0; t < N; ++t)
    for (int e = 0; e < ELLW; ++e) {
      const float v = vals[(size_t)t * ELLW + e];
      if (v == 0.f) continue;
      const int j = cols[(size_t)t * ELLW + e];
      tc[pos[j]] = t;
      tv[pos[j]] = v;
      ++pos[j];
    }
  if (!c->tr_p) HIP_TRY(hipMalloc((void**)&c->tr_p, (size_t)(N + 1) * 4));
  if ((int64_t)tc.size() > c->tr_nnz_cap) {
    if (c->tr_c) HIP_TRY(hipFree(c->tr_c));
    if (c->tr_v) HIP_TRY(hipFree(c->tr_v));
    c->tr_nnz_cap = std::max<int64_t>((int64_t)tc.size(), 1);
    HIP_TRY(hipMalloc((void**)&c->tr_c, c->tr_nnz_cap * 4));
    HIP_TRY(hipMalloc((void**)&c->tr_v, c->tr_nnz_cap * 4));
  }
  HIP_TRY(hipMemcpy(c->tr_p, tp.data(), tp.size() * 4, hipMemcpyHostToDevice));
  if (!tc.empty()) {
    HIP_TRY(hipMemcpy(c->tr_c, tc.data(), tc.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->tr_v, tv.data(), tv.size() * 4, hipMemcpyHostToDevice));
  }
  return SMAML_OK;
}

int smaml_set_gcn_params(smaml_ctx* c, const float* gcn_flat) {
  if (!c || !gcn_flat) return fail(SMAML_EINVAL, "NULL argument");
  if (!aligned16(gcn_flat)) return fail(SMAML_EINVAL, "gcn params must be 16-byte aligned");
  c->gcn = gcn_flat;
  ad_cache_invalidate(c);  // cached features belong to the previous GCN parameters (the slots stay allocated)
  return SMAML_OK;
}

int smaml_reserve(smaml_ctx* c, int32_t tasks, int32_t batch) {
  if (!c || tasks <= 0 || batch <= 0) return fail(SMAML_EINVAL, "bad reserve arguments");
  TRY(ensure_device(c));
  return reserve(c, tasks, batch);
}

int64_t smaml_workspace_bytes(const smaml_ctx* c) { return c ? c->arena_bytes : 0; }

int32_t smaml_so_kept_steps(const smaml_ctx* c) { return c ? c->keep_last : 0; }

int smaml_set_dropout(smaml_ctx* c, float p_gcn, float p_lstm, uint32_t seed) {
  if (!c) return fail(SMAML_EINVAL, "ctx is NULL");
  if (!(p_gcn >= 0.f && p_gcn < 1.f) || !(p_lstm >= 0.f && p_lstm < 1.f))
    return fail(SMAML_EINVAL, "dropout probabilities must lie in [0, 1)");
  c->p_gcn = p_gcn;
  c->p_lstm = p_lstm;
  c->drop_seed = seed;
  return SMAML_OK;
}

int smaml_set_task_ids(smaml_ctx* c, const int32_t* ids_host, int32_t n) {
  if (!c || n < 0 || (n > 0 && !ids_host)) return fail(SMAML_EINVAL, "bad set_task_ids arguments");
  c->task_ids.assign(ids_host, ids_host + n);
  return SMAML_OK;
}

int smaml_gcn_conv(smaml_ctx* c, void* stream, const float* x, int32_t rows, int32_t cin, const float* weight,
                   const float* bias, int32_t cout, float* out) {
  if (!c) return fail(SMAML_EINVAL, "ctx is NULL");
  if (!c->ell_c) return fail(SMAML_ESTATE, "smaml_set_graph not called");
  if (!x || !weight || !bias || !out || rows <= 0 || cin <= 0 || cout <= 0)
    return fail(SMAML_EINVAL, "bad gcn_conv arguments");
  if (cin % 4) return fail(SMAML_EINVAL, "cin must be a multiple of 4");
  if (!aligned16(x) || !aligned16(weight)) return fail(SMAML_EINVAL, "x / weight must be 16-byte aligned");
  TRY(ensure_device(c));
  hipStream_t s = (hipStream_t)stream;
  launch_gcn_layer(s, c->d, 0, 1, 1, nullptr, x, out, false, false, weight, bias, cin, cout, c->ell_c, c->ell_v,
                   rows, std::min(rows, c->d.N));
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

int smaml_gcn_conv_ex(smaml_ctx* c, void* stream, const float* x, int32_t rows, int32_t cin, const float* weight,
                      const float* bias, int32_t cout, int32_t flags, float* out) {
  if (!c) return fail(SMAML_EINVAL, "ctx is NULL");
  const bool plain = (flags & SMAML_GCN_PLAIN) != 0, relu = (flags & SMAML_GCN_RELU) != 0;
  if (!plain && !c->ell_c) return fail(SMAML_ESTATE, "smaml_set_graph not called");
  if (!x || !weight || !bias || !out || rows <= 0 || cin <= 0 || cout <= 0 || (flags & ~3))
    return fail(SMAML_EINVAL, "bad gcn_conv_ex arguments");
  if (cin % 4) return fail(SMAML_EINVAL, "cin must be a multiple of 4");
  if (!aligned16(x) || !aligned16(weight)) return fail(SMAML_EINVAL, "x / weight must be 16-byte aligned");
  TRY(ensure_device(c));
  TRY(check_device_error(c));
  hipStream_t s = (hipStream_t)stream;
  launch_gcn_layer(s, c->d, 0, 1, 1, nullptr, x, out, false, relu, weight, bias, cin, cout, c->ell_c, c->ell_v, rows,
                   plain ? 0 : std::min(rows, c->d.N));
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

int smaml_gcn_conv_backward(smaml_ctx* c, void* stream, const float* x, int32_t rows, int32_t cin,
                            const float* weight, int32_t cout, const float* dz, int32_t flags, float* dx, float* dwb) {
  if (!c) return fail(SMAML_EINVAL, "ctx is NULL");
  const bool plain = (flags & SMAML_GCN_PLAIN) != 0;
  if (!plain && !c->ell_c) return fail(SMAML_ESTATE, "smaml_set_graph not called");
  if (!x || !weight || !dz || rows <= 0 || cin <= 0 || cout <= 0 || (flags & ~SMAML_GCN_PLAIN) || (!dx && !dwb))
    return fail(SMAML_EINVAL, "bad gcn_conv_backward arguments");
  if (cin % 4 || cout % 4) return fail(SMAML_EINVAL, "cin and cout must be multiples of 4");
  if (!aligned16(x) || !aligned16(weight) || !aligned16(dz) || (dx && !aligned16(dx)))
    return fail(SMAML_EINVAL, "x / weight / dz / dx must be 16-byte aligned");
  TRY(ensure_device(c));
  TRY(check_device_error(c));
  TRY(reserve(c, 1, 1));  // the split-K partial slabs of the weight gradient
  hipStream_t s = (hipStream_t)stream;
  const int ng = plain ? 0 : std::min(rows, c->d.N);
  const int64_t need = 2 * (int64_t)rows * std::max(cin, cout);
  if (need > c->bw_scratch_cap) {
    if (c->bw_scratch) HIP_TRY(hipFree(c->bw_scratch));
    HIP_TRY(hipMalloc((void**)&c->bw_scratch, need * 4));
    c->bw_scratch_cap = need;
  }
  float* t0 = c->bw_scratch;
  float* t1 = c->bw_scratch + (int64_t)rows * std::max(cin, cout);
  if (dwb) {
    // dW = dz^T (A_hat x), db = sum_rows dz: the split-K weight-gradient GEMM with its bias column
    const float* ax = x;
    if (ng > 0) {
      launch_gather_rows(s, x, t0, rows, cin, ng, c->ell_c, c->ell_v, nullptr, nullptr, nullptr);
      ax = t0;
    }
    Work w = c->w;
    w.Z = 1;
    w.drop = Drop{};
    w.kn = c->kn;
    launch_wgrad(s, c->d, w, dz, 0, cout, ax, 0, cin, nullptr, 0, 0, rows, 0, dwb, 0, 0, 0,
                 (int64_t)cout * cin, -1, true, false);
  }
  if (dx) {
    // dx = A_hat^T (dz W): the rows past the graph's nodes see only their self loop
    if (ng > 0) {
      launch_gemm_nn_plain(s, dz, rows, cout, weight, cin, t1);
      launch_gather_rows(s, t1, dx, rows, cin, ng, nullptr, nullptr, c->tr_p, c->tr_c, c->tr_v);
    } else {
      launch_gemm_nn_plain(s, dz, rows, cout, weight, cin, dx);
    }
  }
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

int smaml_relu_mask(smaml_ctx* c, void* stream, float* g, const float* h, int64_t n) {
  if (!c || !g || !h || n <= 0) return fail(SMAML_EINVAL, "bad relu_mask arguments");
  TRY(ensure_device(c));
  launch_relu_mask((hipStream_t)stream, g, h, n);
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

int smaml_forward(smaml_ctx* c, void* stream, const float* theta, const float* const* x_host, int32_t nsamples,
                  float* pred, float* feats) {
  TRY(require_ready(c));
  if (!theta || !x_host || nsamples <= 0 || !pred) return fail(SMAML_EINVAL, "bad forward arguments");
  for (int i = 0; i < nsamples; ++i)
    if (!x_host[i] || !aligned16(x_host[i])) return fail(SMAML_EINVAL, "sample x pointers must be 16-B aligned");
  TRY(ensure_device(c));
  hipStream_t s = (hipStream_t)stream;
  TRY(reserve(c, 1, nsamples));
  set_work(c, 1, nsamples);
  TRY(upload_xtab(c, s, x_host, nsamples));
  const float* const* xt = nullptr;
  TRY(xtab_at(c, 0, &xt));
  if (c->p_gcn > 0.f || c->p_lstm > 0.f) {  // train-mode module forward: masks of (seed, task id, step 0)
    TRY(upload_task_ids(c, s, 1));
    set_step_drop(c, 0);  // kept in c->w.drop for the smaml_backward of these activations
  }
  TRY(run_forward(c, s, theta, 0, xt));
  Work w = c->w;
  w.pred = pred;
  launch_head_loss(s, c->d, w, theta, 0, c->po, nullptr, 0.f, false);
  c->act_B = nsamples;
  if (feats) {
    const Dims& d = c->d;
    const int64_t blk = (int64_t)d.N * d.Hc;
    for (int si = 0; si < nsamples; ++si) {
      // F is [T][M][Hc] with M = nsamples*N; feats is [s][T*N][Hc]
      HIP_TRY(hipMemcpy2DAsync(feats + (int64_t)si * d.T * blk, blk * 4, c->w.F + (int64_t)si * blk,
                               (int64_t)nsamples * blk * 4, blk * 4, d.T, hipMemcpyDeviceToDevice, s));
    }
  }
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

int smaml_set_tasks(smaml_ctx* c, int32_t ntasks, const float* const* features_host, const int32_t* t_total_host) {
  if (c) ad_cache_invalidate(c);
  if (!c || ntasks <= 0 || !features_host || !t_total_host) return fail(SMAML_EINVAL, "bad set_tasks arguments");
  c->feats.assign(features_host, features_host + ntasks);
  c->t_total.assign(t_total_host, t_total_host + ntasks);
  for (int j = 0; j < ntasks; ++j) {
    if (!c->feats[j] || !aligned16(c->feats[j])) return fail(SMAML_EINVAL, "feature streams must be 16-B aligned");
    if (c->t_total[j] < c->d.T + c->d.Hf + 1) return fail(SMAML_EINVAL, "feature stream shorter than one sample");
  }
  return SMAML_OK;
}

int smaml_meta_step(smaml_ctx* c, void* stream, const float* theta, int32_t order, int32_t steps, int32_t batch,
                    const int32_t* windows_host, float inner_lr, float max_norm, float query_scale,
                    float* meta_grad, float* losses, float* norms, float* fast_out) {
  TRY(require_ready(c));
  if (c->feats.empty()) return fail(SMAML_ESTATE, "smaml_set_tasks not called");
  if (!theta || steps < 0 || batch <= 0 || !windows_host) return fail(SMAML_EINVAL, "bad meta_step arguments");
  if (order < 0 || order > 2) return fail(SMAML_EINVAL, "order must be 0, 1 or 2");
  if (order >= 1 && !meta_grad) return fail(SMAML_EINVAL, "meta_grad required for order >= 1");
  TRY(ensure_device(c));
  hipStream_t s = (hipStream_t)stream;
  const Dims& d = c->d;
  const int Z = (int)c->feats.size();
  const int B = batch;
  TRY(ensure_bar(c));
  TRY(check_device_error(c));
  TRY(reserve(c, Z, B, order == 2));
  if (order == 2) TRY(ensure_so_store(c, std::max(steps, 1), Z, B));
  if (order == 2) TRY(ensure_keep(c, steps, Z, B));
  set_work(c, Z, B);
  const int nkeep = order == 2 ? std::min(std::min(c->keep_n, c->keep_want), steps) : 0;
  c->keep_last = nkeep;
  // sample window table for every step (support steps then the query batch)
  const int64_t nptr = (int64_t)(steps + 1) * Z * B;
  // (+ each step's per-task first-window pointers, the GCN's consecutive-window tables)
  std::vector<const float*> ptrs(nptr + (int64_t)(steps + 1) * Z);
  const int max_w_off = d.T + d.Hf;  // last stream index read by a sample = w + T + Hf
  for (int k = 0; k <= steps; ++k)
    for (int z = 0; z < Z; ++z)
      for (int b = 0; b < B; ++b) {
        const int64_t i = ((int64_t)k * Z + z) * B + b;
        const int wv = windows_host[i];
        if (wv < 0 || wv + max_w_off >= c->t_total[z])
          return fail(SMAML_EINVAL, "window start out of range for task " + std::to_string(z));
        ptrs[i] = c->feats[z] + (int64_t)wv * d.N * d.Cin0;
      }
  // steps whose every task reads B consecutive windows (the reference's support and query batches)
  std::vector<char> is_consec(steps + 1, 0);
  for (int k = 0; k <= steps; ++k) {
    bool ok = B > 1;
    for (int z = 0; z < Z && ok; ++z) {
      const int32_t* wz = windows_host + ((int64_t)k * Z + z) * B;
      for (int b = 1; b < B && ok; ++b) ok = wz[b] == wz[0] + b;
    }
    for (int z = 0; z < Z; ++z) ptrs[nptr + (int64_t)k * Z + z] = ptrs[((int64_t)k * Z + z) * B];
    is_consec[k] = ok;
  }
  TRY(upload_xtab(c, s, ptrs.data(), (int64_t)ptrs.size()));
  // device table pointers per step: windows [k][Z][B] and (consecutive steps) first windows [k][Z]
  std::vector<const float* const*> xstep(steps + 1, nullptr), consec(steps + 1, nullptr);
  for (int k = 0; k <= steps; ++k) {
    TRY(xtab_at(c, (int64_t)k * Z * B, &xstep[k]));
    if (is_consec[k]) TRY(xtab_at(c, nptr + (int64_t)k * Z, &consec[k]));
  }
  if (!losses) {
    const int64_t need = (int64_t)(steps + 1) * Z;
    if (need > c->scratch_loss_cap) {
      if (c->scratch_loss) HIP_TRY(hipFree(c->scratch_loss));
      HIP_TRY(hipMalloc((void**)&c->scratch_loss, need * 4));
      c->scratch_loss_cap = need;
    }
    losses = c->scratch_loss;
  }
  const int64_t P = c->po.P;
  const float inv = 1.f / ((float)d.N * d.HfC * B);
  const bool dropout = c->p_gcn > 0.f || c->p_lstm > 0.f;
  if (dropout) TRY(upload_task_ids(c, s, Z));
  launch_broadcast(s, theta, P, Z, c->fast);
  const double head_fl = 2.0 * Z * c->w.M * d.HfC * d.H;
  const bool so = order == 2;
  if (so) c->so_fc.assign((size_t)steps, 0);
  for (int k = 0; k < steps; ++k) {
    const float* const* xt = xstep[k];
    if (dropout) set_step_drop(c, k);
    if (so) {
      HIP_TRY(hipMemcpyAsync(c->so_theta + (int64_t)k * Z * P, c->fast, (size_t)Z * P * 4, hipMemcpyDeviceToDevice, s));
      c->w.F = c->so_F ? c->so_F + (int64_t)k * Z * B * d.T * d.N * d.Hc : c->F_main;
    }
    const int slot = steps - 1 - k;
    use_primal(c, slot < nkeep ? slot : SET_MAIN);
    TRY(run_forward(c, s, c->fast, P, xt, consec[k]));
    if (so) c->so_fc[k] = (int8_t)c->w.fcompact;  // (the layout of so_F slot k, for the sweep)
    TIMED(c, s, C_HEAD, head_fl, launch_head_loss(s, d, c->w, c->fast, P, c->po, xt, 2.f * inv, true));
    TIMED(c, s, C_MISC, 0, launch_loss_final(s, c->w, inv, losses + (int64_t)k * Z));
    TRY(run_backward(c, s, c->fast, P, c->grad));
    // the inner SGD step (clip_grad_norm_ + SGD) of every task: one kernel
    if (so) {
      HIP_TRY(hipMemcpyAsync(c->so_grad + (int64_t)k * Z * P, c->grad, (size_t)Z * P * 4, hipMemcpyDeviceToDevice, s));
      TIMED(c, s, C_MISC, 0,
            HIP_TRY(launch_inner_sgd(s, c->fast, c->grad, P, Z, c->w.sqpart, inner_lr, max_norm,
                                     c->so_norm + (int64_t)k * Z, c->so_coef + (int64_t)k * Z, bar_plan(c))));
      if (norms)
        HIP_TRY(hipMemcpyAsync(norms + (int64_t)k * Z, c->so_norm + (int64_t)k * Z, Z * 4, hipMemcpyDeviceToDevice, s));
    } else {
      TIMED(c, s, C_MISC, 0,
            HIP_TRY(launch_inner_sgd(s, c->fast, c->grad, P, Z, c->w.sqpart, inner_lr, max_norm,
                                     norms ? norms + (int64_t)k * Z : nullptr, nullptr, bar_plan(c))));
    }
  }
  const float* const* xq = xstep[steps];
  c->w.F = c->F_main;
  use_primal(c, nkeep > 0 ? SET_QUERY : SET_MAIN);  // slot 0 holds the workspace's own Hs/Cs/Gs
  if (dropout) set_step_drop(c, steps);
  TRY(run_forward(c, s, c->fast, P, xq, consec[steps]));
  TIMED(c, s, C_HEAD, head_fl,
        launch_head_loss(s, d, c->w, c->fast, P, c->po, xq, 2.f * inv * query_scale, true));
  TIMED(c, s, C_MISC, 0, launch_loss_final(s, c->w, inv, losses + (int64_t)steps * Z));
  if (order == 1) {
    TRY(run_backward(c, s, c->fast, P, c->grad));
    TIMED(c, s, C_MISC, 0, launch_sum_tasks(s, c->grad, P, Z, meta_grad));
  } else if (so) {
    // v_K = d(query_scale * L_q)/d theta_K, then back through every inner step:
    //   v_k = v_{k+1} - lr * H_k w_k,  w_k = clip-adjusted v_{k+1}
    if (fast_out) HIP_TRY(hipMemcpyAsync(fast_out, c->fast, (size_t)Z * P * 4, hipMemcpyDeviceToDevice, s));
    fast_out = nullptr;
    TRY(run_backward(c, s, c->fast, P, c->grad));
    use_primal(c, SET_MAIN);
    float* V = c->grad;
    // w_{K-1}: the clip-adjusted direction of the last inner step at v_K (one kernel: dot + direction)
    if (steps > 0)
      TIMED(c, s, C_MISC, 0,
            HIP_TRY(launch_sweep_update(s, V, nullptr, 0.f, c->so_grad + (int64_t)(steps - 1) * Z * P, P, Z,
                                        c->w.sqpart, c->so_norm + (int64_t)(steps - 1) * Z,
                                        c->so_coef + (int64_t)(steps - 1) * Z, max_norm, c->so_u,
                                        bar_plan(c))));
    for (int k = steps - 1; k >= 0; --k) {
      const float* th = c->so_theta + (int64_t)k * Z * P;
      const float* const* xt = xstep[k];
      c->w.F = c->so_F ? c->so_F + (int64_t)k * Z * B * d.T * d.N * d.Hc : c->F_main;
      const int slot = steps - 1 - k;
      use_primal(c, slot < nkeep ? slot : SET_MAIN);
      c->w.primal_kept = slot < nkeep ? 1 : 0;
      if (dropout) set_step_drop(c, k);  // the masks of inner step k's forward
      TRY(run_forward_dual(c, s, th, c->so_u, P, xt, c->so_F != nullptr, consec[k], c->so_fc[k]));
      TIMED(c, s, C_HEAD, 3.0 * head_fl, launch_head_dual(s, d, c->w, th, c->so_u, P, c->po, xt, 2.f * inv));
      TRY(run_backward_dual(c, s, th, c->so_u, P, c->so_hu));
      if (k > 0)  // v_k = v_{k+1} - lr H_k w_k and w_{k-1} (dot g_{k-1} . v_k, direction): one kernel
        TIMED(c, s, C_MISC, 0,
              HIP_TRY(launch_sweep_update(s, V, c->so_hu, -inner_lr, c->so_grad + (int64_t)(k - 1) * Z * P, P, Z,
                                          c->w.sqpart, c->so_norm + (int64_t)(k - 1) * Z,
                                          c->so_coef + (int64_t)(k - 1) * Z, max_norm, c->so_u,
                                          bar_plan(c))));
      else
        TIMED(c, s, C_MISC, 0, launch_axpy(s, V, c->so_hu, (int64_t)Z * P, -inner_lr));
      c->w.primal_kept = 0;
    }
    use_primal(c, SET_MAIN);
    TIMED(c, s, C_MISC, 0, launch_sum_tasks(s, V, P, Z, meta_grad));
    c->w.F = c->F_main;
  }
  if (fast_out) HIP_TRY(hipMemcpyAsync(fast_out, c->fast, (size_t)Z * P * 4, hipMemcpyDeviceToDevice, s));
  c->w.drop = Drop{};
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

// Fill the adaptation feature cache for every window this call reads that it does not hold yet
// (frozen GCN, F2): the missing windows in runs of consecutive starts, each run as ONE GCN pass over
// Z = run-length single-window "tasks" (B = 1), whose [Z][T][N][Hc] output is exactly the run's
// cache slots. Per-row GCN arithmetic does not depend on how many samples a launch holds, so the
// features are bitwise those of the per-step fill (the first epoch no longer runs 960 batch-1 GCNs).
static int ad_cache_fill(smaml_ctx* c, hipStream_t s, const int32_t* windows, int64_t n) {
  const Dims& d = c->d;
  const int64_t fsz = (int64_t)d.T * d.N * d.Hc;
  std::vector<int32_t> need;
  for (int64_t i = 0; i < n; ++i)
    if (!c->ad_valid[windows[i]]) need.push_back(windows[i]);
  if (need.empty()) return SMAML_OK;
  std::sort(need.begin(), need.end());
  need.erase(std::unique(need.begin(), need.end()), need.end());
  std::vector<const float*> ptrs(need.size());
  for (size_t i = 0; i < need.size(); ++i) ptrs[i] = c->feats[0] + (int64_t)need[i] * d.N * d.Cin0;
  TRY(upload_xtab(c, s, ptrs.data(), (int64_t)ptrs.size()));
  for (size_t i = 0; i < need.size();) {
    size_t j = i + 1;
    while (j < need.size() && need[j] == need[j - 1] + 1 && (int)(j - i) < c->ad_gcn_batch) ++j;
    set_work(c, (int)(j - i), 1);
    c->w.F = c->ad_F + (int64_t)need[i] * fsz;
    const float* const* xt = nullptr;
    TRY(xtab_at(c, (int64_t)i, &xt));
    TRY(run_gcn(c, s, xt));
    for (size_t k = i; k < j; ++k) c->ad_valid[need[k]] = 1;
    i = j;
  }
  return SMAML_OK;
}

// Set-up half of smaml_adapt_steps: size the workspace for `B`-sample steps (and, for the batched cache
// fill, ad_gcn_batch single-window "tasks") and allocate the per-window feature cache once per context.
// Both allocations are TOUCHED (memset + stream sync) before returning: the driver may hand out freshly
// released VRAM that it still has to clear, and that clear otherwise lands in the first kernel that
// reads the buffer -- i.e. inside the first timed epoch (round 5: 6.1 s of a 6.8 s first epoch on some
// boxes, 0 on others). Returns with *cache = whether this call's steps use the cache.
static int ad_prepare(smaml_ctx* c, hipStream_t s, int B, bool* cache_out) {
  using clk = std::chrono::steady_clock;
  const Dims& d = c->d;
  auto t0 = clk::now();
  const bool fill_batched = B == 1 && !(c->p_gcn > 0.f) && c->ad_gcn_batch > 1;
  const int64_t had = c->arena_bytes;
  // (the cache fill's GCN passes run ad_gcn_batch windows as tasks: size the workspace for them
  // first, since a growing workspace drops the cache)
  TRY(reserve(c, fill_batched ? c->ad_gcn_batch : 1, B));
  if (c->arena_bytes != had) {
    HIP_TRY(hipMemsetAsync(c->arena, 0, (size_t)c->arena_bytes, s));
    HIP_TRY(hipStreamSynchronize(s));
  }
  auto t1 = clk::now();
  const int64_t fsz = (int64_t)d.T * d.N * d.Hc;  // floats of one window's features
  const int64_t n = c->t_total.empty() ? 0 : c->t_total[0];
  bool cache = B == 1 && !(c->p_gcn > 0.f) && n > 0;
  if (cache && c->ad_F && c->ad_cap < n) ad_cache_drop(c);  // a longer stream than the cache was sized for
  if (cache && !c->ad_F) {
    size_t freeb = 0, totb = 0;
    HIP_TRY(hipMemGetInfo(&freeb, &totb));
    if ((int64_t)freeb > n * fsz * 4 + (8ll << 30) && hipMalloc((void**)&c->ad_F, (size_t)(n * fsz * 4)) == hipSuccess) {
      c->ad_cap = n;
      c->ad_valid.assign((size_t)n, 0);
      HIP_TRY(hipMemsetAsync(c->ad_F, 0, (size_t)(n * fsz * 4), s));
      HIP_TRY(hipStreamSynchronize(s));
    } else {
      (void)hipGetLastError();
      c->ad_F = nullptr;
    }
  }
  auto t2 = clk::now();
  c->ad_ph.ms[AD_RESERVE] += std::chrono::duration<double, std::milli>(t1 - t0).count();
  c->ad_ph.ms[AD_ALLOC] += std::chrono::duration<double, std::milli>(t2 - t1).count();
  *cache_out = cache && c->ad_F;
  return SMAML_OK;
}

int smaml_adapt_prepare(smaml_ctx* c, void* stream, int32_t batch) {
  TRY(require_ready(c));
  if (c->feats.empty()) return fail(SMAML_ESTATE, "smaml_set_tasks not called");
  if (batch <= 0) return fail(SMAML_EINVAL, "bad adapt_prepare batch");
  TRY(ensure_device(c));
  bool cache = false;
  c->ad_ph = AdPhases{};
  return ad_prepare(c, (hipStream_t)stream, batch, &cache);
}

int smaml_adapt_steps(smaml_ctx* c, void* stream, float* theta, float* m, float* v, int32_t step0, int32_t nsteps,
                      int32_t batch, const int32_t* windows_host, const float* lr_dev, float beta1, float beta2,
                      float eps, float weight_decay, float max_norm, float* losses) {
  using clk = std::chrono::steady_clock;
  TRY(require_ready(c));
  if (c->feats.empty()) return fail(SMAML_ESTATE, "smaml_set_tasks not called");
  if (!theta || !m || !v || nsteps <= 0 || batch <= 0 || !windows_host || !lr_dev || !losses || step0 < 0)
    return fail(SMAML_EINVAL, "bad adapt_steps arguments");
  TRY(ensure_device(c));
  hipStream_t s = (hipStream_t)stream;
  const Dims& d = c->d;
  const int B = batch;
  const int64_t nptr = (int64_t)nsteps * B;
  std::vector<const float*> ptrs(nptr);
  for (int64_t i = 0; i < nptr; ++i) {
    const int wv = windows_host[i];
    if (wv < 0 || wv + d.T + d.Hf >= c->t_total[0]) return fail(SMAML_EINVAL, "window start out of range");
    ptrs[i] = c->feats[0] + (int64_t)wv * d.N * d.Cin0;
  }
  c->ad_ph = AdPhases{};
  bool cache = false;
  TRY(ad_prepare(c, s, B, &cache));  // no allocation after smaml_adapt_prepare / an earlier call
  const bool fill_batched = B == 1 && !(c->p_gcn > 0.f) && c->ad_gcn_batch > 1;
  const int64_t P = c->po.P;
  const float inv = 1.f / ((float)d.N * d.HfC * B);
  const bool dropout = c->p_gcn > 0.f || c->p_lstm > 0.f;
  if (dropout) TRY(upload_task_ids(c, s, 1));
  // Batch-1 steps without GCN dropout reuse each window's GCN features across epochs (F2).
  const int64_t fsz = (int64_t)d.T * d.N * d.Hc;  // floats of one window's features
  auto t0 = clk::now();
  if (cache && fill_batched) {
    TRY(ad_cache_fill(c, s, windows_host, nsteps));
    if (c->ad_phase_sync) HIP_TRY(hipStreamSynchronize(s));
  }
  auto t1 = clk::now();
  set_work(c, 1, B);
  TRY(upload_xtab(c, s, ptrs.data(), nptr));
  for (int k = 0; k < nsteps; ++k) {
    const float* const* xt = nullptr;
    TRY(xtab_at(c, (int64_t)k * B, &xt));
    if (dropout) set_step_drop(c, step0 + k);
    if (cache) {
      const int wv = windows_host[k];
      c->w.F = c->ad_F + (int64_t)wv * fsz;
      if (!c->ad_valid[wv]) {
        TRY(run_gcn(c, s, xt));  // writes the window's features straight into its cache slot
        c->ad_valid[wv] = 1;
        c->ad_ph.filled += 1;
      }
      TRY(run_lstm(c, s, theta, 0));
    } else {
      TRY(run_forward(c, s, theta, 0, xt));
    }
    TIMED(c, s, C_HEAD, 2.0 * c->w.M * d.HfC * d.H, launch_head_loss(s, d, c->w, theta, 0, c->po, xt, 2.f * inv, true));
    TRY(run_backward(c, s, theta, 0, c->grad));
    // (the step's loss is summed by the Adam launch's block 0: the backward leaves the head's partials alone)
    TIMED(c, s, C_MISC, 0,
          launch_adam_l2(s, theta, c->grad, m, v, P, c->w.sqpart, lr_dev + k, step0 + k + 1, beta1, beta2, eps,
                         weight_decay, max_norm, c->w.lpart, c->w.lblocks, inv, losses + k));
  }
  if (c->ad_phase_sync) HIP_TRY(hipStreamSynchronize(s));
  auto t2 = clk::now();
  c->ad_ph.ms[AD_FILL] = std::chrono::duration<double, std::milli>(t1 - t0).count();
  c->ad_ph.ms[AD_STEPS] = std::chrono::duration<double, std::milli>(t2 - t1).count();
  c->w.F = c->F_main;
  c->w.drop = Drop{};
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

int smaml_adapt_phases(const smaml_ctx* c, double* ms, int32_t cap, int32_t* count, int64_t* filled) {
  if (!c || cap < 0 || (cap > 0 && !ms)) return fail(SMAML_EINVAL, "bad adapt_phases arguments");
  for (int i = 0; i < AD_NPH && i < cap; ++i) ms[i] = c->ad_ph.ms[i];
  if (count) *count = AD_NPH;
  if (filled) *filled = c->ad_ph.filled;
  return SMAML_OK;
}

int smaml_timing(smaml_ctx* c, int32_t enable) {
  if (!c) return fail(SMAML_EINVAL, "ctx is NULL");
  c->tm.on = enable != 0;
  return SMAML_OK;
}

int smaml_timing_collect(smaml_ctx* c, double* ms, double* flops, int64_t* count, int32_t cap) {
  if (!c) return fail(SMAML_EINVAL, "ctx is NULL");
  TRY(ensure_device(c));
  HIP_TRY(hipDeviceSynchronize());
  for (auto& r : c->tm.recs) {
    float e = 0.f;
    HIP_TRY(hipEventElapsedTime(&e, r.a, r.b));
    c->tm.ms[r.cat] += e;
    c->tm.flops[r.cat] += r.flops;
    c->tm.count[r.cat] += 1;
    c->tm.pool.push_back(r.a);
    c->tm.pool.push_back(r.b);
  }
  c->tm.recs.clear();
  for (int i = 0; i < NCAT && i < cap; ++i) {
    if (ms) ms[i] = c->tm.ms[i];
    if (flops) flops[i] = c->tm.flops[i];
    if (count) count[i] = c->tm.count[i];
    c->tm.ms[i] = 0;
    c->tm.flops[i] = 0;
    c->tm.count[i] = 0;
  }
  return SMAML_OK;
}

int smaml_variant_counts(smaml_ctx* c, int64_t* counts, int32_t cap, int32_t* count, int32_t reset) {
  if (!c || cap < 0 || (cap > 0 && !counts)) return fail(SMAML_EINVAL, "bad variant_counts arguments");
  for (int i = 0; i < NVAR && i < cap; ++i) counts[i] = c->vcount[i];
  if (count) *count = NVAR;
  if (reset)
    for (auto& v : c->vcount) v = 0;
  return SMAML_OK;
}

int smaml_set_option(smaml_ctx* c, const char* key, int64_t value) {
  if (!c || !key) return fail(SMAML_EINVAL, "NULL argument");
  const std::string k(key);
  if (k == "bwd_big_min" && value >= 0) {
    c->kn.bwd_big_min = (int)std::min<int64_t>(value, 1 << 30);
  } else if (k == "bwdd_big_min" && value >= 0) {
    c->kn.bwdd_big_min = (int)std::min<int64_t>(value, 1 << 30);
  } else if (k == "split_max" && value >= 1) {
    c->kn.split_max = (int)std::min<int64_t>(value, 64);
  } else if (k == "wgrad_group_max_rows" && value >= 0) {
    c->kn.wgrad_group_max_rows = (int)std::min<int64_t>(value, 1 << 30);
  } else if (k == "gcn_fused" && (value == 0 || value == 1)) {
    c->kn.gcn_fused = (int)value;
  } else if (k == "gate_img" && (value == 0 || value == 1)) {
    c->kn.gate_img = (int)value;
  } else if (k == "wgrad_wide" && (value == 0 || value == 1)) {
    c->kn.wgrad_wide = (int)value;
  } else if (k == "wgrad_pair" && (value == 0 || value == 1)) {
    c->kn.wgrad_pair = (int)value;
  } else if (k == "bwdd_remap" && (value == 0 || value == 1)) {
    c->kn.bwdd_remap = (int)value;
  } else if (k == "small_kw" && value >= 0 && value <= 2) {
    c->kn.small_kw = (int)value;
  } else if (k == "gcn_dedup" && (value == 0 || value == 1)) {
    c->kn.gcn_dedup = (int)value;
  } else if (k == "xg_dedup" && (value == 0 || value == 1)) {
    c->kn.xg_dedup = (int)value;
  } else if (k == "wgrad_dedup" && (value == 0 || value == 1)) {
    c->kn.wgrad_dedup = (int)value;
  } else if (k == "bptt_streams" && value >= 1 && value <= 4) {
    c->kn.bptt_streams = (int)value;
  } else if (k == "f_compact" && (value == 0 || value == 1)) {
    c->kn.f_compact = (int)value;
  } else if (k == "fwd_streams" && value >= 0 && value <= 4) {
    c->kn.fwd_streams = (int)value;
  } else if (k == "adapt_phase_sync" && (value == 0 || value == 1)) {
    c->ad_phase_sync = (int)value;
  } else if (k == "adapt_gcn_batch" && value >= 0 && value <= 256) {
    c->ad_gcn_batch = (int)value;
  } else if (k == "wgrad_group_wgs" && value >= 1) {
    c->kn.wgrad_group_wgs = (int)std::min<int64_t>(value, 1 << 20);
  } else if (k == "grid_barrier" && (value == 0 || value == 1)) {
    c->bar_fused = (int)value;
  } else if (k == "barrier_timeout_us" && value >= 1) {
    c->bar_timeout_us = std::min<int64_t>(value, 600000000);
  } else if (k == "comm_timeout_ms" && value >= 1) {
    c->comm_timeout_ms = std::min<int64_t>(value, 3600000);
  } else if (k == "barrier_oversize" && value >= 0 && value <= 64) {
    c->bar_oversize = (int)value;
  } else if (k == "keep" && value >= -1) {
    c->keep_max = (int)std::min<int64_t>(value, 1 << 20);
    c->keep_tried_K = -1;  // re-plan the kept slots on the next second-order meta-step
  } else {
    return fail(SMAML_EINVAL, "unknown option or bad value: " + k);
  }
  return SMAML_OK;
}

int smaml_adamw_step(smaml_ctx* c, void* stream, float* theta, const float* grad, float* m, float* v, int64_t n,
                     int32_t step, float lr, float beta1, float beta2, float eps, float weight_decay, float max_norm,
                     float* norm_out) {
  if (!c || !theta || !grad || !m || !v || n <= 0 || step < 1) return fail(SMAML_EINVAL, "bad adamw arguments");
  TRY(ensure_device(c));
  TRY(check_device_error(c));
  TRY(reserve(c, 1, 1));
  hipStream_t s = (hipStream_t)stream;
  const double bc1 = 1.0 - std::pow((double)beta1, step);
  const double bc2 = 1.0 - std::pow((double)beta2, step);
  launch_adamw(s, theta, grad, m, v, n, c->w.sqpart + (int64_t)c->z_cap * SQB, lr, beta1, beta2, eps, weight_decay,
               (float)(lr / bc1), (float)std::sqrt(bc2), max_norm, norm_out);
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}


// ---- finer-grained entry points --------------------------------------

int smaml_backward(smaml_ctx* c, void* stream, const float* theta, const float* dpred, float* grad) {
  TRY(require_ready(c));
  if (!theta || !dpred || !grad) return fail(SMAML_EINVAL, "bad backward arguments");
  if (c->act_B < 1 || c->w.Z != 1) return fail(SMAML_ESTATE, "smaml_backward needs the activations of smaml_forward");
  TRY(ensure_device(c));
  hipStream_t s = (hipStream_t)stream;
  const Dims& d = c->d;
  // dpred [B][N*Hf][C] (rows n*Hf+h) == w.dpred [M = B*N][Hf*C]: same flat order
  HIP_TRY(hipMemcpyAsync(c->w.dpred, dpred, (size_t)c->w.M * d.HfC * 4, hipMemcpyDeviceToDevice, s));
  HIP_TRY(hipMemsetAsync(grad, 0, (size_t)c->po.P * 4, s));
  c->act_B = -1;  // the BPTT overwrites the saved gates with dG
  TRY(run_backward(c, s, theta, 0, grad));
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

int smaml_dropout(smaml_ctx* c, void* stream, float* x, int64_t n, float p, uint32_t seed, int32_t layer) {
  if (!c || !x || n < 0 || !(p >= 0.f && p < 1.f) || layer < 0) return fail(SMAML_EINVAL, "bad dropout arguments");
  TRY(ensure_device(c));
  if (p > 0.f && n > 0) launch_dropout_inplace((hipStream_t)stream, x, n, p, seed, layer);
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

int smaml_gcn_forward(smaml_ctx* c, void* stream, const float* const* x_host, int32_t nsamples, float* feats) {
  TRY(require_ready(c));
  if (!x_host || nsamples <= 0 || !feats) return fail(SMAML_EINVAL, "bad gcn_forward arguments");
  for (int i = 0; i < nsamples; ++i)
    if (!x_host[i] || !aligned16(x_host[i])) return fail(SMAML_EINVAL, "sample x pointers must be 16-B aligned");
  TRY(ensure_device(c));
  hipStream_t s = (hipStream_t)stream;
  TRY(reserve(c, 1, nsamples));
  set_work(c, 1, nsamples);
  TRY(upload_xtab(c, s, x_host, nsamples));
  const float* const* xt = nullptr;
  TRY(xtab_at(c, 0, &xt));
  TRY(run_gcn(c, s, xt));
  const Dims& d = c->d;
  const int64_t blk = (int64_t)d.N * d.Hc;
  for (int si = 0; si < nsamples; ++si)  // F [T][M][Hc] -> feats [s][T*N][Hc]
    HIP_TRY(hipMemcpy2DAsync(feats + (int64_t)si * d.T * blk, blk * 4, c->w.F + (int64_t)si * blk,
                             (int64_t)nsamples * blk * 4, blk * 4, d.T, hipMemcpyDeviceToDevice, s));
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

int smaml_lstm_forward(smaml_ctx* c, void* stream, const float* theta, const float* feats, int32_t nsamples,
                       float* hT) {
  if (!c) return fail(SMAML_EINVAL, "ctx is NULL");
  if (!theta || !feats || nsamples <= 0 || !hT) return fail(SMAML_EINVAL, "bad lstm_forward arguments");
  TRY(ensure_device(c));
  hipStream_t s = (hipStream_t)stream;
  TRY(reserve(c, 1, nsamples));
  set_work(c, 1, nsamples);
  const Dims& d = c->d;
  const int64_t blk = (int64_t)d.N * d.Hc;
  for (int si = 0; si < nsamples; ++si)  // feats [s][T*N][Hc] -> F [T][M][Hc]
    HIP_TRY(hipMemcpy2DAsync(c->w.F + (int64_t)si * blk, (int64_t)nsamples * blk * 4, feats + (int64_t)si * d.T * blk,
                             blk * 4, blk * 4, d.T, hipMemcpyDeviceToDevice, s));
  TRY(run_lstm(c, s, theta, 0));
  const int64_t lsz = (int64_t)d.T * c->w.M * d.H;
  const float* top = c->w.Hs + (int64_t)(d.L - 1) * lsz + (int64_t)(d.T - 1) * c->w.M * d.H;
  HIP_TRY(hipMemcpyAsync(hT, top, (size_t)c->w.M * d.H * 4, hipMemcpyDeviceToDevice, s));
  c->act_B = nsamples;
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

int smaml_lstm_backward(smaml_ctx* c, void* stream, const float* theta, const float* dhT, float* grad) {
  if (!c) return fail(SMAML_EINVAL, "ctx is NULL");
  if (!theta || !dhT || !grad) return fail(SMAML_EINVAL, "bad lstm_backward arguments");
  if (c->act_B < 1 || c->w.Z != 1)
    return fail(SMAML_ESTATE, "smaml_lstm_backward needs the activations of smaml_lstm_forward");
  TRY(ensure_device(c));
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipMemcpyAsync(c->w.dH, dhT, (size_t)c->w.M * c->d.H * 4, hipMemcpyDeviceToDevice, s));
  HIP_TRY(hipMemsetAsync(grad, 0, (size_t)c->po.P * 4, s));
  c->act_B = -1;
  TRY(run_bptt(c, s, theta, 0, grad));
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

int smaml_head_loss(smaml_ctx* c, void* stream, const float* theta, const float* hT, const float* const* y_host,
                    int32_t nsamples, float* pred, float* loss, float* dpred) {
  if (!c) return fail(SMAML_EINVAL, "ctx is NULL");
  if (!theta || !hT || nsamples <= 0 || !pred) return fail(SMAML_EINVAL, "bad head_loss arguments");
  if (y_host && (!loss || !dpred)) return fail(SMAML_EINVAL, "loss and dpred are required with targets");
  if (!aligned16(hT) || !aligned16(theta)) return fail(SMAML_EINVAL, "hT / theta must be 16-byte aligned");
  TRY(ensure_device(c));
  hipStream_t s = (hipStream_t)stream;
  // the head only needs the small per-launch buffers; keep saved LSTM activations intact
  if (nsamples > c->zb_cap) TRY(reserve(c, 1, nsamples));
  const int act = c->act_B;
  const Work saved = c->w;
  set_work(c, 1, nsamples);
  if (y_host) {
    for (int i = 0; i < nsamples; ++i)
      if (!y_host[i]) return fail(SMAML_EINVAL, "null target pointer");
    TRY(upload_xtab(c, s, y_host, nsamples));
  }
  const float* const* yt = nullptr;
  if (y_host) TRY(xtab_at(c, 0, &yt));
  const Dims& d = c->d;
  const float inv = 1.f / ((float)nsamples * d.N * d.HfC);  // mean over samples and elements (F9)
  launch_head_loss_y(s, d, c->w, hT, theta, c->po, yt, pred, dpred, 2.f * inv);
  if (y_host) launch_loss_final(s, c->w, inv, loss);
  c->w = saved;
  c->act_B = act;
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

int smaml_clip_sgd(smaml_ctx* c, void* stream, float* theta, const float* grad, int32_t ntasks, float lr,
                   float max_norm, float* norms) {
  if (!c || !theta || !grad || ntasks <= 0) return fail(SMAML_EINVAL, "bad clip_sgd arguments");
  TRY(ensure_device(c));
  if (ntasks > c->z_cap) TRY(reserve(c, ntasks, 1));
  TRY(ensure_bar(c));
  hipStream_t s = (hipStream_t)stream;
  TRY(check_device_error(c));
  HIP_TRY(launch_inner_sgd(s, theta, grad, c->po.P, ntasks, c->w.sqpart, lr, max_norm, norms, nullptr, bar_plan(c)));
  HIP_TRY(hipGetLastError());
  return SMAML_OK;
}

int smaml_sync(smaml_ctx* c, void* stream) {
  if (!c) return fail(SMAML_EINVAL, "ctx is NULL");
  TRY(ensure_device(c));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  return check_device_error(c);
}

int smaml_inner_loop(smaml_ctx* c, void* stream, const float* theta, int32_t steps, int32_t batch,
                     const int32_t* windows_host, float inner_lr, float max_norm, float* fast_out, float* losses,
                     float* norms) {
  if (!fast_out) return fail(SMAML_EINVAL, "fast_out is required");
  return smaml_meta_step(c, stream, theta, 0, steps, batch, windows_host, inner_lr, max_norm, 1.f, nullptr, losses,
                         norms, fast_out);
}

int smaml_alloc(smaml_ctx* c, int64_t bytes, void** out) {
  if (!c || bytes <= 0 || !out) return fail(SMAML_EINVAL, "bad alloc arguments");
  TRY(ensure_device(c));
  if (hipMalloc(out, (size_t)bytes) != hipSuccess) {
    (void)hipGetLastError();
    *out = nullptr;
    return fail(SMAML_ENOMEM, "hipMalloc of " + std::to_string(bytes) + " B failed");
  }
  return SMAML_OK;
}

int smaml_free(smaml_ctx* c, void* p) {
  if (!c) return fail(SMAML_EINVAL, "ctx is NULL");
  if (!p) return SMAML_OK;
  TRY(ensure_device(c));
  HIP_TRY(hipFree(p));
  return SMAML_OK;
}

}  // extern "C"

// ---- RCCL communicator (one process per GPU). librccl is resolved at first use with dlopen,
// so the library has no link-time RCCL dependency (and shares the process's RCCL if torch
// has already loaded one). Only the handful of symbols below are used.
namespace {
// ncclConfig_t as of NCCL 2.14 (size / magic / version + the first user fields): the library reads only
// the fields the declared version has, so this prefix works with the RCCL torch bundles and /opt/rocm's
struct NcclConfig214 {
  size_t size = sizeof(NcclConfig214);
  unsigned magic = 0xcafebeef;
  unsigned version = 21400;  // NCCL_VERSION(2, 14, 0)
  int blocking = 0;          // non-blocking: ncclCommInitRankConfig returns at once, progress is polled
  int cgaClusterSize = (int)0x80000000, minCTAs = (int)0x80000000, maxCTAs = (int)0x80000000;  // UNDEF_INT
  const char* netName = nullptr;
};
struct Rccl {
  void* h = nullptr;
  int (*get_unique_id)(void*) = nullptr;                                   // ncclGetUniqueId
  int (*comm_init_rank)(void**, int, std::array<char, 128>, int) = nullptr;  // ncclCommInitRank
  int (*comm_init_rank_config)(void**, int, std::array<char, 128>, int, NcclConfig214*) = nullptr;
  int (*get_async_error)(void*, int*) = nullptr;                           // ncclCommGetAsyncError
  int (*comm_abort)(void*) = nullptr;                                      // ncclCommAbort
  int (*all_reduce)(const void*, void*, size_t, int, int, void*, hipStream_t) = nullptr;
  int (*comm_destroy)(void*) = nullptr;
  int (*comm_finalize)(void*) = nullptr;                                   // ncclCommFinalize (optional)
  const char* (*error_string)(int) = nullptr;
  bool nonblocking() const { return comm_init_rank_config && get_async_error && comm_abort; }
};
constexpr int NCCL_FLOAT32 = 7, NCCL_SUM = 0, NCCL_IN_PROGRESS = 7;  // ncclFloat32, ncclSum, ncclInProgress

int rccl(Rccl** out) {
  static Rccl r;
  static bool tried = false;
  if (!tried) {
    tried = true;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      r.h = dlopen(name, RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
      if (!r.h) r.h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
      if (r.h) break;
    }
    if (r.h) {
      r.get_unique_id = (int (*)(void*))dlsym(r.h, "ncclGetUniqueId");
      r.comm_init_rank = (int (*)(void**, int, std::array<char, 128>, int))dlsym(r.h, "ncclCommInitRank");
      r.comm_init_rank_config =
          (int (*)(void**, int, std::array<char, 128>, int, NcclConfig214*))dlsym(r.h, "ncclCommInitRankConfig");
      r.get_async_error = (int (*)(void*, int*))dlsym(r.h, "ncclCommGetAsyncError");
      r.comm_abort = (int (*)(void*))dlsym(r.h, "ncclCommAbort");
      r.all_reduce = (int (*)(const void*, void*, size_t, int, int, void*, hipStream_t))dlsym(r.h, "ncclAllReduce");
      r.comm_destroy = (int (*)(void*))dlsym(r.h, "ncclCommDestroy");
      r.comm_finalize = (int (*)(void*))dlsym(r.h, "ncclCommFinalize");
      r.error_string = (const char* (*)(int))dlsym(r.h, "ncclGetErrorString");
    }
  }
  if (!r.h || !r.get_unique_id || !r.comm_init_rank || !r.all_reduce || !r.comm_destroy)
    return fail(SMAML_ESTATE, "librccl not found (dlopen librccl.so.1)");
  *out = &r;
  return SMAML_OK;
}

int nccl_fail(Rccl* r, int rc, const char* what) {
  return fail(SMAML_EHIP, std::string(what) + ": " + (r->error_string ? r->error_string(rc) : std::to_string(rc)));
}

// A non-blocking communicator's call returned rc: wait (bounded) until its state leaves ncclInProgress.
// Returns the final state (0 = success), or -1 on timeout.
int nccl_wait(Rccl* r, void* comm, int rc, int64_t timeout_ms) {
  if (rc != NCCL_IN_PROGRESS || !comm || !r->get_async_error) return rc;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    int st = 0;
    const int q = r->get_async_error(comm, &st);
    if (q != 0) return q;
    if (st != NCCL_IN_PROGRESS) return st;
    if (std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count() >
        timeout_ms)
      return -1;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}
}  // namespace

extern "C" {

int smaml_comm_unique_id(uint8_t* id_out) {
  if (!id_out) return fail(SMAML_EINVAL, "id_out is NULL");
  Rccl* r = nullptr;
  TRY(rccl(&r));
  const int rc = r->get_unique_id(id_out);
  return rc ? nccl_fail(r, rc, "ncclGetUniqueId") : SMAML_OK;
}

// Bounded: with ncclCommInitRankConfig available the communicator is created non-blocking and its
// progress polled for at most comm_timeout_ms (smaml_set_option "comm_timeout_ms", default 120 s), so a
// rank whose peers never arrive (one of them failed before or inside its init) returns SMAML_EHIP
// instead of blocking forever; the half-built communicator is aborted.
int smaml_comm_init(smaml_ctx* c, int32_t rank, int32_t world, const uint8_t* id) {
  if (!c || !id || world < 1 || rank < 0 || rank >= world) return fail(SMAML_EINVAL, "bad comm_init arguments");
  if (c->comm) return fail(SMAML_ESTATE, "communicator already initialised");
  Rccl* r = nullptr;
  TRY(rccl(&r));
  TRY(ensure_device(c));
  std::array<char, 128> uid;
  std::memcpy(uid.data(), id, 128);
  void* comm = nullptr;
  if (r->nonblocking()) {
    NcclConfig214 cfg;
    int rc = r->comm_init_rank_config(&comm, world, uid, rank, &cfg);
    if (rc != 0 && rc != NCCL_IN_PROGRESS) {
      if (comm) (void)r->comm_abort(comm);
      return nccl_fail(r, rc, "ncclCommInitRankConfig");
    }
    rc = nccl_wait(r, comm, NCCL_IN_PROGRESS, c->comm_timeout_ms);
    if (rc != 0) {
      if (comm) (void)r->comm_abort(comm);
      if (rc < 0)
        return fail(SMAML_EHIP, "ncclCommInitRankConfig: timed out after " + std::to_string(c->comm_timeout_ms) +
                                    " ms waiting for the other ranks (communicator aborted)");
      return nccl_fail(r, rc, "ncclCommInitRankConfig");
    }
    c->comm_nb = 1;
  } else {
    const int rc = r->comm_init_rank(&comm, world, uid, rank);
    if (rc) return nccl_fail(r, rc, "ncclCommInitRank");
    c->comm_nb = 0;
  }
  c->comm = comm;
  return SMAML_OK;
}

int smaml_comm_allreduce(smaml_ctx* c, void* stream, float* buf, int64_t n) {
  if (!c || !buf || n < 0) return fail(SMAML_EINVAL, "bad allreduce arguments");
  if (!c->comm) return fail(SMAML_ESTATE, "smaml_comm_init not called");
  Rccl* r = nullptr;
  TRY(rccl(&r));
  TRY(ensure_device(c));
  int rc = r->all_reduce(buf, buf, (size_t)n, NCCL_FLOAT32, NCCL_SUM, c->comm, (hipStream_t)stream);
  if (c->comm_nb) rc = nccl_wait(r, c->comm, rc, c->comm_timeout_ms);  // enqueue completes (not the collective)
  if (rc < 0) return fail(SMAML_EHIP, "ncclAllReduce: enqueue timed out");
  return rc ? nccl_fail(r, rc, "ncclAllReduce") : SMAML_OK;
}

int smaml_comm_destroy(smaml_ctx* c) {
  if (!c) return fail(SMAML_EINVAL, "ctx is NULL");
  if (!c->comm) return SMAML_OK;
  Rccl* r = nullptr;
  TRY(rccl(&r));
  void* comm = c->comm;
  c->comm = nullptr;
  if (c->comm_nb && r->comm_finalize) {
    // non-blocking protocol: finalize (flushes outstanding work, reports its errors), poll it to completion
    // under the same bound as the init, then destroy; a finalize that never completes is aborted
    int rc = nccl_wait(r, comm, r->comm_finalize(comm), c->comm_timeout_ms);
    if (rc != 0) {
      (void)r->comm_abort(comm);
      if (rc < 0)
        return fail(SMAML_EHIP, "ncclCommFinalize: timed out after " + std::to_string(c->comm_timeout_ms) +
                                    " ms (communicator aborted)");
      return nccl_fail(r, rc, "ncclCommFinalize");
    }
  }
  int rc = r->comm_destroy(comm);
  if (c->comm_nb && rc == NCCL_IN_PROGRESS) rc = 0;  // (after finalize the destroy only frees resources)
  return rc ? nccl_fail(r, rc, "ncclCommDestroy") : SMAML_OK;
}

}  // extern "C"
