// Host-logic checks of libsmaml's C ABI under AddressSanitizer + UBSan (a CPU sanitizer
// build of the host C++). Built by tests/test_host_sanitize_cpu.py from the library's own sources
// (api.cpp with -fsanitize on the host side only, the kernel units host-only), run without a GPU.
// Covers the code that validates and transforms caller input before any launch: dimension checks,
// the parameter layout (state_dict order, 64-float padded offsets), the normalised ELL build of the
// graph (gcn_norm with self loops, in-degree limit), and the error paths of the entry points
// (NULL handles / buffers, no device). Round 5: also the launch-plan builders every kernel launch
// depends on (kernels.h: the LSTM wavefront diagonals, the split-K weight-gradient plans and their
// pairing, the grid-barrier sizing), built with -Werror=missing-field-initializers, each plan checked
// field by field against what was asked for. Exit status 0 = every check passed.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <set>
#include <utility>
#include <vector>

#include "kernels.h"
#include "smaml.h"

static int failures = 0;
#define CHECK(cond)                                                 \
  do {                                                              \
    if (!(cond)) {                                                  \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                   \
    }                                                               \
  } while (0)

static smaml_dims dims_cfg2() {
  smaml_dims d;
  d.num_nodes = 441;
  d.window_size = 24;
  d.input_channels = 24;
  d.hidden_channels = 256;
  d.lstm_hidden_size = 128;
  d.lstm_num_layers = 4;
  d.forecast_horizon = 8;
  d.output_channels = 12;
  return d;
}

// 4-neighbour grid graph (both directions), edge_index [2][E]
static std::vector<int64_t> grid_edges(int side) {
  std::vector<int64_t> src, dst;
  for (int r = 0; r < side; ++r)
    for (int c = 0; c < side; ++c) {
      const int i = r * side + c;
      const int nb[4][2] = {{r - 1, c}, {r + 1, c}, {r, c - 1}, {r, c + 1}};
      for (auto& q : nb)
        if (q[0] >= 0 && q[0] < side && q[1] >= 0 && q[1] < side) {
          src.push_back(q[0] * side + q[1]);
          dst.push_back(i);
        }
    }
  std::vector<int64_t> ei(src);
  ei.insert(ei.end(), dst.begin(), dst.end());
  return ei;
}

static smaml::Dims kdims_cfg2() {
  smaml::Dims d;
  d.N = 441;
  d.T = 24;
  d.Cin0 = 24;
  d.Hc = 256;
  d.H = 128;
  d.L = 4;
  d.Hf = 8;
  d.C = 12;
  d.HfC = 96;
  return d;
}

// The wavefront diagonals cover every (layer, step) exactly once, each problem's dependencies lie on
// earlier diagonals, and the block ranges are disjoint, increasing multiples of the per-problem count.
static void check_waves() {
  using namespace smaml;
  const Dims d = kdims_cfg2();
  Work w;
  w.Z = 5;
  w.B = 32;
  w.M = w.B * d.N;
  ParamOff po;
  for (int l = 0; l < d.L; ++l) po.lay[l].cin = l == 0 ? d.Hc : d.H;
  std::set<std::pair<int, int>> fwd, bwd;
  double ffl = 0.0, bfl = 0.0;
  for (int diag = 0; diag < d.T + d.L - 1; ++diag) {
    FwdWave wv;
    ffl += fwd_wave(d, w, po, diag, 16, false, wv);
    CHECK(wv.n >= 1 && wv.n <= d.L && wv.off[0] == 0);
    for (int q = 0; q < wv.n; ++q) {
      CHECK(wv.l[q] + wv.t[q] == diag && wv.l[q] >= 0 && wv.l[q] < d.L && wv.t[q] >= 0 && wv.t[q] < d.T);
      CHECK(wv.off[q + 1] - wv.off[q] == 16);
      CHECK(fwd.insert({wv.l[q], wv.t[q]}).second);
      CHECK(wv.lo[q].cin == po.lay[wv.l[q]].cin);
    }
    BwdWave bv;
    bfl += bwd_wave(d, w, po, diag, 16, false, bv);
    CHECK(bv.n >= 1 && bv.n <= d.L && bv.off[0] == 0);
    for (int q = 0; q < bv.n; ++q) {
      CHECK((d.L - 1 - bv.l[q]) + (d.T - 1 - bv.t[q]) == diag);
      CHECK(bv.off[q + 1] - bv.off[q] == 16);
      CHECK(bwd.insert({bv.l[q], bv.t[q]}).second);
    }
  }
  CHECK((int)fwd.size() == d.L * d.T && (int)bwd.size() == d.L * d.T);
  // LSTM fwd = 2 T N 4H (Hc + H) + 2 T N 4H 2H (L - 1) per sample, less the recurrent
  // products of the t = 0 steps (h_{-1} = 0: not executed, not counted)
  const double lstm = 2.0 * d.T * d.N * 4 * d.H * (d.Hc + d.H) + 2.0 * d.T * d.N * 4 * d.H * 2 * d.H * (d.L - 1) -
                      2.0 * d.N * 4 * d.H * d.H * d.L;
  CHECK(std::fabs(ffl - lstm * w.Z * w.B) <= 1e-9 * ffl);
  CHECK(bfl > 0.0);
}

// plan_wgrad fills every field from its arguments, its K slices cover [0, K) exactly, and its partial
// slabs fit the buffer; pair_wgrad keeps both halves inside the buffer or leaves the plan unchanged.
static void check_wgrad_plans() {
  using namespace smaml;
  Work w;
  w.Z = 5;
  w.B = 32;
  w.M = w.B * 441;
  w.wpart_floats = (int64_t)w.Z * 512 * (256 + 128 + 1) * SMAML_WGRAD_MAXSPLIT;
  w.wpart = reinterpret_cast<float*>(0x1000);
  w.kn.wgrad_wide = 1;
  const float* A = reinterpret_cast<const float*>(0x2000);
  const float* B1 = reinterpret_cast<const float*>(0x3000);
  const float* B2 = reinterpret_cast<const float*>(0x4000);
  float* grad = reinterpret_cast<float*>(0x5000);
  struct Case {
    int Mrows, c1, c2;
    int64_t K;
  } cases[] = {{512, 256, 128, 24LL * 14112}, {512, 128, 128, 24LL * 14112}, {96, 128, 0, 14112},
               {512, 128, 128, 24LL * 441}, {512, 256, 128, 16}, {96, 128, 0, 1}};
  for (const Case& k : cases) {
    WgradPlan p;
    plan_wgrad(w, A, 11, k.Mrows, B1, 12, k.c1, k.c2 ? B2 : nullptr, 13, k.c2, k.K, 7, grad, 606336, 100, 200, 300,
               400, true, false, p);
    CHECK(p.A == A && p.a_zstride == 11 && p.Mrows == k.Mrows && p.B1 == B1 && p.c1 == k.c1 && p.c2 == k.c2);
    CHECK(p.B2 == (k.c2 ? B2 : nullptr) && p.b1_zstride == 12 && p.b2_zstride == 13 && p.K == k.K && p.Mshift == 7);
    CHECK(p.grad == grad && p.P == 606336 && p.off_w1 == 100 && p.off_w2 == 200 && p.off_b1 == 300 && p.off_b2 == 400);
    CHECK(p.with_bias && !p.accumulate && p.Z == w.Z && p.part == w.wpart && p.ldp == k.c1 + k.c2 + 1);
    CHECK(p.ntm >= 1 && p.ntn >= 1 && p.nsplit >= 1 && p.kchunk >= 1);
    CHECK((int64_t)p.nsplit * p.kchunk >= k.K && (int64_t)(p.nsplit - 1) * p.kchunk < k.K);
    CHECK((int64_t)p.nsplit * p.Z * p.Mrows * p.ldp <= w.wpart_floats);
    CHECK(p.A2 == nullptr && p.nsplit1 == 0 && p.drop_layer == -1 && p.drop.thr_lstm == 0);
    WgradPlan q = p;
    if (pair_wgrad(q, w, A, B1, B2)) {
      CHECK(q.nsplit == 2 * q.nsplit1 && q.A2 == A && q.B1s == B1 && q.B2s == B2);
      CHECK((int64_t)q.nsplit1 * q.kchunk >= k.K && (int64_t)(q.nsplit1 - 1) * q.kchunk < k.K);
      CHECK((int64_t)q.nsplit * q.Z * q.Mrows * q.ldp <= w.wpart_floats);
    } else {
      CHECK(q.nsplit == p.nsplit && q.kchunk == p.kchunk && q.A2 == nullptr);
    }
  }
  // a slab buffer too small for two slices: the pair is refused, the plan stays as planned
  Work tiny = w;
  tiny.wpart_floats = (int64_t)w.Z * 512 * 385;
  WgradPlan p;
  plan_wgrad(tiny, A, 0, 512, B1, 0, 256, B2, 0, 128, 24LL * 14112, 0, grad, 0, 0, 0, 0, 0, true, false, p);
  CHECK(p.nsplit == 1);
  CHECK(!pair_wgrad(p, tiny, A, B1, B2) && p.nsplit == 1 && p.A2 == nullptr);
}

static void check_barrier_grid() {
  using smaml::grid_barrier_grid;
  CHECK(grid_barrier_grid(0, 100, 0) == 0);      // capacity unknown: the two-launch form
  CHECK(grid_barrier_grid(1024, 0, 0) == 0);
  CHECK(grid_barrier_grid(1024, 100, 0) == 100);  // fewer items than a quarter of the capacity
  CHECK(grid_barrier_grid(1024, 5000, 0) == 256);
  CHECK(grid_barrier_grid(3, 5000, 0) == 1);
  CHECK(grid_barrier_grid(1024, 5000, 2) == 2049);  // debug oversize: never co-resident
}

int main() {
  CHECK(smaml_abi_version() == 7);
  check_waves();
  check_wgrad_plans();
  check_barrier_grid();
  CHECK(smaml_build_info() != nullptr && std::strlen(smaml_build_info()) > 0);

  // ---- parameter layout (hybrid_model.py state_dict order) ----
  smaml_dims d = dims_cfg2();
  int32_t count = 0;
  int64_t total = 0;
  CHECK(smaml_param_layout(&d, 0, nullptr, nullptr, 0, &count, &total) == 0);
  CHECK(count == 4 * 4 + 2);  // 4 LSTM layers x (W_ih, W_hh, b_ih, b_hh) + head weight, bias
  std::vector<int64_t> off(count), sz(count);
  CHECK(smaml_param_layout(&d, 0, off.data(), sz.data(), count, &count, &total) == 0);
  int64_t nvalid = 0;
  for (int i = 0; i < count; ++i) {
    nvalid += sz[i];
    CHECK(off[i] % 64 == 0);
    if (i) CHECK(off[i] >= off[i - 1] + sz[i - 1]);
  }
  CHECK(nvalid == 606304);  // the 18 trainable tensors
  CHECK(total >= nvalid && total % 64 == 0);
  CHECK(sz[0] == 4 * 128 * 256 && sz[1] == 4 * 128 * 128 && sz[count - 2] == 96 * 128 && sz[count - 1] == 96);
  // a short caller buffer: count and total still reported, only `cap` entries written
  std::vector<int64_t> off2(3, -1);
  CHECK(smaml_param_layout(&d, 0, off2.data(), nullptr, 3, &count, &total) == 0 && count == 18 && off2[2] >= 0);
  CHECK(smaml_param_layout(&d, 1, nullptr, nullptr, 0, &count, &total) == 0 && count == 8);
  CHECK(smaml_param_layout(&d, 2, nullptr, nullptr, 0, &count, &total) == SMAML_EINVAL);
  CHECK(smaml_param_layout(nullptr, 0, nullptr, nullptr, 0, &count, &total) == SMAML_EINVAL);
  smaml_dims bad = d;
  bad.num_nodes = 0;
  CHECK(smaml_param_layout(&bad, 0, nullptr, nullptr, 0, &count, &total) == SMAML_EINVAL);
  bad = d;
  bad.lstm_hidden_size = 100;
  CHECK(smaml_param_layout(&bad, 0, nullptr, nullptr, 0, &count, &total) == SMAML_EINVAL);
  bad = d;
  bad.hidden_channels = 30;
  CHECK(smaml_param_layout(&bad, 0, nullptr, nullptr, 0, &count, &total) == SMAML_EINVAL);
  bad = d;
  bad.lstm_num_layers = 99;
  CHECK(smaml_param_layout(&bad, 0, nullptr, nullptr, 0, &count, &total) == SMAML_EINVAL);
  bad = d;
  bad.output_channels = 48;
  CHECK(smaml_param_layout(&bad, 0, nullptr, nullptr, 0, &count, &total) == SMAML_EINVAL);
  CHECK(std::strlen(smaml_last_error()) > 0);

  // ---- normalised ELL of the graph (PyG gcn_norm: self loops, D^-1/2 (A + I) D^-1/2) ----
  const int side = 21, N = side * side, W = 8;
  std::vector<int64_t> ei = grid_edges(side);
  const int64_t E = (int64_t)ei.size() / 2;
  std::vector<int32_t> cols((size_t)N * W, -1);
  std::vector<float> vals((size_t)N * W, -1.f);
  CHECK(smaml_graph_ell(ei.data(), E, N, cols.data(), vals.data()) == 0);
  std::vector<int> deg(N, 1);
  for (int64_t e = 0; e < E; ++e) deg[ei[E + e]] += 1;
  for (int i = 0; i < N; ++i) {
    bool self = false;
    double wsum = 0.0;
    for (int j = 0; j < W; ++j) {
      const int32_t cidx = cols[(size_t)i * W + j];
      CHECK(cidx >= 0 && cidx < N);
      const float v = vals[(size_t)i * W + j];
      CHECK(std::isfinite(v) && v >= 0.f);
      if (v == 0.f) continue;
      if (cidx == i) {
        self = true;
        CHECK(std::fabs(v - 1.f / deg[i]) < 1e-6f);
      } else {
        CHECK(std::fabs(v - 1.f / std::sqrt((float)deg[i] * (float)deg[cidx])) < 1e-6f);
      }
      wsum += v;
    }
    CHECK(self);
    CHECK(wsum > 0.0);
  }
  // no edges: the self loop alone (weight 1)
  CHECK(smaml_graph_ell(ei.data(), 0, N, cols.data(), vals.data()) == 0);
  CHECK(cols[0] == 0 && vals[0] == 1.f && vals[1] == 0.f);
  // a node id outside [0, N) and an in-degree above the ELL width are rejected
  std::vector<int64_t> badei = {0, 1, 1, N};
  CHECK(smaml_graph_ell(badei.data(), 2, N, cols.data(), vals.data()) == SMAML_EINVAL);
  badei = {-1, 0, 0, 1};
  CHECK(smaml_graph_ell(badei.data(), 2, N, cols.data(), vals.data()) == SMAML_EINVAL);
  std::vector<int64_t> star;  // 8 in-edges into node 0
  for (int k = 1; k <= 8; ++k) star.push_back(k);
  for (int k = 1; k <= 8; ++k) star.push_back(0);
  CHECK(smaml_graph_ell(star.data(), 8, N, cols.data(), vals.data()) == SMAML_EINVAL);
  CHECK(smaml_graph_ell(nullptr, 2, N, cols.data(), vals.data()) == SMAML_EINVAL);
  CHECK(smaml_graph_ell(ei.data(), E, 0, cols.data(), vals.data()) == SMAML_EINVAL);

  // ---- entry points on a NULL handle / without a device ----
  smaml_ctx* ctx = nullptr;
  const int rc = smaml_create(&d, 0, &ctx);
  if (rc == 0) {  // a device is present: the handle must be usable and destroyable
    CHECK(ctx != nullptr);
    CHECK(smaml_set_option(ctx, "no_such_knob", 1) == SMAML_EINVAL);
    CHECK(smaml_set_option(ctx, "keep", -2) == SMAML_EINVAL);
    CHECK(smaml_set_dropout(ctx, 1.5f, 0.f, 0) == SMAML_EINVAL);
    CHECK(smaml_destroy(ctx) == 0);
  } else {
    CHECK(ctx == nullptr);
    CHECK(rc == SMAML_EINVAL || rc == SMAML_EHIP);
  }
  CHECK(smaml_create(&d, -1, &ctx) != 0);
  CHECK(smaml_create(&bad, 0, &ctx) == SMAML_EINVAL);
  CHECK(smaml_create(&d, 0, nullptr) == SMAML_EINVAL);
  CHECK(smaml_destroy(nullptr) == 0);
  int32_t ids[2] = {0, 1};
  CHECK(smaml_set_task_ids(nullptr, ids, 2) == SMAML_EINVAL);
  CHECK(smaml_set_dropout(nullptr, 0.1f, 0.1f, 1) == SMAML_EINVAL);
  CHECK(smaml_set_option(nullptr, "keep", 1) == SMAML_EINVAL);
  CHECK(smaml_sync(nullptr, nullptr) == SMAML_EINVAL);
  CHECK(smaml_set_option(nullptr, "barrier_timeout_us", 1000) == SMAML_EINVAL);
  CHECK(smaml_meta_step(nullptr, nullptr, nullptr, 2, 1, 1, nullptr, 0.01f, 1.f, 0.5f, nullptr, nullptr, nullptr,
                        nullptr) == SMAML_EINVAL);
  CHECK(smaml_reserve(nullptr, 1, 1) == SMAML_EINVAL);
  CHECK(smaml_set_graph(nullptr, ei.data(), E) == SMAML_EINVAL);
  CHECK(smaml_variant_counts(nullptr, nullptr, 0, nullptr, 0) == SMAML_EINVAL);
  CHECK(smaml_workspace_bytes(nullptr) == 0 && smaml_so_kept_steps(nullptr) == 0);

  if (failures) std::fprintf(stderr, "%d check(s) failed\n", failures);
  else std::printf("host sanitize checks: all passed\n");
  return failures ? 1 : 0;
}
