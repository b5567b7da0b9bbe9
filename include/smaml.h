/*
 * smaml.h -- C ABI of libsmaml.so, the MI355X (gfx950) STGCN-LSTM MAML hot path.
 *
 * The reference (Yalt8826/WeatherForecast_STGCN_MAML) is pure Python with no FFI layer;
 * its boundary for this path is the module API of model.py / hybrid_model.py and the
 * train loop entry points of train_hybrid_maml_v5.py. Each entry point below names the
 * reference interface it replaces. The Python host package
 * (weatherforecast_stgcn_maml_amd/_capi.py) binds these with ctypes; INTEGRATION.md
 * shows the binding.
 *
 * Conventions
 *  - Every function returns an int status: 0 = OK, else an SMAML_E* code;
 *    smaml_last_error() returns the message of the calling thread's last failure.
 *  - Device buffers are caller-owned device pointers (e.g. torch tensors' data_ptr()),
 *    fp32, contiguous. Host arrays are marked _host.
 *  - `stream` is a hipStream_t passed as void* (NULL = default stream). All work is
 *    enqueued on it; no call synchronises the device unless documented.
 *  - A context is bound to one GPU, is not thread-safe, and is driven by one host thread.
 *  - Trainable parameters (LSTM + head, the only tensors that receive gradients: SURVEY
 *    F2) live in one flat "theta" vector in state_dict order; smaml_param_layout gives
 *    each tensor's offset (offsets are padded to 64 floats; pads must be zero).
 */
#ifndef SMAML_H
#define SMAML_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SMAML_OK 0
#define SMAML_EINVAL 1   /* bad argument / shape */
#define SMAML_EHIP 2     /* HIP runtime error */
#define SMAML_ENOMEM 3   /* device allocation failed */
#define SMAML_ESTATE 4   /* missing set_graph / set_gcn_params / reserve / set_tasks */
#define SMAML_ENOTIMPL 5 /* requested mode not built */

typedef struct smaml_ctx smaml_ctx;

/* Model shapes: model.STGCN(...) (model.py:8-28) + HybridSTGCN_LSTM(...) (hybrid_model.py:16-58). */
typedef struct smaml_dims {
  int32_t num_nodes;         /* N: grid nodes per region (441 = 21x21) */
  int32_t window_size;       /* T (24) */
  int32_t input_channels;    /* 24 */
  int32_t hidden_channels;   /* GCN hidden (256) */
  int32_t lstm_hidden_size;  /* 128 (multiple of 32) */
  int32_t lstm_num_layers;   /* 4 */
  int32_t forecast_horizon;  /* 8 */
  int32_t output_channels;   /* 12 */
} smaml_dims;

const char* smaml_last_error(void);
int32_t smaml_abi_version(void);
/* Build description: the product form of each GEMM family (bf16x6 = each f32 operand split into
 * three bf16 pieces, six piece products on v_mfma_f32_32x32x16_bf16 accumulated in f32; or the
 * f32 MFMA). Host-only, no GPU needed. */
const char* smaml_build_info(void);

/* ---- host-only helpers (no GPU needed) ------------------------------------------ */

/* Flat layout of the trainable vector (which=0: lstm.* then output_layer.*, the order of
 * HybridSTGCN_LSTM.get_trainable_parameters(), hybrid_model.py:119-124) or of the frozen
 * GCN vector (which=1: base_stgcn.conv{1..4}.{bias,lin.weight}). Writes up to `cap`
 * offsets/sizes, *count tensors and *total padded floats. */
int smaml_param_layout(const smaml_dims* dims, int32_t which, int64_t* offsets, int64_t* sizes,
                       int32_t cap, int32_t* count, int64_t* total);

/* Normalised t=0 adjacency of PyG gcn_norm as ELL (width 8): replaces the
 * add_remaining_self_loops + degree + norm part of GCNConv (model.py:23-26) for the
 * edge_index of graphBuilder.build_spatial_graph (graphBuilder.py:9-47). */
int smaml_graph_ell(const int64_t* edge_index_host, int64_t num_edges, int32_t num_nodes,
                    int32_t* cols_host, float* vals_host);

/* ---- context ----------------------------------------------------------------------- */
int smaml_create(const smaml_dims* dims, int32_t device, smaml_ctx** out);
int smaml_destroy(smaml_ctx* ctx);

/* Upload the graph (edge_index [2, E] int64, host). */
int smaml_set_graph(smaml_ctx* ctx, const int64_t* edge_index_host, int64_t num_edges);

/* Frozen GCN parameters (flat, layout which=1), device pointer kept by reference. */
int smaml_set_gcn_params(smaml_ctx* ctx, const float* gcn_flat);

/* Size the workspace for `tasks` x `batch` samples per step (grows, never shrinks). */
int smaml_reserve(smaml_ctx* ctx, int32_t tasks, int32_t batch);

/* Bytes of device workspace currently held. */
int64_t smaml_workspace_bytes(const smaml_ctx* ctx);

/* Inner steps whose primal activations the last second-order smaml_meta_step kept for its
 * meta-backward sweep (tangent-only dual kernels there; the rest are recomputed). Sized to
 * free HBM, capped by smaml_set_option("keep") / the SMAML_KEEP environment variable. New; no reference counterpart. */
int32_t smaml_so_kept_steps(const smaml_ctx* ctx);

/* Train-mode dropout of smaml_meta_step / smaml_adapt_steps (replaces the nn.Dropout calls at
 * hybrid_model.py:67,70,73 (p_gcn = STGCN dropout_rate), the nn.LSTM inter-layer dropout
 * hybrid_model.py:42-49 and the head input dropout :108 (p_lstm = lstm_dropout)). Masks are
 * counter-based (seed, global task id, inner step, site, element), identical in the
 * forward, the backward and the second-order sweep; p = 0 (the default) disables them.
 * The reference draws masks from torch's RNG, so runs agree with it only at p = 0. */
int smaml_set_dropout(smaml_ctx* ctx, float p_gcn, float p_lstm, uint32_t seed);

/* Global task id of each task of the next smaml_set_tasks batch (the dropout masks' task
 * index, so a task's masks do not depend on how tasks are grouped or sharded). */
int smaml_set_task_ids(smaml_ctx* ctx, const int32_t* ids_host, int32_t n);

/* ---- forward (module API) ----------------------------------------------------------- */

/* GCNConv.forward(x, edge_index) (PyG semantics, F3): x [rows, cin] -> out [rows, cout].
 * Rows < num_nodes aggregate over the graph, the rest see only their self loop. */
int smaml_gcn_conv(smaml_ctx* ctx, void* stream, const float* x, int32_t rows, int32_t cin,
                   const float* weight, const float* bias, int32_t cout, float* out);

/* GCNConv / Linear forward and backward for the module API's autograd (model.py:7-52: STGCN trained on
 * its own; the hybrid path keeps the GCN frozen, F2). flags: SMAML_GCN_RELU applies ReLU to the output,
 * SMAML_GCN_PLAIN skips the graph aggregation (a plain x W^T + b, e.g. STGCN.output_layer). */
#define SMAML_GCN_RELU 1
#define SMAML_GCN_PLAIN 2
int smaml_gcn_conv_ex(smaml_ctx* ctx, void* stream, const float* x, int32_t rows, int32_t cin,
                      const float* weight, const float* bias, int32_t cout, int32_t flags, float* out);

/* Backward of z = A_hat x W^T + b (SMAML_GCN_PLAIN: A_hat = I) given dz = dL/dz [rows][cout]:
 * dx = A_hat^T dz W [rows][cin] (optional), dwb = [dL/dW (cout x cin, row-major) | dL/db (cout)]
 * (optional). Deterministic (fixed-order sums). Replaces autograd through PyG GCNConv / nn.Linear. */
int smaml_gcn_conv_backward(smaml_ctx* ctx, void* stream, const float* x, int32_t rows, int32_t cin,
                            const float* weight, int32_t cout, const float* dz, int32_t flags, float* dx, float* dwb);

/* g *= (h > 0) over n elements: the ReLU derivative from the post-activation h (F.relu's backward). */
int smaml_relu_mask(smaml_ctx* ctx, void* stream, float* g, const float* h, int64_t n);

/* HybridSTGCN_LSTM.forward(x, edge_index) (hybrid_model.py:80-117) for `nsamples` samples:
 * x_host[s] = device pointer to sample s's x [T*N, input_channels] (time-major rows);
 * pred [nsamples][N*Hf][C] (rows n*Hf + h); feats (optional) [nsamples][T*N][Hc] = the
 * extract_base_features output (hybrid_model.py:60-78). With smaml_set_dropout p > 0 this is the
 * train-mode forward (masks of (seed, task id 0 of smaml_set_task_ids, step 0)); the following
 * smaml_backward applies the same masks. */
int smaml_forward(smaml_ctx* ctx, void* stream, const float* theta, const float* const* x_host,
                  int32_t nsamples, float* pred, float* feats);

/* ---- training ------------------------------------------------------------------------ */

/* Register the tasks' feature streams: features_host[j] = device pointer to a
 * [t_total[j], N, input_channels] stream (WeatherGraphDataset.features, dataset.py:6-25).
 * A sample is addressed by its window start w: x = stream[w:w+T], targets
 * stream[w+T+1 .. w+T+Hf, :, :C] (dataset.py:30-48, F5). */
int smaml_set_tasks(smaml_ctx* ctx, int32_t ntasks, const float* const* features_host,
                    const int32_t* t_total_host);

/* One meta-step over all registered tasks (meta_update_v4, train_hybrid_maml_v5.py:144-184,
 * wrapping inner_loop_v4, :110-141):
 *   per task: fast = theta; for k < steps: B-sample support step (mean MSE, backward,
 *   clip_grad_norm_(max_norm), SGD(inner_lr)); then one B-sample query batch.
 * windows_host: int32 [(steps+1)][ntasks][batch] window starts (row `steps` = query).
 * order 0: reference semantics (the reference's outer step is a no-op):
 *          query loss only; order 1: first-order MAML meta-gradient; order 2: second-order.
 * meta_grad [P]: sum over tasks of d(query_scale * query_mse)/d(theta) (order >= 1).
 * losses [(steps+1)][ntasks]: per-step support MSE; last row = query MSE (unscaled).
 * norms [steps][ntasks] (optional): pre-clip gradient norms. fast_out [ntasks][P]
 * (optional): adapted parameters. */
int smaml_meta_step(smaml_ctx* ctx, void* stream, const float* theta, int32_t order, int32_t steps,
                    int32_t batch, const int32_t* windows_host, float inner_lr, float max_norm,
                    float query_scale, float* meta_grad, float* losses, float* norms, float* fast_out);

/* Outer update (train_hybrid_maml_v5.py:174-179, 245-249): clip_grad_norm_(max_norm) of
 * `grad` then torch.optim.AdamW step `step` (1-based) on theta, m, v (n floats).
 * norm_out (optional, device float): pre-clip norm. */
int smaml_adamw_step(smaml_ctx* ctx, void* stream, float* theta, const float* grad, float* m, float* v,
                     int64_t n, int32_t step, float lr, float beta1, float beta2, float eps,
                     float weight_decay, float max_norm, float* norm_out);

/* Regional adaptation (adapt_hybrid_v5.adaptModel, adapt_hybrid_v5.py:182-203): `nsteps`
 * sequential fine-tuning steps on task 0 of smaml_set_tasks, each on `batch` windows
 * (windows_host [nsteps][batch]; the reference uses batch 1, shuffled): forward, MSE,
 * backward, clip_grad_norm_(max_norm), torch.optim.Adam with coupled L2 weight decay
 * (create_climate_optimizer, adaptive_scheduler.py:68-94) at learning rate lr_dev[k]
 * (device floats; ClimateAwareLRScheduler values) and Adam step step0+k+1.
 * theta, m, v: flat trainable vectors (device). losses [nsteps] (device): per-step MSE.
 * At batch 1 without GCN dropout each window's GCN features are cached on first use and reused
 * by later calls (frozen GCN): call smaml_set_gcn_params again after changing the GCN
 * parameters in place (it, smaml_set_graph and smaml_set_tasks drop the cache). */
int smaml_adapt_steps(smaml_ctx* ctx, void* stream, float* theta, float* m, float* v, int32_t step0,
                      int32_t nsteps, int32_t batch, const int32_t* windows_host, const float* lr_dev,
                      float beta1, float beta2, float eps, float weight_decay, float max_norm,
                      float* losses);

/* Set-up half of smaml_adapt_steps, for callers that keep allocation out of their timed epochs
 * (adaptModel builds its model and optimiser before the epoch loop, adapt_hybrid_v5.py:152-181):
 * sizes the workspace for `batch`-sample steps and allocates the per-window GCN feature cache
 * (batch 1), touching both once and synchronising `stream`. smaml_adapt_steps does the same on its
 * first call when this was not called. No compute; the cache stays cold. */
int smaml_adapt_prepare(smaml_ctx* ctx, void* stream, int32_t batch);

/* Host-timed phases of the last smaml_adapt_steps call, in ms: [0] workspace reserve, [1] feature-
 * cache allocation, [2] the batched feature-cache fill, [3] the step loop ([2] and [3] are enqueue
 * times unless smaml_set_option("adapt_phase_sync", 1), which ends each with a stream sync).
 * Writes min(cap, count) entries; *count = number of phases; *filled = windows whose features a
 * step computed itself (outside the batched fill). Measurement only; no reference counterpart. */
int smaml_adapt_phases(const smaml_ctx* ctx, double* ms, int32_t cap, int32_t* count, int64_t* filled);

/* ---- finer-grained operators (the module pieces callers compose) -------- */

/* Backward of the most recent smaml_forward (same theta): dpred [nsamples][N*Hf][C]
 * (device) = dLoss/dpred -> grad [P] (trainable layout, overwritten; GCN gets none: F2).
 * What loss.backward() computes through HybridSTGCN_LSTM.forward (hybrid_model.py:80-117,
 * train_hybrid_maml_v5.py:134). Consumes the saved activations (ESTATE if there are none). */
int smaml_backward(smaml_ctx* ctx, void* stream, const float* theta, const float* dpred, float* grad);

/* In-place train-mode dropout of one STGCN conv output (model.py:33,36,39,42: after conv
 * layer+1's ReLU, STGCN.forward): x [n] (device) gets the counter-based mask of the GCN site
 * `layer` (0..3), seed `seed`, and the 1/(1-p) scale. */
int smaml_dropout(smaml_ctx* ctx, void* stream, float* x, int64_t n, float p, uint32_t seed, int32_t layer);

/* GCN x4 of extract_base_features (hybrid_model.py:60-78, no_grad): x_host[s] = device
 * pointer to sample s's window [T*N][Cin0] -> feats [nsamples][T*N][Hc] (device). */
int smaml_gcn_forward(smaml_ctx* ctx, void* stream, const float* const* x_host, int32_t nsamples, float* feats);

/* nn.LSTM stack (hybrid_model.py:93-102) over layer-0 inputs feats [nsamples][T*N][Hc]
 * (device, row t*N+n) -> hT [nsamples][N][H] (top layer, t = T-1). Saves the activations
 * for smaml_lstm_backward. */
int smaml_lstm_forward(smaml_ctx* ctx, void* stream, const float* theta, const float* feats, int32_t nsamples,
                       float* hT);

/* BPTT after smaml_lstm_forward: dhT [nsamples][N][H] (device) -> the LSTM entries of
 * grad [P] (overwritten; head entries zero). */
int smaml_lstm_backward(smaml_ctx* ctx, void* stream, const float* theta, const float* dhT, float* grad);

/* Head + MSELoss with the F4 row pairing (hybrid_model.py:105-115, train_hybrid_maml_v5.py:
 * 119,133): hT [nsamples][N][H] -> pred [nsamples][N*Hf][C]. With targets (y_host[s] = device
 * pointer to y [Hf*N][C], dataset.py:40-48): loss (1 device float, mean over samples and
 * elements) and dpred = dloss/dpred [nsamples][N*Hf][C]. y_host NULL: prediction only. */
int smaml_head_loss(smaml_ctx* ctx, void* stream, const float* theta, const float* hT, const float* const* y_host,
                    int32_t nsamples, float* pred, float* loss, float* dpred);

/* clip_grad_norm_(max_norm) + SGD(lr) (train_hybrid_maml_v5.py:135-139) on ntasks flat
 * vectors theta/grad [ntasks][P] (device), theta in place; norms [ntasks] (optional). */
int smaml_clip_sgd(smaml_ctx* ctx, void* stream, float* theta, const float* grad, int32_t ntasks, float lr,
                   float max_norm, float* norms);

/* Synchronise `stream` and report device-side failures of this context's kernels: SMAML_EHIP if a
 * grid-barrier bookkeeping kernel (the fused clip + SGD step above, the second-order sweep update)
 * timed out waiting for a grid that was not co-resident (its results are then invalid; the barrier
 * state is reset). Every compute entry point also checks the flag on entry, without syncing.
 * Replaces the implicit error surfacing of torch's synchronous CPU ops at
 * train_hybrid_maml_v5.py:135-139 (`loss.item()` after the inner step). */
int smaml_sync(smaml_ctx* ctx, void* stream);

/* inner_loop_v4 (train_hybrid_maml_v5.py:110-141) for every task of smaml_set_tasks:
 * `steps` support steps of `batch` windows (windows_host [steps+1][ntasks][batch], the last
 * row is the query batch, evaluated but not trained on) -> fast_out [ntasks][P]; losses /
 * norms as in smaml_meta_step. */
int smaml_inner_loop(smaml_ctx* ctx, void* stream, const float* theta, int32_t steps, int32_t batch,
                     const int32_t* windows_host, float inner_lr, float max_norm, float* fast_out, float* losses,
                     float* norms);

/* Device memory on the context's GPU (for hosts without their own allocator). */
int smaml_alloc(smaml_ctx* ctx, int64_t bytes, void** out);
int smaml_free(smaml_ctx* ctx, void* p);

/* ---- RCCL communicator (one process per GPU) ---------------------------- *
 * librccl is loaded on first use. Rank 0 calls smaml_comm_unique_id and ships the 128 bytes
 * to the other ranks (env/file/store); every rank then calls smaml_comm_init. The meta-
 * gradient all-reduce of one meta-step is smaml_comm_allreduce(meta_grad, P) (in-place sum,
 * fp32, on the given stream). The Python path uses torch.distributed's RCCL instead.
 * smaml_comm_init is bounded: where librccl has ncclCommInitRankConfig it creates the
 * communicator non-blocking and polls it for at most smaml_set_option("comm_timeout_ms")
 * (default 120 s); a rank whose peers never arrive gets SMAML_EHIP (communicator aborted)
 * instead of blocking forever, so the ranks can agree on the outcome afterwards. */
int smaml_comm_unique_id(uint8_t* id_out /* 128 bytes */);
int smaml_comm_init(smaml_ctx* ctx, int32_t rank, int32_t world, const uint8_t* id /* 128 bytes */);
int smaml_comm_allreduce(smaml_ctx* ctx, void* stream, float* buf, int64_t n);
int smaml_comm_destroy(smaml_ctx* ctx);

/* ---- measurement (no reference counterpart; bench / profiling only) ------------------ */

/* Enable/disable per-kernel-category HIP-event timing of the launches this context
 * enqueues (events recorded on the launch stream around each kernel). */
int smaml_timing(smaml_ctx* ctx, int32_t enable);

/* Synchronise, then report and reset per category: summed kernel milliseconds, summed
 * algorithmic FLOPs, launch counts. One kernel symbol per category (index): 0 gcn_layer,
 * 1 lstm_fwd_step, 2 lstm_fwd_dual, 3 head_loss, 4 head_dh, 5 lstm_bwd_step, 6 lstm_bwd_dual,
 * 7 wgrad (split-K GEMM), 8 wgrad_reduce, 9 misc, 10 xg_proj (layer 0's input projection formed before
 * the wavefront: k_xg_dedup once per distinct stream row of consecutive windows, or the batch-1
 * k_gemm_nt), 11 dg_rowsum (k_dg_rowsum: layer 0's dG summed per distinct stream row before its
 * input-weight gradient), 12-15 lstm_fwd_step_wall, lstm_fwd_dual_wall, lstm_bwd_step_wall,
 * lstm_bwd_dual_wall: the wall time of a forward / tangent-forward / BPTT / tangent-BPTT sweep whose
 * diagonals ran as concurrent row chunks on side streams (options fwd_streams / bptt_streams; the
 * per-category kernel times 1, 2, 5, 6 then sum the concurrent chunks' launches). */
int smaml_timing_collect(smaml_ctx* ctx, double* ms, double* flops, int64_t* count, int32_t cap);

/* Launch counts per kernel variant (tile configuration) since the last reset, in the order of
 * kernels.h enum Variant (_capi.VARIANTS): fwd, fwd_drop, fwd_split, fwd_img, fwd_dual,
 * fwd_dual_kept, fwd_dual_img, bwd_big, bwd_small, bwd_split, bwd_dual_big, bwd_dual_big_kept,
 * bwd_dual_small, bwd_dual_small_kept, wgrad, wgrad_wide, wgrad_pair, fwd_kw, bwd_kw, gcn_dedup,
 * xg_dedup, wgrad_dedup, f_compact.
 * Writes min(cap, count) entries, *count = number of variants; reset != 0 zeroes them. Host-side
 * counters: no synchronisation. Lets tests assert which configurations ran. */
int smaml_variant_counts(smaml_ctx* ctx, int64_t* counts, int32_t cap, int32_t* count, int32_t reset);

/* Run-time knobs (tests / A-B; defaults = build-time values):
 *   "bwd_big_min", "bwdd_big_min": primal / tangent BPTT launches with at least this many
 *                                  64-row tile units use the 128x128 tiles (else 64x64 or
 *                                  split-K tiles);
 *   "split_max":                   split-K ways of small-grid LSTM steps (1 = off);
 *   "keep":                        cap on second-order inner steps whose primal is kept
 *                                  (-1 = the SMAML_KEEP environment variable / all that fit);
 *   "wgrad_group_max_rows":        a backward with tasks x rows <= this runs all LSTM weight
 *                                  gradients as one launch after the BPTT (batch-1 adaptation);
 *   "wgrad_group_wgs":             workgroups that grouped launch aims for;
 *   "gcn_fused", "gate_img":       fused GCN stack for the rows t >= 1 / pre-split gate weight
 *                                  images (1 = on, the default);
 *   "wgrad_wide":                  weight gradients whose column count is a multiple of 256 on
 *                                  256 x 256 tiles (1, the default) or 512 x 128 tiles (0);
 *   "wgrad_pair":                  the two passes of a tangent weight gradient (LSTM layers >= 1)
 *                                  as one split-K launch (1, the default) or two (0);
 *   "grid_barrier":                the clip + SGD step and the sweep update as one grid-barrier
 *                                  launch each (1, the default) or two launches each (0; bitwise
 *                                  equal);
 *   "barrier_timeout_us":          bound on a grid-barrier wait (default 4 s); on expiry the kernel
 *                                  exits and the next call / smaml_sync returns SMAML_EHIP;
 *   "comm_timeout_ms":             bound on smaml_comm_init's wait for the other ranks (default
 *                                  120000);
 *   "barrier_oversize":            debug: > 0 launches the grid-barrier kernels with that many
 *                                  times the resident capacity (+1 block), which can never be
 *                                  co-resident, to exercise the bounded wait;
 *   "bwdd_remap":                  tangent BPTT tiles dealt in pair-segment order per XCD (1) or in
 *                                  hardware order (0; bitwise equal);
 *   "small_kw":                    small-grid (batch-1) LSTM forward / BPTT diagonals as one launch
 *                                  with the K reduction split over the waves of a workgroup (1; 2 =
 *                                  also with pre-split BPTT weight images), or as the split-K part +
 *                                  cell launch pair (0);
 *   "adapt_gcn_batch":             smaml_adapt_steps fills its per-window GCN feature cache up front,
 *                                  runs of up to this many consecutive missing windows per GCN pass
 *                                  (default 32; 0 or 1 = one window per step as it is first read;
 *                                  bitwise equal);
 *   "adapt_phase_sync":            smaml_adapt_steps synchronises its stream after the feature-cache fill
 *                                  and after the step loop so smaml_adapt_phases reports GPU time (0,
 *                                  the default; measurement only);
 *   "gcn_dedup":                   smaml_meta_step steps whose every task reads B consecutive windows
 *                                  run the fused GCN rows t >= 1 once per distinct stream row and
 *                                  store each to every (sample, step) holding it (1, the default;
 *                                  bitwise equal to 0, which computes every sample's rows);
 *   "xg_dedup":                    the same steps form layer 0's input projection F . W_ih0^T (and, in the
 *                                  second-order sweep, F . U_ih0^T) once per distinct stream row
 *                                  (k_xg_dedup) and the big-tile gate kernels start layer 0's
 *                                  accumulators from it (1, the default; the forward adds it in the
 *                                  epilogue: equal to 0 up to f32 rounding, the tangent bitwise);
 *   "wgrad_dedup":                 the same steps form layer 0's input-weight gradient (and its tangent)
 *                                  over the distinct stream rows: dG0 summed per stream row
 *                                  (k_dg_rowsum) times the gathered F rows, (2B + T - 2) N rows
 *                                  instead of T B N (1, the default; equal to 0 up to summation order);
 *   "bptt_streams", "fwd_streams": every BPTT / forward diagonal (primal and tangent) of a large
 *                                  launch split into this many row chunks on side streams (1-4; rows are
 *                                  independent through the whole recurrence, so a chunk's next diagonal
 *                                  fills another's tail; bitwise equal to 1). Defaults: bptt_streams 2,
 *                                  fwd_streams 0 = auto (2 when a problem's gate launch fills at most
 *                                  two workgroups per CU, else 1);
 *   "f_compact":                   where every reader of a step's GCN features goes through the distinct
 *                                  stream rows (xg_dedup forwards on the big tiles, wgrad_dedup
 *                                  backwards), the GCN stores each distinct row once instead of to every
 *                                  (sample, step) holding it (1, the default; bitwise equal to 0).
 *   (Round 6 removed the options of arms that measured slower -- bptt_push, wgrad_ws, rowsum_side,
 *   gcn_side, reduce_side, wgrad_overlap, wgrad_min_kt, wgrad_threads, and its own h_img; DESIGN.md
 *   keeps their A/B record.) */
int smaml_set_option(smaml_ctx* ctx, const char* key, int64_t value);

#ifdef __cplusplus
}
#endif
#endif /* SMAML_H */
