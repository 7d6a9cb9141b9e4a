/*
 * xpgnn.h — C-ABI of the MI355X-native XP-GNN perturbation-scoring engine (libxpgnn.so).
 *
 * Every entry point is `extern "C"`, takes plain device pointers + sizes + a HIP stream
 * (`xpg_stream_t`, NULL = legacy default stream) and returns an int status (XPG_OK = 0);
 * `xpg_last_error()` returns a thread-local message for the last failure.  No entry point
 * allocates device memory, frees or synchronises (the xpg_profile_* measurement hooks aside):
 * device memory (inputs, outputs, workspaces) is owned by the caller (PyTorch tensors in the
 * Python host), so every call can be captured in a hipGraph.  The one handle an entry point
 * creates: xpg_masked_forward's wide path (more than one 32-row pass, stream not capturing)
 * creates, once per device, a side stream and five events for its pass overlap.
 *
 * Mask bit layout ("row bits"): uint32 [rows][words], words = ceil(cols / 32); element c of
 * row r is bit (c & 31) of word r*words + (c >> 5).  Bits past `cols` in the last word are 0.
 *
 * Reference interfaces replaced (paths relative to /root/reference/src/pathway_explanations):
 *   xpg_pack_masks / xpg_unpack_masks  — bool mask batches handed between masks.py and
 *                                        wlm.py (DataLoader batches, masks.py:197-229)
 *   xpg_sample_shapley                 — Mask.shapley_mask           masks.py:231-260
 *   xpg_sample_shapley_dev             — same, device-resident seed (graph replays)
 *   xpg_sample_shapley_sets            — same, one draw per repeat in one call
 *   xpg_plan_arrays_build / _take      — ForwardPlan receptive-field arrays (host)
 *   xpg_sample_communities             — Mask.get_internal_mask / get_external_indices +
 *                                        Pathways.mask_generator (masks.py:81-194,
 *                                        pathways.py:234-385)
 *   xpg_edge_keep                      — Data.build_edge_mask        data.py:390-451
 *   xpg_rows_no_edge                   — the empty-copy test of the multi-node-type loop
 *                                        (a copy keeping no edge outputs 0)  model.py:213-215
 *   xpg_popcount_rows + xpg_shap_kernel— Kernel.compute             kernels.py:115-174
 *   xpg_masked_forward                 — Data.perturbator + Model.infer + extract_node_edge_output
 *                                        (wlm.py:349-436 -> data.py:591-648, model.py:62-116,
 *                                        model.py:295-328) for GCNConv / SAGEConv / HeteroConv-sum
 *                                        conv stacks with a dense head; with edge_masks set, the
 *                                        edge problem's Data.perturb_edge (data.py:500-554: mask
 *                                        columns are edges) and a dot-product link decoder
 *   xpg_dense                          — the dense feature x weight contraction inside each layer
 *                                        (PyG Linear / GCNConv.lin / SAGEConv.lin_l|lin_r)
 *   xpg_wlm_fit                        — train_model's epoch loop     wlm.py:132-278 with
 *                                        LinearRegression, regularizer, weighted_mse_loss and
 *                                        torch.optim.Adam(weight_decay=1e-2) (wlm.py:17-129,441-520)
 */
#ifndef XPGNN_H
#define XPGNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define XPG_ABI_VERSION 21
#define XPG_MAX_TERMS 8

typedef void* xpg_stream_t; /* hipStream_t */

enum xpg_status { XPG_OK = 0, XPG_EINVAL = 1, XPG_EHIP = 2, XPG_ENOSPC = 3 };

enum xpg_act { XPG_ACT_NONE = 0, XPG_ACT_RELU = 1, XPG_ACT_SIGMOID = 2, XPG_ACT_TANH = 3,
               XPG_ACT_LEAKY_RELU = 4, XPG_ACT_ELU = 5 };

/* aggregation term kinds of one conv layer (one term per relation, plus ROOT for SAGE) */
enum xpg_term { XPG_TERM_GCN = 0,   /* D^-1/2 (A_r + I) D^-1/2 over relation r               */
                XPG_TERM_MEAN = 1,  /* mean over kept in-edges of relation r (SAGE aggr)      */
                XPG_TERM_ROOT = 2   /* the target's own row (SAGE lin_r)                     */ };

int xpg_abi_version(void);
const char* xpg_last_error(void);

/* ---------------------------------------------------------------- masks */
int xpg_pack_masks(const uint8_t* mask, int64_t rows, int64_t cols, uint32_t* bits,
                   xpg_stream_t stream);
int xpg_unpack_masks(const uint32_t* bits, int64_t rows, int64_t cols, uint8_t* mask,
                     xpg_stream_t stream);
/* Shapley masks, P(bit) = 1/2, counter-based Philox4x32-10 keyed by (seed, global row). */
int xpg_sample_shapley(uint64_t seed, int64_t row_offset, int64_t rows, int64_t cols,
                       uint32_t* bits, xpg_stream_t stream);
/* Same rows with the seed read from device memory (*seed, uint64) when the kernel runs: a captured
 * HIP graph of the hot path draws new masks on every replay once the caller advances *seed on
 * the stream (v11). */
int xpg_sample_shapley_dev(const uint64_t* seed, int64_t row_offset, int64_t rows, int64_t cols,
                           uint32_t* bits, xpg_stream_t stream);
/* n_sets independent Shapley draws in one call: set k = xpg_sample_shapley(seeds[k], 0, rows, cols)
 * written at bits + k * rows * ceil(cols/32) (bits = [n_sets][rows][words]); seeds is a HOST array.
 * Explainer.run(times = n_sets) draws every repeat's masks this way (one host call, v18). */
int xpg_sample_shapley_sets(const uint64_t* seeds, int32_t n_sets, int64_t rows, int64_t cols,
                            uint32_t* bits, xpg_stream_t stream);
/* HOST function (no GPU work): the reference's compat Shapley draw torch.randint(0, 2, (rows, cols),
 * dtype=torch.bool) on torch's CPU generator (masks.py:231-260), replayed from the generator's
 * at::mt19937 state (state[624] words, left, next as torch.get_rng_state() stores them) and
 * written as bit-packed rows bits[rows][ceil(cols/32)] (host memory); the state is advanced past
 * the rows * cols outputs exactly as torch would (the caller writes it back with
 * torch.set_rng_state).  Bit-identical to the torch draw (v15). */
int xpg_mt19937_mask_bits(uint32_t* state, int32_t* left, int32_t* next, int64_t rows, int64_t cols,
                          uint32_t* bits);
/* HOST function (no GPU work): the per-repeat draws Explainer.run makes on torch's CPU generator
 * with the device Shapley sampler, in the reference's order (explainer.py:490-519): per repeat
 * the sampler seed torch.randint(0, 2**62, (1,)) -> seeds[t], the surrogate's initial weights
 * LinearRegression(S) = uniform_(from, to) on S floats (wlm.py:40-45) -> w0[t][S], and the
 * DataLoader iterator's base seed draw (value discarded).  State as in xpg_mt19937_mask_bits;
 * `fma` selects the fused x * (to - from) + from form of ATen's uniform_real (v20). */
int xpg_mt19937_repeat_draws(uint32_t* state, int32_t* left, int32_t* next, int32_t times, int64_t S,
                             float from, float to, int32_t fma, int64_t* seeds, float* w0);
/* HOST function (no GPU work): the reference's compat COMMUNITY draws (Mask.mask_generator with
 * communities, masks.py:299-348: per community in length-descending order get_internal_mask's
 * randint masks.py:130, Pathways.mask_generator's antithetic randint rows pathways.py:260-281,
 * activate_dead_mask's randperm pathways.py:318, pathway_mask2node_mask pathways.py:336-385 and
 * the member assignment masks.py:338) replayed from the at::mt19937 state as above, written
 * UNSHUFFLED as bit-packed rows bits[rows][ceil(cols/32)] (host memory); the caller applies the
 * row shuffle (torch.randperm, masks.py:385, on the returned state) or the S > 4000 truncation.
 * comm_ptr / comm_cols: CSR [n_comm + 1] / [nnz] of every community's member columns, ascending
 * (the reference sorts each community in place, masks.py:323); blocks: int32 [n_blocks][5] =
 * {row_start, size, size_internal, own community, b} back to back (Mask.community_plan), rows =
 * their total.  Bit-identical to the torch path, state advanced exactly as torch would (v16). */
int xpg_mt19937_community_bits(uint32_t* state, int32_t* left, int32_t* next, int64_t cols,
                               int32_t n_comm, const int32_t* comm_ptr, const int32_t* comm_cols,
                               const int32_t* blocks, int32_t n_blocks, int64_t rows, uint32_t* bits);
/* HOST functions (no GPU work): the receptive-field plan arrays of a forward plan
 * (engine.plan_arrays; the frontier walk of Model's L message-passing layers over the
 * computational subgraph, explainer.py:345-480 / model.py:62-116).  Edges relation by relation
 * (rel_ptr [n_rel + 1] offsets into src / dst [E]), optional per-edge mask columns eid [E]
 * (edge-mask plans; NULL = 0), the query positions [nq] (distinct, < S), L layers.  build
 * computes and keeps the arrays behind *handle and writes their sizes: the L + 1 frontier sizes,
 * then per CSR (the F_0 degree CSR, then layers 1..L) the sizes of {ptr, src, eid, smul, sptr,
 * seid}; take copies them back to back into out (int64, the sum of the sizes) and releases the
 * handle (free releases it without copying).  Frontier L = the queries, frontier l - 1 = frontier
 * l + its sorted new in-neighbours; CSRs group each target's in-edges (self-loops apart, counted
 * in smul with their columns in sptr / seid) in edge order, offsets absolute across relations;
 * the degree CSR holds source node ids, the layer CSRs source positions in F_0 (v19). */
int xpg_plan_arrays_build(int64_t S, int32_t n_rel, const int64_t* rel_ptr, const int64_t* src,
                          const int64_t* dst, const int64_t* eid, const int64_t* queries, int64_t nq,
                          int32_t L, void** handle, int64_t* sizes);
int xpg_plan_arrays_take(void* handle, int64_t* out);
int xpg_plan_arrays_free(void* handle);
/* Same bits, plus counts[r] = popcount of row r (the KernelSHAP coalition sizes, kernels.py:144),
 * accumulated while sampling so KernelSHAP needs no second pass over the bits. */
int xpg_sample_shapley_counts(uint64_t seed, int64_t row_offset, int64_t rows, int64_t cols,
                              uint32_t* bits, int32_t* counts, xpg_stream_t stream);
/* Community-aware masks — replaces Mask.get_internal_mask / get_external_indices and
 * Pathways.mask_generator / activate_dead_mask / pathway_mask2node_mask (masks.py:81-194,
 * pathways.py:234-385) plus the row shuffle (masks.py:375-380), generated in HBM.
 * blocks (device, int32 [n_blocks][5]) = {row_start, size, size_internal, own, off} per
 * community in length-descending order (the host plan, masks.py:309-340); col_ptr / col_comm
 * (device, int32 [cols+1] / [nnz]) = the communities each column belongs to.  Output row r is
 * source row perm(r) (shuffle != 0; a seeded bijection of [0, src_rows)) or r (shuffle == 0,
 * the S > 4000 truncation branch); prow (nullable) gets the row's community (pathway_rows). */
int xpg_sample_communities(uint64_t seed, int64_t rows, int64_t cols, int32_t n_comm,
                           const int32_t* blocks, int32_t n_blocks, int64_t src_rows,
                           int32_t shuffle, const int32_t* col_ptr, const int32_t* col_comm,
                           uint32_t* bits, int32_t* prow, xpg_stream_t stream);
/* the same rows' global range [row_offset, row_offset + rows) only, written to bits / prow from row 0
 * (row r of the full call == row r - row_offset here): a rank generates its own shard (ABI v14) */
int xpg_sample_communities_rows(uint64_t seed, int64_t row_offset, int64_t rows, int64_t cols,
                                int32_t n_comm, const int32_t* blocks, int32_t n_blocks,
                                int64_t src_rows, int32_t shuffle, const int32_t* col_ptr,
                                const int32_t* col_comm, uint32_t* bits, int32_t* prow,
                                xpg_stream_t stream);

/* ---------------------------------------------------------------- perturbation */
/* keep[b*n_edges + e] = bit(b, src[e]) & bit(b, dst[e])   (data.py:420-449) */
int xpg_edge_keep(const uint32_t* bits, int64_t rows, int64_t cols, const int32_t* src,
                  const int32_t* dst, int64_t n_edges, uint8_t* keep, xpg_stream_t stream);

/* empty[r] = 1 iff mask row r keeps no edge (src[e] and dst[e] both set), else 0: the multi-node-type
 * loop's copies without edges (model.py:213-215), one byte per row; stops at a row's first kept
 * edge.  (ABI v14) */
int xpg_rows_no_edge(const uint32_t* bits, int64_t rows, int64_t cols, const int32_t* src,
                     const int32_t* dst, int64_t n_edges, uint8_t* empty, xpg_stream_t stream);

/* ---------------------------------------------------------------- KernelSHAP */
int xpg_popcount_rows(const uint32_t* bits, int64_t rows, int64_t cols, int32_t* counts,
                      xpg_stream_t stream);
/* kernel_out[r] from counts[r] with M = cols-1: exact formula for M <= 1000, the reference's
 * ref-1000 approximation with its 0.9 back-off otherwise, then +-inf/NaN -> 0. */
int xpg_shap_kernel(const int32_t* counts, int64_t rows, int64_t cols, double* kernel_out,
                    xpg_stream_t stream);

/* ---------------------------------------------------------------- dense (MFMA fp32) */
/* C[m, n] = act(sum_k A[m, k] * W[n, k] + bias[n]) for n < n_real, 0 for n_real <= n < n_pad.
 * k_pad % 8 == 0 (A and W zero-padded in k), n_pad % 32 == 0 (<= 256), W has n_pad rows,
 * lda/ldw/ldc multiples of 4, pointers 16-byte aligned. */
int xpg_dense(const float* A, int64_t M, int64_t lda, const float* W, int64_t ldw,
              int64_t k_pad, const float* bias, int64_t n_real, int64_t n_pad, int act,
              float* C, int64_t ldc, xpg_stream_t stream);

/* ---------------------------------------------------------------- masked forward */
/* Frontier formulation: F_L ⊆ ... ⊆ F_1 ⊆ F_0 are the subgraph nodes whose layer outputs are
 * needed (the query's receptive field; or every node for a full-graph pass).  All CSR arrays
 * are device pointers; per-relation CSRs are concatenated (ptr arrays hold absolute offsets,
 * relation r's segment of a ptr array starts at r * (n + 1)). */
typedef struct xpg_term_desc {
  int32_t kind;            /* enum xpg_term                                             */
  int32_t rel;             /* relation index (degree slot); ignored for ROOT           */
  const float* table;      /* layer 1 only: pre-transformed F_0 rows [n0][f_out_pad]   */
  int32_t dst_type;        /* multi-node-type plans: the term only reaches targets of   */
                           /* this node type (HeteroConv relation destination); -1 = all */
} xpg_term_desc;

typedef struct xpg_layer_desc {
  int32_t n_terms;
  int32_t act;             /* activation after the conv (enum xpg_act)                 */
  int32_t f_in_pad;        /* width of this layer's input rows (layer >= 2), % 8 == 0   */
  int32_t f_out;           /* real output width                                        */
  int32_t f_out_pad;       /* padded output width, % 32 == 0, <= 256                   */
  int32_t n_tgt;           /* |F_l|                                                    */
  int32_t n_edges;         /* agg_src / agg_f0 length (all relations)                  */
  const int32_t* tgt_prev; /* [n_tgt] position of each target inside F_{l-1}          */
  const int32_t* tgt_f0;   /* [n_tgt] position of each target inside F_0; frontiers are */
                           /* prefix-ordered (F_l = the first |F_l| nodes of F_{l-1}),  */
                           /* so every target of every layer sits in F_0[0, |F_1|)      */
  const int32_t* agg_ptr;  /* [n_rel * (n_tgt + 1)] in-edges per target, self-loops out */
  const int32_t* agg_src;  /* source positions inside F_{l-1}                          */
  const int32_t* agg_f0;   /* source positions inside F_0                              */
  const int32_t* self_mult;/* [n_rel * n_tgt] multiplicity of (t, t) edges             */
  xpg_term_desc terms[XPG_MAX_TERMS];
  const float* weight;     /* layer >= 2: [f_out_pad][n_terms * f_in_pad]               */
  const float* bias;       /* [n_types][f_out_pad], summed over relations, zero-padded */
  const int32_t* tgt_type; /* multi-node-type plans: [n_tgt] node type of each target;   */
                           /* NULL for homogeneous / single-node-type graphs             */
  int32_t n_types;         /* rows of bias (1 when tgt_type is NULL)                   */
  /* edge-mask plans only (plan.edge_masks = 1; NULL otherwise):                          */
  const int32_t* agg_eid;  /* [n_edges] mask column (subgraph edge id) of each in-edge   */
  const int32_t* self_ptr; /* [n_rel * (n_tgt + 1)] self-loop edges of each target       */
  const int32_t* self_eid; /* their mask columns (MEAN terms count the kept ones)        */
} xpg_layer_desc;

typedef struct xpg_head_desc {
  int32_t k_pad, n_real, n_pad, act;
  const float* weight;     /* [n_pad][k_pad], zero-padded                              */
  const float* bias;       /* [n_pad], zero-padded                                     */
} xpg_head_desc;

typedef struct xpg_forward_plan {
  int64_t cols;            /* mask columns S                                           */
  int32_t n_rel;           /* relations (1 for homogeneous graphs)                     */
  int32_t n0;              /* |F_0|                                                    */
  const int32_t* f0_node;  /* [n0] subgraph node id of each F_0 position              */
  const int32_t* deg_ptr;  /* [n_rel * (n0 + 1)] in-edges of F_0 nodes, self-loops out */
  const int32_t* deg_src;  /* subgraph node ids                                        */
  int64_t n_deg_edges;     /* deg_src length (all relations)                           */
  int32_t n_layers;
  const xpg_layer_desc* layers;   /* host array [n_layers]                             */
  int32_t n_head;
  const xpg_head_desc* head;      /* host array [n_head]                               */
  int32_t out_col;         /* output column extracted (0)                              */
  /* Edge masks (Data.perturb_edge, data.py:500-554): mask columns are the subgraph's edges
   * (cols = edge count) and edge e is kept in row r iff its bit is set; every node stays
   * active.  Degrees and aggregations test the edge's own bit (deg_eid / agg_eid / self_eid);
   * GCN keeps one weight-1 self-loop per node whatever the mask (add_remaining_self_loops),
   * MEAN counts the kept self-loop edges.  Only the multi-kernel path takes these plans. */
  int32_t edge_masks;      /* 0: node masks (default), 1: edge masks                   */
  const int32_t* deg_eid;  /* [n_deg_edges] mask column of each deg_src entry          */
  /* Link decoder (edge problems): y[r] = act(<h_a, h_b>) over the n_real columns of the
   * last layer (head output, else last conv) of last-frontier targets a and b, instead of
   * one output column per target (then y has 1 column). */
  int32_t edge_dot;        /* 0: per-target outputs (default), 1: dot-product decoder   */
  int32_t dot_a, dot_b;    /* target positions in the last frontier                   */
  int32_t dot_act;         /* enum xpg_act applied to the dot product                  */
} xpg_forward_plan;

/* Workspace needed by xpg_masked_forward for `rows` mask rows. */
int xpg_forward_workspace(const xpg_forward_plan* plan, int64_t rows, size_t* bytes);
/* y[r * n_last + i] = model output (column out_col) of target i of the last conv layer for
 * mask row r (n_last = layers[n_layers-1].n_tgt; 1 for a single query); with edge_dot set,
 * y[r] = the decoded score of the target pair (dot_a, dot_b).  The workspace also holds the
 * launch's block-scheduling counters (zeroed on the stream before the kernel); its prior
 * contents never matter (no kernel reads a workspace byte it did not write).  Calls that may
 * run at the same time (different streams) need workspaces of their own.  Concurrent calls from
 * several host threads are safe under that rule: the wide path's shared side stream and pass
 * events are held by one call's whole enqueue sequence at a time. */
int xpg_masked_forward(const xpg_forward_plan* plan, const uint32_t* bits, int64_t rows,
                       float* y, void* workspace, size_t workspace_bytes, xpg_stream_t stream);

/* Optional per-kernel timing of xpg_masked_forward's wide (full-graph) path (v13): with profiling
 * on, every launch of a profiled kernel is bracketed by two hipEvents on its stream;
 * xpg_profile_read waits for them and returns, per slot, the summed device milliseconds and the
 * launch count, then releases them.  xpg_profile_enable (0 / 1) also drops unread records.  For
 * measurement only: never enable it around a graph capture.  Slots: */
enum xpg_prof_slot { XPG_PROF_WIDE_BITS = 0, XPG_PROF_WIDE_F0 = 1, XPG_PROF_WIDE_DEGREE = 2,
                     XPG_PROF_WIDE_L1 = 3, XPG_PROF_WIDE_L2 = 4, XPG_PROF_SLOTS = 5 };
int xpg_profile_enable(int on);
int xpg_profile_read(double* ms, int64_t* launches, int32_t n_slots);

/* ---------------------------------------------------------------- weighted linear surrogate */
typedef struct xpg_wlm_params {
  float lr, l1_lambda, beta1, beta2, eps, weight_decay;
} xpg_wlm_params;

/* Workspace needed by xpg_wlm_fit. */
int xpg_wlm_workspace(int64_t n_fits, int64_t rows, int64_t cols, int64_t batch, size_t* bytes);
/* Which fit kernel a shape takes (v13): *kind = XPG_WLM_SINGLE (one workgroup per fit),
 * XPG_WLM_MULTI (*parts co-resident workgroups per fit), XPG_WLM_GRID (the many-column
 * streaming fit, three launches per Adam step) or XPG_WLM_GRID_FUSED (v21: the many-column fit
 * as one persistent launch per fit, *parts co-resident workgroups, one per CU; the grid kinds
 * have no xpg_wlm_prepare / xpg_wlm_fit_prepared); *parts = 1 unless MULTI / GRID_FUSED.  The
 * choice depends on the current device's CU count and the XPG_WLM / XPG_MC_* overrides
 * (XPG_WLM=grid3: the three-launch grid fit). */
enum xpg_wlm_kind { XPG_WLM_SINGLE = 0, XPG_WLM_MULTI = 1, XPG_WLM_GRID = 2, XPG_WLM_GRID_FUSED = 3 };
int xpg_wlm_plan(int64_t n_fits, int64_t rows, int64_t cols, int64_t batch, int32_t* kind,
                 int32_t* parts);
/* Runs ceil(rows / batch) Adam steps of train_model over consecutive row batches for n_fits
 * independent surrogates (e.g. the `times` repeats of Explainer.run), one workgroup each.
 * Arrays are fit-major and contiguous: bits [n_fits][rows][words], y / kernel [n_fits][rows],
 * w / adam_m / adam_v [n_fits][cols] (updated in place), losses [n_fits][steps] (fp64),
 * best_epoch [n_fits] (first argmin).  `step0` = Adam steps already taken with (m, v).
 * status (device int32 [1], nullable, zeroed by the caller): sticky — the call ORs a nonzero
 * error word into it when the multi-workgroup fit's cross-workgroup exchange timed out (a
 * partner workgroup was not co-resident) and never clears it (v13), so one word checked after
 * many fits (e.g. K replays of a captured chain) reports a failure in any of them; every
 * output of a failed call is invalid and the caller must not use it. */
int xpg_wlm_fit(int64_t n_fits, const uint32_t* bits, int64_t rows, int64_t cols,
                int64_t batch, const float* y, const double* kernel,
                const xpg_wlm_params* params, int64_t step0, float* w, float* adam_m,
                float* adam_v, double* losses, int32_t* best_epoch, int32_t* status,
                void* workspace, size_t workspace_bytes, xpg_stream_t stream);
/* Same fit started from initial weights w0 [n_fits][cols] with zero Adam moments (step0 = 0):
 * w = w0, adam_m = adam_v = 0 are written by the fit's own prologue kernel, so a fresh fit
 * needs no copy / fill launches of its own (v11). */
int xpg_wlm_fit_from(int64_t n_fits, const uint32_t* bits, int64_t rows, int64_t cols,
                     int64_t batch, const float* y, const double* kernel,
                     const xpg_wlm_params* params, const float* w0, float* w, float* adam_m,
                     float* adam_v, double* losses, int32_t* best_epoch, int32_t* status,
                     void* workspace, size_t workspace_bytes, xpg_stream_t stream);
/* xpg_wlm_fit_from in two launches on one workspace (v12): xpg_wlm_prepare runs the fit's
 * prologue (per-step constants from y / kernel, column bit vectors, w = w0, zero moments,
 * exchange-slot reset) and xpg_wlm_fit_prepared the Adam steps + losses / best epoch / status.
 * Same results bit for bit; a caller with two workspaces can prepare the next fit while the
 * current one runs.  Shapes that take the many-column grid fit have no prologue: EINVAL. */
int xpg_wlm_prepare(int64_t n_fits, const uint32_t* bits, int64_t rows, int64_t cols,
                    int64_t batch, const float* y, const double* kernel,
                    const xpg_wlm_params* params, const float* w0, float* w, float* adam_m,
                    float* adam_v, void* workspace, size_t workspace_bytes, xpg_stream_t stream);
int xpg_wlm_fit_prepared(int64_t n_fits, const uint32_t* bits, int64_t rows, int64_t cols,
                         int64_t batch, const double* kernel, const xpg_wlm_params* params,
                         float* w, float* adam_m, float* adam_v, double* losses,
                         int32_t* best_epoch, int32_t* status, void* workspace,
                         size_t workspace_bytes, xpg_stream_t stream);

/* xpg_wlm_fit_prepared in its two launches (v17): the Adam steps (the fit kernel: w, adam_m,
 * adam_v) and then, in stream order after them, the losses / first best epoch / status word
 * (k_wlm_loss_best).  A caller that needs the next fit to start right after this one's steps can
 * put the losses on another stream (after an event on the steps' stream). */
int xpg_wlm_fit_steps(int64_t n_fits, const uint32_t* bits, int64_t rows, int64_t cols, int64_t batch,
                      const double* kernel, const xpg_wlm_params* params, float* w, float* adam_m,
                      float* adam_v, void* workspace, size_t workspace_bytes, xpg_stream_t stream);
int xpg_wlm_fit_losses(int64_t n_fits, int64_t rows, int64_t cols, int64_t batch, const double* kernel,
                       const xpg_wlm_params* params, double* losses, int32_t* best_epoch,
                       int32_t* status, void* workspace, size_t workspace_bytes, xpg_stream_t stream);

/* ---------------------------------------------------------------- k-hop computational subgraph */
/* Replaces Data.comp_graph's PyG k_hop_subgraph(seed, hops, edge_index, relabel_nodes=True,
 * flow='source_to_target') call (reference data.py:331-333).  Workspace for a graph of
 * n_nodes nodes and n_edges edges. */
int xpg_khop_workspace(int64_t n_nodes, int64_t n_edges, size_t* bytes);
/* edge_index: int64 [2][n_edges] (row 0 = source, row 1 = target).  Outputs (device):
 * subset [n_nodes capacity] sorted node ids; sub_src / sub_dst [n_edges capacity] relabelled
 * kept edges in original order; edge_mask [n_edges] (0/1 bytes); counts [4] =
 * {|subset|, kept edges, position of seed in subset, 1 if any edge id was out of range}.
 * Asynchronous: the caller reads counts after synchronising the stream. */
int xpg_khop_subgraph(const int64_t* edge_index, int64_t n_edges, int64_t n_nodes, int64_t seed,
                      int32_t hops, int64_t* subset, int64_t* sub_src, int64_t* sub_dst,
                      uint8_t* edge_mask, int64_t* counts, void* workspace,
                      size_t workspace_bytes, xpg_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* XPGNN_H */
