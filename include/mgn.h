/*
 * libmgn — MI355X-native (gfx950) MeshGraphNet message-passing library. C ABI.
 *
 * This is the drop-in boundary for the hot path of cviviers/graph-physics: everything the
 * reference executes from EncodeProcessDecode.forward downwards (reference
 * graphphysics/models/processors.py:111-137) and its autograd backward:
 *
 *   mgn_topology_build   replaces the index bookkeeping torch-geometric 2.6.1 does inside
 *                        MessagePassing.propagate for edge_index[2,E] (reference
 *                        graphphysics/models/layers.py:688-696: row,col = edge_index; x[col],
 *                        x[row]; scatter-add over edge_index[1] with dim_size = x.size(0)).
 *   mgn_mlp_pack         nn.Linear weights of build_mlp (layers.py:77-113) → MFMA fragment order.
 *   mgn_mlp_forward      build_mlp forward (Linear/ReLU chain + RMSNorm layers.py:49-74);
 *                        used for nodes_encoder / edges_encoder / decode_module
 *                        (processors.py:72-90,127-128,136).
 *   mgn_mlp_backward     its backward (data + weight gradients).
 *   mgn_block_forward    GraphNetBlock.forward (layers.py:667-746): edge MLP on
 *                        [e ‖ x[col] ‖ x[row]], sum-aggregation into targets, node MLP on
 *                        [x ‖ aggr], both residuals.
 *   mgn_block_backward   its backward (index_put_/gather/addmm backward of the reference).
 *   mgn_adamw            torch.optim.AdamW step (lightning_module.py:275-282) over a flat
 *                        parameter buffer.
 *
 * Conventions
 *  - All device memory is owned by the caller (PyTorch caching allocator); raw pointers + sizes.
 *    The library holds no device allocations and no global mutable state besides the
 *    thread-local error string (per-call options such as CU caps are arguments: mgn_call_opts;
 *    ABI v17). Every call is asynchronous on the given stream except mgn_topology_build (which reads back one validation word; mgn_topology_build_async does not).
 *  - Input validation that needs the data (edge_index range, node-type range) never reads back to
 *    the host on the asynchronous entry points: kernels OR an MGN_ERR_* bit into a caller-owned
 *    device word (uint32, zeroed by the caller), keep every access in bounds (clamped index /
 *    all-zero one-hot row), and the caller checks the word lazily and raises the reference's
 *    exception (IndexError / RuntimeError).
 *  - Return value: 0 on success, otherwise a nonzero status; mgn_last_error() describes it.
 *  - Edge order inside the library is target-sorted ("CSC" order: stable sort of the caller's
 *    edges by edge_index[1]); csc_eid maps it back to the caller's order.
 *  - dtype: MGN_F32 = fp32 storage + exact fp32 MFMA (parity path);
 *           MGN_BF16 = bf16 storage of activations/packed weights, fp32 accumulation and fp32
 *           epilogues (RMSNorm, residual), fp32 master weights and gradients.
 *  - Deterministic: no floating-point atomics; every reduction has a fixed order.
 */
#ifndef MGN_H
#define MGN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* mgn_stream_t; /* == hipStream_t */

#define MGN_ABI_VERSION 17
#define MGN_F32 0
#define MGN_BF16 1
#define MGN_MAX_LAYERS 8

/* ---------------------------------------------------------------- status */
int mgn_abi_version(void);
const char* mgn_last_error(void);

/* bits of the device error word */
#define MGN_ERR_EDGE_INDEX 1u /* edge_index outside [0, N): reference IndexError (ATen index)         */
#define MGN_ERR_TYPE_NEG 2u   /* node type < 0 or NaN: F.one_hot "Class values must be non-negative." */
#define MGN_ERR_TYPE_BIG 4u   /* node type >= n_types: "Class values must be smaller than num_classes." */
#define MGN_ERR_HANDOFF 8u    /* ABI v17: a bounded hand-off wait inside a pipelined kernel (the recomputed
                                 weight gradients, mgn_block_backward_deferred3) timed out; the kernel
                                 wrote NaN into its partial sums instead of a partial result           */
#define MGN_ERR_ANY 0xFFFFu   /* any validation error (bits 0-15)                                      */
/* State updates are predicated on the word, so an error raised lazily (one call late) leaves the
 * training state as the reference's immediate exception would (ABI v11): mgn_adamw_dev skips its
 * update while any MGN_ERR_ANY bit is set, counts the skip in bits 16-23 (MGN_ERR_SKIP_ONE each,
 * saturating at 255) and sets MGN_ERR_STALE; mgn_simulator_preamble skips the node / edge
 * normalizers' accumulation while any bit is set (the reference's F.one_hot raises after the output
 * normalizer has accumulated, simulator.py:_build_input_graph) and the output normalizer's once
 * MGN_ERR_STALE is set (the error belongs to an earlier step the reference would have stopped at). */
#define MGN_ERR_SKIP_ONE (1u << 16)
#define MGN_ERR_SKIP_MASK (0xFFu << 16)
#define MGN_ERR_STALE (1u << 31)

/* ---------------------------------------------------------------- topology */
typedef struct mgn_topology {
    int64_t num_nodes;
    int64_t num_edges;
    const int32_t* csc_src;  /* [E] source node (edge_index[0]) of the k-th target-sorted edge  */
    const int32_t* csc_dst;  /* [E] target node (edge_index[1]), non-decreasing                  */
    const int32_t* csc_eid;  /* [E] caller edge id of the k-th target-sorted edge                */
    const int32_t* col_ptr;  /* [N+1] in-edge segment of node i = [col_ptr[i], col_ptr[i+1])     */
    const int32_t* row_ptr;  /* [N+1] out-edge segment of node j within row_perm                 */
    const int32_t* row_perm; /* [E] target-sorted positions, stably sorted by source node         */
} mgn_topology;

size_t mgn_topology_workspace_bytes(int64_t num_edges, int64_t num_nodes);
/* edge_index: device int64 [2,E] row-major (reference layout). Fails with a nonzero status and
 * "edge_index out of range" if any index is outside [0, N) (the reference raises IndexError). */
int mgn_topology_build(const int64_t* edge_index, int64_t num_edges, int64_t num_nodes,
                       int32_t* csc_src, int32_t* csc_dst, int32_t* csc_eid, int32_t* col_ptr,
                       int32_t* row_ptr, int32_t* row_perm, void* ws, size_t ws_bytes,
                       mgn_stream_t stream);
/* The same without any host read-back (a new batch's topology never synchronises): an index
 * outside [0, N) sets MGN_ERR_EDGE_INDEX in *err_word and is clamped into range. Host-side
 * failures (sizes, N = 0 with E > 0) still return a nonzero status. */
int mgn_topology_build_async(const int64_t* edge_index, int64_t num_edges, int64_t num_nodes,
                             int32_t* csc_src, int32_t* csc_dst, int32_t* csc_eid, int32_t* col_ptr,
                             int32_t* row_ptr, int32_t* row_perm, void* ws, size_t ws_bytes,
                             uint32_t* err_word, mgn_stream_t stream);

/* ---------------------------------------------------------------- MLP (build_mlp) */
typedef struct mgn_mlp {
    int32_t n_layers; /* number of nn.Linear (reference nb_of_layers, >= 2)                    */
    int32_t in_dim;   /* input features of Linear 0                                          */
    int32_t hidden;   /* hidden width the kernels run (16, 32, 64, 128 or 256)                */
    int32_t out_dim;  /* output features of the last Linear (== hidden, or 1..16)            */
    int32_t has_norm; /* RMSNorm(out_dim) after the last Linear                              */
    int32_t dtype;    /* MGN_F32 | MGN_BF16                                                  */
    int32_t norm_dim; /* ABI v11: the RMSNorm's d in rms = |x|·d^(-1/2) (0: out_dim). A model of hidden
                         size h the kernels do not instantiate runs on the next supported width with
                         exactly-zero padded channels; its RMSNorm still divides by the true h      */
    int32_t reserved;
    const void* wpack;  /* forward fragments, mgn_mlp_pack_elems() elements of dtype         */
    const void* wtpack; /* transposed fragments (backward), same element count                */
    const float* bias[MGN_MAX_LAYERS]; /* fp32 master biases                                  */
    const float* scale;                /* fp32 RMSNorm scale [out_dim] or NULL                */
} mgn_mlp;

/* Forward state kept for the backward. `act` holds the INPUT of every Linear (layer 0: the
 * MLP input — not for GraphNetBlock MLPs; layer l>0: the ReLU output of layer l-1) in the row-octet
 * layout (element (m,c) at ((m/8)*cols + c)*8 + m%8, rows padded to 64) that makes every weight-
 * gradient MFMA fragment one 16-byte load; `mask` holds the hidden layers' ReLU masks (64-bit
 * wave-ballot words, or the chained kernels' per-lane words — opaque to callers: only the backward of
 * the same MLP reads it). Sizes: mgn_mlp_saved_elems(). */
typedef struct mgn_mlp_saved {
    void* act;    /* act_elems elements of dtype                                             */
    void* mask;   /* mask_words x 8 bytes                                                    */
    void* z;      /* [M, hidden] last Linear output before RMSNorm (dtype); NULL w/o norm    */
    float* rden;  /* [M] RMSNorm denominator rms+eps; NULL w/o norm                          */
} mgn_mlp_saved;
/* block_mlp != 0 for the edge/node MLPs of a GraphNetBlock: their layer-0 input is not saved (the
 * weight-gradient kernel re-gathers [e ‖ x_i ‖ x_j] / [x ‖ aggr]). */
int mgn_mlp_saved_elems(const mgn_mlp* m, int64_t rows, int32_t block_mlp, int64_t* act_elems,
                        int64_t* mask_words);

/* Pack job: one nn.Linear weight [n, k] fp32 row-major → fragment buffers (dtype). */
typedef struct mgn_pack_job {
    const float* w;
    void* dst;   /* forward fragments  */
    void* dstT;  /* transposed fragments */
    int32_t n, k, dtype;
    /* ABI v11, zero-padded packs (0: none): the source w is [n_src][k_src] row-major, packed as the
     * [n][k] matrix whose rows >= n_src are 0 and whose k axis is blocks of kb_pad columns holding
     * kb_src source columns each (rest 0): e.g. [e ‖ x_i ‖ x_j] of hidden h on width H: kb_src = h,
     * kb_pad = H */
    int32_t n_src, k_src, kb_src, kb_pad, reserved;
} mgn_pack_job;

/* ABI v15: an fp32 Linear with n == 128 and k a multiple of 128 carries one 128x128 "chain image" per
 * 128-column input block (v14: of the first block only) — the register-chained fp32 edge and node MLP
 * kernels' LDS-DMA source; the count changes, the layout stays opaque to callers. */
int64_t mgn_linear_pack_elems(int32_t n, int32_t k, int32_t dtype);
int64_t mgn_mlp_pack_elems(const mgn_mlp* m); /* Σ over layers of mgn_linear_pack_elems */
/* jobs: DEVICE array of njobs mgn_pack_job; max_elems = max over jobs of n*k. One launch. */
int mgn_pack_weights(const mgn_pack_job* jobs, int32_t njobs, int64_t max_elems,
                     mgn_stream_t stream);

/* Input description of a dense MLP: rows r of `in` (ld elements apart), optionally gathered
 * through in_rows[r]; in_dtype MGN_F32 or the MLP dtype. */
int mgn_mlp_forward(const mgn_mlp* m, const void* in, int32_t in_dtype, int64_t in_ld,
                    const int32_t* in_rows, int64_t rows, void* out, int32_t out_dtype,
                    mgn_mlp_saved* saved, mgn_stream_t stream);
size_t mgn_mlp_backward_workspace_bytes(const mgn_mlp* m, int64_t rows);
/* grads: flat fp32 [W0, b0, W1, b1, ..., W_{L-1}, b_{L-1}, scale] (nn.Module parameter order),
 * overwritten. din (optional, NULL to skip): gradient w.r.t. the (gathered) input rows. */
int mgn_mlp_backward(const mgn_mlp* m, const void* in, int32_t in_dtype, int64_t in_ld,
                     const int32_t* in_rows, int64_t rows, const mgn_mlp_saved* saved,
                     const void* dout, int32_t dout_dtype, void* din, int32_t din_dtype,
                     float* grads, void* ws, size_t ws_bytes, mgn_stream_t stream);

/* ---------------------------------------------------------------- GraphNetBlock */
typedef struct mgn_block_saved {
    mgn_mlp_saved edge; /* rows = E (target-sorted order) */
    mgn_mlp_saved node; /* rows = N */
    void* aggr;         /* [N, hidden] aggregated messages (dtype) */
    /* ABI v16: NULL, or (training forward of a chained bf16 h=128 block) the block's forward workspace
     * `ws`, which the caller then keeps intact until the block's backward: the forward writes no R8
     * inputs of the edge MLP's hidden layers (edge.act is not written) and the backward recomputes them
     * from e and the node projections in ws for those layers' weight gradients (one pass, no re-read
     * of saved activations). */
    void* proj;
} mgn_block_saved;

/* x:[N,h], e:[E,h] (target-sorted edge order), dtype of the MLPs. x_out/e_out may not alias.
 * The edge MLP's first Linear on [e ‖ x_i ‖ x_j] is evaluated as e·W0aᵀ + P_i[dst] + P_j[src]
 * with the node projections P = [x·W0bᵀ ‖ x·W0cᵀ] (fp32, N rows) computed once per block into
 * ws (scratch, free again when the call's work has run).
 * Inference (no autograd, e.g. the reference's validation/rollout _make_prediction under
 * torch.no_grad, lightning_module.py:168-202): saved->edge.act = saved->node.act = NULL selects
 * kernels that write only the edge MLP's z/rden (scratch the node MLP's aggregation reads) and no
 * backward saves; aggr and the node saves may be NULL. Available where
 * mgn_block_forward_inference_supported() is 1 (bf16, h = 128, 4 layers + RMSNorm). */
int mgn_block_forward_inference_supported(const mgn_mlp* edge, const mgn_mlp* node);
size_t mgn_block_forward_workspace_bytes(const mgn_topology* t, const mgn_mlp* edge,
                                         const mgn_mlp* node);
int mgn_block_forward(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node,
                      const void* x, const void* e, void* x_out, void* e_out,
                      mgn_block_saved* saved, void* ws, size_t ws_bytes, mgn_stream_t stream);
/* A processor stack of blocks (processors.py:129-131, `for block in self.processor_list`) chained:
 * the same forward, plus two hand-offs between consecutive blocks. proj_ready = 1: ws already holds
 * this block's node projections (written by the previous call's next_ws). next_edge / next_ws
 * (optional): the NEXT block's edge MLP and its workspace — the node-MLP kernel then also computes
 * that block's projections from this block's x_out (no projection launch of its own) and sets
 * *next_proj_ready = 1; it stays 0 where the chained bf16 h=128 kernels do not apply (the caller
 * then passes proj_ready = 0 to the next call). Results are those of mgn_block_forward. */
int mgn_block_forward_chain(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node,
                            const void* x, const void* e, void* x_out, void* e_out,
                            mgn_block_saved* saved, void* ws, size_t ws_bytes, int proj_ready,
                            const mgn_mlp* next_edge, void* next_ws, size_t next_ws_bytes,
                            int* next_proj_ready, mgn_stream_t stream);
/* ABI v17: mgn_block_forward_chain with a scratch buffer for the edge-side aggregation. For graphs of
 * high in-degree (default E >= 16 N; env MGN_EDGE_AGG = 0 / 1 forces it off / on for chained blocks, "fwd"
 * / "bwd" one direction only) the training forward's edge-MLP kernel also sums each 16-edge tile's
 * messages per run of equal target and the node-MLP kernel adds those partial rows — a few per node —
 * instead of re-reading every in-edge's output row (reference layers.py:694-696, the sum aggregation; the
 * fp32 sums re-associated, in a fixed order). The backward does the same for the target-direction sums of
 * the edge MLP's layer-0 gradient (the index backward of x[col]) inside mgn_block_backward*'s workspace
 * (mgn_block_backward_workspace_bytes includes it). mgn_block_forward_scratch_bytes: the scratch it needs, 0 where it does not apply (then the call
 * is mgn_block_forward_chain). The scratch is free again when the call's work has run (one buffer can
 * serve every block of a stack). */
size_t mgn_block_forward_scratch_bytes(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node);
int mgn_block_forward_chain2(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node,
                             const void* x, const void* e, void* x_out, void* e_out,
                             mgn_block_saved* saved, void* ws, size_t ws_bytes, int proj_ready,
                             const mgn_mlp* next_edge, void* next_ws, size_t next_ws_bytes,
                             int* next_proj_ready, void* scratch, size_t scratch_bytes,
                             mgn_stream_t stream);
size_t mgn_block_backward_workspace_bytes(const mgn_topology* t, const mgn_mlp* edge,
                                          const mgn_mlp* node);
/* dx/de: gradients w.r.t. the block inputs (overwritten). edge_grads/node_grads: flat fp32 as
 * in mgn_mlp_backward (overwritten). de_out may be NULL (a zero edge-output gradient: the last
 * processor block, whose e' EncodeProcessDecode discards) where
 * mgn_block_forward_inference_supported() is 1. */
int mgn_block_backward(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node,
                       const void* x, const void* e, const mgn_block_saved* saved,
                       const void* dx_out, const void* de_out, void* dx, void* de,
                       float* edge_grads, float* node_grads, void* ws, size_t ws_bytes,
                       mgn_stream_t stream);
/* Deferred weight-gradient reduction (a processor stack's backward, processors.py:129-131 in
 * reverse): mgn_block_backward_deferred is mgn_block_backward except that, for the chained bf16
 * h=128 MLPs, the fixed-order reduction of the weight-gradient slabs is NOT launched: the slabs and
 * RMSNorm-scale partials go to `keep` (mgn_block_backward_keep_bytes, one buffer per block, alive
 * until the reduction) and reduce2[0..1] describe the reduction; mgn_wgrad_reduce_many then runs
 * every block's in ONE launch — the same sums in the same order, one launch instead of one per
 * block. Deferred for the chained bf16 h=128 MLPs, the fp32 h=128 ones (fp32 ring) and (ABI v12) the
 * generic hidden 16/32/64 MLPs (one multi-job weight-gradient launch per block); other shapes (e.g.
 * hidden 256: generic kernels, 128 x 128 weight-gradient tiles) are reduced at once (reduce2 zeroed). */
typedef struct mgn_wgrad_reduce {
    const float* part;
    const float* dsp;
    float* grads;
    int64_t G;
    int32_t nchunks, ntiles, NS, blocks;
    int32_t w0_n, w0_k, xcol0, nchunks_x; /* W0 columns >= xcol0 sum only nchunks_x slabs */
    int64_t hoff;                         /* ABI v16: outputs g >= hoff > 0 sum only nchunks_h slabs */
    int32_t nchunks_h, pad;
} mgn_wgrad_reduce;
size_t mgn_block_backward_keep_bytes(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node);
int mgn_block_backward_deferred(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node,
                                const void* x, const void* e, const mgn_block_saved* saved,
                                const void* dx_out, const void* de_out, void* dx, void* de,
                                float* edge_grads, float* node_grads, void* ws, size_t ws_bytes,
                                void* keep, size_t keep_bytes, mgn_wgrad_reduce* reduce2,
                                mgn_stream_t stream);
/* mgn_block_backward_deferred with row layouts of the gradients handed between consecutive chained
 * processor blocks (flags; 0 = mgn_block_backward_deferred): the pair layout stores feature
 * 16t + 4g + r of a row at 32(t>>1) + 8g + 4(t&1) + r (libmgn's gather layout: one 16-byte load per
 * lane and tile pair). MGN_BWD_DE_OUT_PAIR / MGN_BWD_DX_OUT_PAIR: de_out / dx_out are in it (the
 * previous call's de / dx written with MGN_BWD_DE_PAIR / MGN_BWD_DX_PAIR). The caller keeps
 * row-major for gradients handed in from outside and for the de / dx it consumes itself (the first
 * block's, for the encoders). Chained bf16 h=128 edge + node MLPs only (else an error status,
 * mgn_last_error). keep = NULL: nothing deferred — the block's weight gradients are reduced at once
 * (mgn_block_backward with the layout flags; reduce2 zeroed). */
#define MGN_BWD_DE_OUT_PAIR 1
#define MGN_BWD_DE_PAIR 2
#define MGN_BWD_DX_OUT_PAIR 4
#define MGN_BWD_DX_PAIR 8
/* ABI v13: the same call split in two halves over the same arguments (keep != NULL): DATA_ONLY runs
 * the data gradients (dx, de, and what the weight gradients read: dZ saves in `ws`, partials in
 * `keep`); WGRAD_ONLY then runs the block's single weight-gradient launch and fills reduce2. The
 * WGRAD_ONLY call may be issued on another stream (ordered after DATA_ONLY by the caller) and run
 * beside the next block's DATA_ONLY call on ANOTHER workspace; mgn_block_backward_deferred3's
 * mgn_call_opts gives each its CUs. */
#define MGN_BWD_DATA_ONLY 16
#define MGN_BWD_WGRAD_ONLY 32
int mgn_block_backward_deferred2(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node,
                                 const void* x, const void* e, const mgn_block_saved* saved,
                                 const void* dx_out, const void* de_out, void* dx, void* de,
                                 float* edge_grads, float* node_grads, void* ws, size_t ws_bytes,
                                 void* keep, size_t keep_bytes, mgn_wgrad_reduce* reduce2,
                                 int32_t flags, mgn_stream_t stream);
int mgn_wgrad_reduce_many(const mgn_wgrad_reduce* reds, int32_t n, mgn_stream_t stream);
/* ABI v14: mgn_mlp_backward_deferred in two halves over the same arguments (flags 0 = the whole call):
 * MGN_BWD_DATA_ONLY runs the data gradients (din, and the dZ saves / partials the weight gradients read
 * in `ws` / `keep`) and leaves in reduce1 only the partial-row count; MGN_BWD_WGRAD_ONLY, given that
 * reduce1, runs the weight gradients (on another stream if the caller orders it after DATA_ONLY) and
 * fills reduce1 for mgn_wgrad_reduce_many. EncodeProcessDecode's decoder (reference processors.py:131)
 * uses it to run its weight gradients beside the first processor block's data gradients. */
int mgn_mlp_backward_deferred2(const mgn_mlp* m, const void* in, int32_t in_dtype, int64_t in_ld,
                               const int32_t* in_rows, int64_t rows, const mgn_mlp_saved* saved,
                               const void* dout, int32_t dout_dtype, void* din, int32_t din_dtype,
                               float* grads, void* ws, size_t ws_bytes, void* keep, size_t keep_bytes,
                               mgn_wgrad_reduce* reduce1, int32_t flags, mgn_stream_t stream);
/* ABI v17: per-call options of the backward entry points (NULL = none; replaces v13's process-global
 * mgn_set_grid_cus, which two models or streams in one process shared):
 *   data_cus / wgrad_cus  caps on the CUs the persistent grids of this call's launches are sized for
 *                         (0 = the whole device): data_cus for every launch except the weight-gradient
 *                         launches, wgrad_cus for those. The results do not depend on the caps except
 *                         for the weight-gradient slab partition (summation order of the fp32 reductions).
 *                         A captured hipGraph keeps the grids it recorded.
 *   err_word              device word (as mgn_topology_build_async's) the call's pipelined kernels OR
 *                         MGN_ERR_HANDOFF into when a bounded hand-off wait times out (NULL: the NaN
 *                         partials alone report it). mgn_adamw_dev skips its update while it is set. */
typedef struct mgn_call_opts {
    int32_t data_cus;
    int32_t wgrad_cus;
    uint32_t* err_word;
} mgn_call_opts;
/* mgn_block_backward_deferred2 / mgn_mlp_backward_deferred2 with per-call options (same flags; for the
 * MLP, flags 0 = the whole deferred call, mgn_mlp_backward_deferred). */
int mgn_block_backward_deferred3(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node,
                                 const void* x, const void* e, const mgn_block_saved* saved,
                                 const void* dx_out, const void* de_out, void* dx, void* de,
                                 float* edge_grads, float* node_grads, void* ws, size_t ws_bytes,
                                 void* keep, size_t keep_bytes, mgn_wgrad_reduce* reduce2,
                                 int32_t flags, const mgn_call_opts* opts, mgn_stream_t stream);
int mgn_mlp_backward_deferred3(const mgn_mlp* m, const void* in, int32_t in_dtype, int64_t in_ld,
                               const int32_t* in_rows, int64_t rows, const mgn_mlp_saved* saved,
                               const void* dout, int32_t dout_dtype, void* din, int32_t din_dtype,
                               float* grads, void* ws, size_t ws_bytes, void* keep, size_t keep_bytes,
                               mgn_wgrad_reduce* reduce1, int32_t flags, const mgn_call_opts* opts,
                               mgn_stream_t stream);
/* Diagnostics builds (MGN_STAMPS) only, else an error status: per-wave [start, end] s_memrealtime ticks
 * (100 MHz) of the last launch of a chained kernel kind (0 edge fwd, 1 edge bwd, 2 node fwd, 3 node
 * bwd), n <= 4096 waves in workgroup-major order. */
int mgn_debug_wave_times(int32_t kind, uint64_t* out, int32_t n);
/* ABI v12: mgn_mlp_backward (the encoders / decoder of processors.py:71-109, 129-137) with the
 * reduction deferred like mgn_block_backward_deferred: the RMSNorm-scale partials and weight-gradient
 * slabs go to `keep` (mgn_mlp_backward_keep_bytes, alive until the reduction) and *reduce1 describes
 * the reduction for mgn_wgrad_reduce_many — so a whole EncodeProcessDecode backward ends in ONE
 * reduction launch. */
size_t mgn_mlp_backward_keep_bytes(const mgn_mlp* m, int64_t rows);
int mgn_mlp_backward_deferred(const mgn_mlp* m, const void* in, int32_t in_dtype, int64_t in_ld,
                              const int32_t* in_rows, int64_t rows, const mgn_mlp_saved* saved,
                              const void* dout, int32_t dout_dtype, void* din, int32_t din_dtype,
                              float* grads, void* ws, size_t ws_bytes, void* keep, size_t keep_bytes,
                              mgn_wgrad_reduce* reduce1, mgn_stream_t stream);
/* The same backward as two calls over one workspace (same arguments): _data writes dx, de (and, for
 * MLPs outside the chained bf16 h=128 kernels, the node-MLP weight gradients); _wgrad then writes the
 * weight gradients from what _data left in `ws` plus the forward saves, and may run on another
 * stream (ordered after _data by the caller) concurrently with the next block's _data on ANOTHER
 * workspace — the weight-gradient launch overlaps the latency-bound kernels of the next block. */
int mgn_block_backward_data(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node,
                            const void* x, const void* e, const mgn_block_saved* saved,
                            const void* dx_out, const void* de_out, void* dx, void* de,
                            float* edge_grads, float* node_grads, void* ws, size_t ws_bytes,
                            mgn_stream_t stream);
int mgn_block_backward_wgrad(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node,
                             const void* x, const void* e, const mgn_block_saved* saved,
                             const void* dx_out, const void* de_out, void* dx, void* de,
                             float* edge_grads, float* node_grads, void* ws, size_t ws_bytes,
                             mgn_stream_t stream);

/* ---------------------------------------------------------------- primitives */
/* out[k,:] = in[idx[k],:] (gather), or out[idx[k],:] = in[k,:] when scatter != 0. */
int mgn_permute_rows(const void* in, void* out, const int32_t* idx, int64_t rows, int32_t cols,
                     int32_t in_dtype, int32_t out_dtype, int32_t scatter, mgn_stream_t stream);
/* Segment sum over target-sorted edges: out[i,:] = Σ_{k in [col_ptr[i], col_ptr[i+1])} src[k,:].
 * The stand-alone form of the aggregation fused into mgn_block_forward. */
int mgn_segment_sum(const void* src, const int32_t* seg_ptr, int64_t segments, int32_t cols,
                    int32_t dtype, void* out, mgn_stream_t stream);

/* Column sums and sums of squares of a row-major fp32 [rows, cols] matrix (row stride ld), the
 * batch statistics of Normalizer._accumulate (reference layers.py:333-352): sums[0:cols] = Σ_r x,
 * sums[cols:2cols] = Σ_r x². cols <= 32. Fixed reduction order (deterministic). */
size_t mgn_column_stats_workspace_bytes(int64_t rows, int32_t cols);
int mgn_column_stats(const float* x, int64_t rows, int32_t cols, int64_t ld, float* sums, void* ws,
                     size_t ws_bytes, mgn_stream_t stream);

/* Normalizer.forward (reference layers.py:265-392, _accumulate 333-352, _mean/_std_with_epsilon
 * 354-369) on a row-major fp32 [rows, cols] matrix x (row stride ld), cols <= 32: when
 * accumulate != 0 and *num_acc < max_acc, the batch statistics — column sums of x and x² and the
 * row count, or the caller's pending = float[2*cols + 1] {Σx, Σx², count} (e.g. already summed
 * over ranks) — are added to the module's fp32 buffers acc_sum[cols], acc_sum_sq[cols],
 * *acc_count and *num_acc (+1); then out[rows, cols] (contiguous) = (x - mean) / max(sqrt(max(var,
 * 0)), eps), mean = acc_sum / max(acc_count, 1), var = acc_sum_sq / max(acc_count, 1) - mean².
 * Same fp32 expressions as the reference's torch ops (bit-identical results). */
size_t mgn_normalizer_workspace_bytes(int64_t rows, int32_t cols);
int mgn_normalizer_forward(const float* x, int64_t rows, int32_t cols, int64_t ld, int32_t accumulate,
                           const float* pending, float* acc_sum, float* acc_sum_sq, float* acc_count, float* num_acc,
                           float max_acc, float eps, float* out, void* ws, size_t ws_bytes, mgn_stream_t stream);

/* The Simulator's train/eval preamble (reference simulator.py:206-290, Simulator._build_input_graph):
 * the three Normalizer.forward calls of mgn_normalizer_forward on
 *   target delta   y[:, 0:oe-os] - x[:, os:oe]                          -> target_out [N, oe-os]
 *   node features  [x[:, fs:fe] ‖ one_hot(long(x[:, type_index]), n_types)] -> node_out [N, fe-fs+n_types]
 *   edge_attr      [E, edge_cols] (row stride lde; edge_norm NULL: none)  -> edge_out [E, edge_cols]
 * read straight from x [N, ldx], y [N, ldy] and edge_attr (no intermediate tensors), in 3 launches.
 * Statistics, buffers and outputs are bit-identical to the torch expressions + three
 * mgn_normalizer_forward calls (same partition and order). A node type outside [0, n_types) gives an
 * all-zero one-hot row and sets MGN_ERR_TYPE_NEG / MGN_ERR_TYPE_BIG in *err_word (if non-NULL); the
 * caller raises F.one_hot's RuntimeError from it. Output columns <= 32 per normalizer. */
typedef struct mgn_normalizer_state {
    float* acc_sum;      /* [cols] */
    float* acc_sum_sq;   /* [cols] */
    float* acc_count;    /* scalar */
    float* num_acc;      /* scalar */
    const float* pending; /* NULL or float[2*cols + 1] {Σx, Σx², count} (see mgn_normalizer_forward) */
    float max_acc, eps;
} mgn_normalizer_state;
size_t mgn_simulator_preamble_workspace_bytes(int64_t num_nodes, int64_t num_edges);
int mgn_simulator_preamble(const float* x, int64_t N, int64_t ldx, int32_t feat_start, int32_t feat_end,
                           int32_t type_index, int32_t n_types, int32_t out_start, int32_t out_end,
                           const float* y, int64_t ldy, const float* edge_attr, int64_t E,
                           int32_t edge_cols, int64_t lde, int32_t accumulate,
                           const mgn_normalizer_state* out_norm, const mgn_normalizer_state* node_norm,
                           const mgn_normalizer_state* edge_norm, float* target_out, float* node_out,
                           float* edge_out, uint32_t* err_word, void* ws, size_t ws_bytes,
                           mgn_stream_t stream);

/* The batch statistics of the same three normalizers without updating them (the data-parallel
 * prologue: summed over ranks, then handed to mgn_simulator_preamble as `pending`): packed =
 * [Σ target delta, Σ target delta², N, Σ node features, Σ node features², N, (Σ edge_attr,
 * Σ edge_attr², E if edge_attr != NULL)] — each block the float[2*cols + 1] layout of `pending`, with
 * the same sums as mgn_column_stats. Workspace: mgn_simulator_preamble_workspace_bytes. Node types
 * are validated as in mgn_simulator_preamble (err_word may be NULL). */
int mgn_simulator_statistics(const float* x, int64_t N, int64_t ldx, int32_t feat_start, int32_t feat_end,
                             int32_t type_index, int32_t n_types, int32_t out_start, int32_t out_end,
                             const float* y, int64_t ldy, const float* edge_attr, int64_t E,
                             int32_t edge_cols, int64_t lde, float* packed, uint32_t* err_word, void* ws,
                             size_t ws_bytes, mgn_stream_t stream);

/* Masked L2 loss (reference utils/loss.py:10-65): *loss = Σ_r m_r Σ_c (pred - target)² / (count ·
 * cols) over row-major fp32 [rows, cols] pred/target, m_r = 1 when node_type[r·nt_ld] (a float
 * column, e.g. a strided view of x) is an integer t < 32 with bit t of type_mask set; count =
 * *count when given (data-parallel global count), else Σ m (written to *count_out if non-null).
 * Backward: grad = (*grad_loss or 1) · 2 (pred - target) · m / (count · cols). Deterministic. */
size_t mgn_masked_mse_workspace_bytes(int64_t rows);
int mgn_masked_mse(const float* pred, const float* target, int64_t rows, int32_t cols, const float* node_type,
                   int64_t nt_ld, uint32_t type_mask, const float* count, float* loss, float* count_out, void* ws,
                   size_t ws_bytes, mgn_stream_t stream);
int mgn_masked_mse_backward(const float* pred, const float* target, int64_t rows, int32_t cols,
                            const float* node_type, int64_t nt_ld, uint32_t type_mask, const float* count,
                            const float* grad_loss, float* grad, mgn_stream_t stream);

/* torch.optim.AdamW semantics (decoupled weight decay p *= 1 - lr*wd, bias-corrected moments,
 * denominator sqrt(v)/sqrt(1-beta2^t) + eps), fp32, over n contiguous elements. */
int mgn_adamw(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
              double lr, double beta1, double beta2, double eps, double weight_decay,
              int64_t step, mgn_stream_t stream);

/* As mgn_adamw with lr and step read from device memory: hyper = double[2] {lr, step}. The launch
 * can be captured in a hipGraph and replayed with a new schedule (host updates hyper). err_word
 * (nullable, ABI v11): no update while a validation error is pending on it (see MGN_ERR_STALE). */
int mgn_adamw_dev(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                  const double* hyper, double beta1, double beta2, double eps, double weight_decay,
                  uint32_t* err_word, mgn_stream_t stream);
/* ABI v12: as mgn_adamw_dev; a skipped update is counted in err_word's MGN_ERR_SKIP_* field only when
 * count_skip != 0 — an optimizer step that issues several launches (one per parameter group or
 * parameter) passes 1 on its first launch and 0 on the others, so the field counts STEPS.
 * mgn_adamw_dev == mgn_adamw_dev2(..., count_skip = 1, ...). Replaces the same optimizer step as
 * mgn_adamw (reference lightning_module.py:275-282). */
int mgn_adamw_dev2(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                   const double* hyper, double beta1, double beta2, double eps, double weight_decay,
                   uint32_t* err_word, int32_t count_skip, mgn_stream_t stream);

/* ---------------------------------------------------------------- graph construction */
/* On-device replacements for the reference's per-sample host preprocessing (SURVEY.md §8(f)
 * rows 1 and 4). Edge lists are int64 [2, E] row-major (row block, then col block). Outputs are
 * coalesced: sorted by (row, col), duplicates removed. These calls synchronise the stream once to
 * return the data-dependent count to the host. Indices outside [0, num_nodes) fail with
 * "edge_index out of range" (the reference raises from ATen). */
#define MGN_COALESCE_SYMMETRIZE 1      /* add (col, row) for every (row, col): to_undirected */
#define MGN_COALESCE_DROP_SELF_LOOPS 2 /* drop (i, i)                                          */
size_t mgn_coalesce_workspace_bytes(int64_t num_keys);
/* torch_geometric.utils.to_undirected(edge_index, num_nodes) / torch sparse coalesce() of the
 * pattern (reference dataset/preprocessing.py:135, utils/torch_graph.py:32-36). out capacity:
 * 2·num_keys int64, num_keys = num_edges (·2 with MGN_COALESCE_SYMMETRIZE); out[0:2E] holds the
 * [2, E] result, *num_out = E (host). */
int mgn_coalesce(const int64_t* edge_index, int64_t num_edges, int64_t num_nodes, int32_t flags,
                 int64_t* out, int64_t* num_out, void* ws, size_t ws_bytes, mgn_stream_t stream);
/* T.FaceToEdge(remove_faces=False) (reference dataset/preprocessing.py:410,431): cells [k, C]
 * int64 row-major, k = 3 (triangles: pairs (f0,f1), (f1,f2), (f0,f2)) or k = 4 (tetrahedra split
 * into the 4 triangles of utils/torch_graph.py:173-181), then to_undirected. Workspace and out
 * capacity from num_keys = mgn_face_to_edge_keys(k, C). */
int64_t mgn_face_to_edge_keys(int32_t verts_per_cell, int64_t num_cells);
int mgn_face_to_edge(const int64_t* cells, int32_t verts_per_cell, int64_t num_cells, int64_t num_nodes,
                     int64_t* edge_index, int64_t* num_edges, void* ws, size_t ws_bytes, mgn_stream_t stream);
/* One hop of compute_k_hop_edge_index (reference utils/torch_graph.py:38-51): the pattern of
 * A_k + A_k·A with self loops removed, coalesced. edge_index_a = A must be coalesced (sorted by
 * row); A_k any edge list. Two calls: mgn_khop_count returns the candidate count num_keys
 * (= E_k + Σ_k deg_A(col_k)), then mgn_khop_hop (workspace mgn_khop_workspace_bytes, out capacity
 * 2·num_keys) produces the result and *num_out. */
size_t mgn_khop_count_workspace_bytes(int64_t num_edges_k, int64_t num_edges_a, int64_t num_nodes);
int mgn_khop_count(const int64_t* edge_index_k, int64_t num_edges_k, const int64_t* edge_index_a,
                   int64_t num_edges_a, int64_t num_nodes, int64_t* num_keys, void* ws, size_t ws_bytes,
                   mgn_stream_t stream);
size_t mgn_khop_workspace_bytes(int64_t num_keys, int64_t num_edges_k, int64_t num_nodes);
int mgn_khop_hop(const int64_t* edge_index_k, int64_t num_edges_k, const int64_t* edge_index_a,
                 int64_t num_edges_a, int64_t num_nodes, int64_t num_keys, int64_t* out, int64_t* num_out,
                 void* ws, size_t ws_bytes, mgn_stream_t stream);
/* T.Cartesian(norm=False) ‖ T.Distance(norm=False) (reference dataset/preprocessing.py:16-23) and
 * add_world_pos_features (143-174): out[k, 0:dim] = pos[row_k] − pos[col_k], out[k, dim] = its
 * L2 norm; fp32, pos row stride pos_ld, out row stride out_ld >= dim + 1, dim <= 3. ws >= 4 B. */
int mgn_edge_features(const float* pos, int64_t pos_ld, int32_t dim, const int64_t* edge_index,
                      int64_t num_edges, int64_t num_nodes, float* out, int64_t out_ld, void* ws,
                      size_t ws_bytes, mgn_stream_t stream);
/* cKDTree(pos).query_pairs(radius) of add_world_edges (reference dataset/preprocessing.py:114-121):
 * all (i, j), i < j, with the fp64 distance <= radius, as a [2, P] int64 list in out[0:2P]
 * (out[0:P] = i, out[P:2P] = j); pair order unspecified. node_type (float
 * column, stride node_type_ld) non-null keeps only OBSTACLE(1)–NORMAL(0) pairs in either order
 * (preprocessing.py:123-133). *num_pairs = P always; nothing is written when out is NULL or
 * capacity < P (call again with capacity >= P). */
size_t mgn_radius_pairs_workspace_bytes(int64_t num_nodes);
int mgn_radius_pairs(const float* pos, int64_t pos_ld, int32_t dim, int64_t num_nodes, double radius,
                     const float* node_type, int64_t node_type_ld, int64_t* out, int64_t capacity,
                     int64_t* num_pairs, void* ws, size_t ws_bytes, mgn_stream_t stream);

/* ---------------------------------------------------------------- opt-in profiler */
/* Kernel classes: 0 edge-MLP fwd, 1 node-MLP fwd, 2 dense-MLP fwd, 3 edge-MLP bwd-data,
 * 4 node-MLP bwd-data, 5 dense-MLP bwd-data, 6 weight-grad, 7 weight-grad reduce,
 * 8 node-gradient combine (segment sums of dZ0 + dP·W0[:, h:3h] GEMM), 9 weight pack,
 * 10 AdamW, 11 node projection x·W0[:, h:3h]ᵀ. */
int mgn_profile_enable(int on);
int mgn_profile_collect(int kind, double* total_ms, int64_t* count);

#ifdef __cplusplus
}
#endif
#endif /* MGN_H */
