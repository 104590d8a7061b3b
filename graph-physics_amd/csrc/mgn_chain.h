// Internal interface of the register-chained bf16 h=128 MLP kernels (mgn_chain16.hip).
#pragma once
#include "mgn_common.h"

struct ChainFwdArgs {
    const __bf16* e;            // [M][128] edge state, target-sorted
    const __bf16* proj;         // [N][256] node projections (x·W0bᵀ + b0 ‖ x·W0cᵀ), bf16
    const int32_t* proj_i;      // dst per edge
    const int32_t* proj_j;      // src per edge
    const __bf16* wpack;        // forward 16x16x32 fragments of the 4 layers
    int64_t woff[4];
    int32_t wks[4];
    const float* bias[4];
    const float* scale;
    float dinv;
    int64_t M, ntiles;
    __bf16* out;                // [M][128] e + MLP(...)
    __bf16* z_save;             // [M][128] pre-norm output
    float* rden_save;           // [M]
    __bf16* act8;               // R8 saved inputs of layers 1..3
    int64_t act_off[4];
    unsigned* mask32;           // [3][ntiles*64] 32-bit lane words (ReLU bits)
    int64_t mask_stride;        // 64-bit words per layer
    // round 6, edge-side aggregation (EdgeAgg: graphs of high in-degree): the tile's segment sums of the
    // messages s ⊙ z / q over its runs of equal dst (fp32 [*][128] rows): complete segments into
    // agg_full[dst], a run continuing from the previous tile into agg_head[tile], one continuing into
    // the next tile into agg_tail[tile]
    float* agg_full;
    float* agg_head;
    float* agg_tail;
};

// Edge MLP weight gradients of layers 1..3 with their inputs RECOMPUTED (round 5): the forward writes no
// R8 activations (chain16_fwd_kernel SACT = false); one workgroup per row chunk re-runs layers 0..2 on
// its rows (the forward's exact operations: bit-identical X1..X3) and accumulates dW_l = dZ_lᵀ X_l,
// db_l = Σ dZ_l from the backward's R8 dZ saves, into its slab.
struct ChainRewArgs {
    const __bf16* e;            // [M][128] the block's edge state (target-sorted)
    const __bf16* proj;         // [N][256] its node projections (pair layout, b0 folded in P_i)
    const int32_t* proj_i;
    const int32_t* proj_j;
    const __bf16* wpack;        // forward fragments (layers 0..2 used)
    int64_t woff[4];
    int32_t wks[4];
    const float* bias[4];
    const __bf16* dz8;          // R8 [4][RP][128] dZ saves of the edge backward (layers 1..3 used)
    int64_t M, RP;
    int32_t rows_per_chunk, nchunks;
    float* part;                // slab c at part + c * G
    int64_t G;
    int64_t w_off[4], b_off[4]; // layer l's weight / bias offsets in a slab
    uint32_t* err;              // device error word (mgn_call_opts; may be NULL): MGN_ERR_HANDOFF on a timeout
    uint32_t spin;              // polls per hand-off wait before it gives up
};

struct ChainBwdArgs {
    const __bf16* dout;         // [M][128] de_out
    const __bf16* gath;         // [N][128] d_aggr, added at gath_idx[row]
    const int32_t* gath_idx;
    const __bf16* z_save;
    const float* rden_save;
    const float* scale;
    float dinv;
    const unsigned* mask32;
    int64_t mask_stride;
    const __bf16* wtpack;       // transposed 16x16x32 fragments of the 4 layers
    int64_t woff[4];
    int32_t wks[4];
    int64_t M, ntiles;
    __bf16* dz8;                // R8 [4][RP][128]
    int64_t RP;
    float* dscale_part;         // [grid][128]
    __bf16* de;                 // [M][128] de_out + dZ0·W0a
    __bf16* dz0;                // [M][128] dZ0 row-major
    // round 6, EdgeAgg in the backward: dZ0's dst-direction segment sums per tile run (node_grad's dP_i)
    float* agg_full;
    float* agg_head;
    float* agg_tail;
};

// Node MLP (16-row chained kernels): in = [x ‖ aggr], aggr[v] = Σ_{k: dst(k)=v} s_e ⊙ z_k / q_k
struct ChainNodeFwdArgs {
    const __bf16* x;            // [N][128]
    const int32_t* seg_ptr;     // CSC segment offsets (col_ptr)
    const __bf16* agg_z;        // edge MLP z [E][128]
    const float* agg_rden;      // edge MLP rden [E]
    const float* agg_scale;     // edge MLP RMSNorm scale [128]
    const __bf16* wpack;        // node MLP forward 16x16x32 fragments (layer 0: K = 256)
    int64_t woff[4];
    int32_t wks[4];
    const float* bias[4];
    const float* scale;
    float dinv;
    int64_t M, ntiles;
    __bf16* out;                // x_out = x + MLP
    __bf16* aggr_save;          // [N][128]
    __bf16* z_save;
    float* rden_save;
    __bf16* act8;
    int64_t act_off[4];
    unsigned* mask32;
    int64_t mask_stride;        // 64-bit words per layer
    // optional: the next block's node projections from x_out (nullptr pn_out: none)
    const __bf16* pn_pack;      // next edge MLP's forward pack (layer 0 first: [128][3·128], 12 k-steps)
    const float* pn_b0;         // its layer-0 bias (folded into P_i)
    __bf16* pn_out;             // [N][256] bf16: P_i ‖ P_j
    int32_t pn_kst;             // k-steps per row tile of its layer-0 pack
    // edge-side aggregation (round 6; the edge forward's ChainFwdArgs agg_*): aggr[v] = agg_full[v] when
    // v's in-edges lie in one 16-edge tile, else agg_tail[tb] + agg_head[tb + 1] + ... + agg_head[te]
    const float* agg_full;
    const float* agg_head;
    const float* agg_tail;
};

struct ChainNodeBwdArgs {
    const __bf16* dout;         // dx_out [N][128]
    const __bf16* z_save;
    const float* rden_save;
    const float* scale;
    float dinv;
    const unsigned* mask32;
    int64_t mask_stride;
    const __bf16* wtpack;       // node MLP transposed 16x16x32 fragments
    int64_t woff[4];
    int32_t wks[4];
    int64_t M, ntiles;
    __bf16* dz8;
    int64_t RP;
    float* dscale_part;
    __bf16* dx_part;            // dx_out + dA0[:, :128]
    __bf16* d_aggr;             // dA0[:, 128:]
};

bool chain_eligible(const mgn_mlp* m);
int chain16_edge_backward_parts(int64_t M);
int chain16_node_backward_parts(int64_t M);
bool chain_node_eligible(const mgn_mlp* m);  // bf16, 256 -> 128 -> 128, 4 layers, RMSNorm
// next_edge / next_proj (optional): also write the next block's node projections (bf16 [N][2·128],
// b0 folded into P_i) from x_out — the chained edge forward's proj input, without its own launch
// agg_scratch (optional, chain16_edge_agg_bytes): the edge forward already summed the messages per tile
// run (EdgeAgg) — the node forward adds those partial rows instead of gathering every in-edge's z
int chain16_node_forward(const mgn_mlp* m, const void* x, const mgn_topology* t, const mgn_mlp* edge,
                         const mgn_mlp_saved* edge_sv, int64_t M, void* x_out, void* aggr_save, mgn_mlp_saved* sv,
                         hipStream_t st, const mgn_mlp* next_edge = nullptr, void* next_proj = nullptr,
                         void* agg_scratch = nullptr);
// EdgeAgg scratch: [N][128] + 2 x [rows_pad(E)/16][128] fp32 (full / head / tail partial rows)
size_t chain16_edge_agg_bytes(int64_t N, int64_t E);
// din2: dout (dx_out) in the pair layout (mgn_block_backward_deferred2, MGN_BWD_DX_OUT_PAIR)
int chain16_node_backward(const mgn_mlp* m, int64_t M, const mgn_mlp_saved* sv, const void* dout, void* dz8,
                          float* dscale_part, int* nparts, void* dx_part, void* d_aggr, hipStream_t st,
                          bool din2 = false);
// edge MLP forward / backward: 16x16x32 tiles, 12 waves per workgroup (three per SIMD);
// nparts: number of dscale partial rows written (the reduction's row count)
// Pair layout (mgn_chain16.hip col_of): the bf16 node projections P are always in it; z_p2 / p2 =
// the block's node MLP is chained too (then the edge z and d_aggr rows are in it as well)
// save_act = false (the recomputed weight gradients, chain16_edge_wgrad_recompute): ReLU masks, z and rden
// only — no R8 layer inputs
int chain16_edge_forward(const mgn_mlp* m, const void* e, const void* proj, const int32_t* pi, const int32_t* pj,
                         int64_t M, void* out, mgn_mlp_saved* sv, hipStream_t st, bool z_p2, bool save_act = true,
                         int64_t N = 0, void* agg_scratch = nullptr);
// dW / db of the edge MLP's layers 1..3 into slabs part[0 .. nchunks) (chunks of rows_per_chunk rows, a
// multiple of 32), their inputs recomputed from e and the projections (ChainRewArgs)
int chain16_edge_wgrad_recompute(const mgn_mlp* m, const void* e, const void* proj, const int32_t* pi, const int32_t* pj,
                                 int64_t M, const void* dz8, float* part, int64_t G, int rows_per_chunk, int nchunks,
                                 hipStream_t st);
// din2 / dout2 (p2 only): de_out read / de written in the pair layout (between the edge backwards of
// consecutive processor blocks, mgn_block_backward_deferred2)
// agg_scratch (optional, chain16_edge_agg_bytes(N, M)): also dZ0's dst-direction sums per tile run
int chain16_edge_backward(const mgn_mlp* m, int64_t M, const mgn_mlp_saved* sv, const void* dout, const void* gath,
                          const int32_t* gath_idx, void* dz8, float* dscale_part, int* nparts, void* de, void* dz0,
                          hipStream_t st, bool p2, bool din2 = false, bool dout2 = false, int64_t N = 0,
                          void* agg_scratch = nullptr);
// the EdgeAgg scratch's parts (full [N][128], head / tail [rows_pad(E)/16][128] fp32)
void chain16_edge_agg_parts(void* scratch, int64_t N, int64_t E, float** full, float** head, float** tail);
// dense MLP in_dim <= 32 -> 128 -> 128 -> 128 -> 128 + RMSNorm, bf16 (the encoders): 16-row chained
// kernels with the generic DENSE save layout (ReLU masks: chained lane words)
bool chain_dense_eligible(const mgn_mlp* m);
int chain16_dense_forward(const mgn_mlp* m, const void* in, int in_dtype, int64_t in_ld, const int32_t* in_rows,
                          int64_t M, void* out, int out_dtype, mgn_mlp_saved* sv, hipStream_t st);
int chain16_dense_backward(const mgn_mlp* m, int64_t M, const mgn_mlp_saved* sv, const void* dout, int dout_dtype,
                           void* din, int din_dtype, int64_t din_ld, void* dz8, float* dscale_part, int* nparts,
                           hipStream_t st);
