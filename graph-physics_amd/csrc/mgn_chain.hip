// Register-chained edge-MLP kernels for the bf16, h=128 GraphNetBlock (gfx950).
//
// The edge MLP of a GraphNetBlock (reference graphphysics/models/layers.py:77-113,689-699) is four
// 128x128 Linears once its [e ‖ x_i ‖ x_j] input Linear is split into e·W0aᵀ plus node projections
// (mgn_mlp.hip, node_proj_kernel). Here ONE wave owns 32 edges and runs the whole chain:
//
//   * v_mfma_f32_32x32x16_bf16 with D[n][m] = Σ_k W[n][k]·X[m][k]: weights are the A operand,
//     activations the B operand. A 32x32 accumulator has the edge m on the lane and 16 features
//     in registers, so after bias/ReLU/bf16 the accumulator IS the next layer's B operand (no LDS
//     round trip): registers 8s..8s+7 of out-tile t form k-step 2t+s, whose element j of lane half
//     h is feature 16(2t+s) + 8(j>>2) + 4h + (j&3). The weights are staged in LDS in exactly that
//     permuted k order, so every layer — the e input included — uses it.
//   * All four layers' weights (4 x 32 KiB) stay resident in LDS for the life of a persistent
//     workgroup (4 waves, one per SIMD); waves then run their own tiles with no workgroup barrier.
//     The next tile's inputs (and the gather indices of the one after) are prefetched into
//     registers while the current tile computes.
//   * Saved activations / dZ for the weight-gradient kernel are written in the row-octet (R8)
//     layout through a small per-wave LDS transpose; row-major outputs through the same scratch as
//     coalesced 16-byte row stores.
//   * ReLU masks: each lane keeps the 64 bits of its own accumulator elements (bit 16t + r), one
//     8-byte word per lane per tile and layer; the backward kernel has the identical lane map.
#include "mgn_chain.h"

#include <cmath>
#include <cstring>
#include <mutex>

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int H = 128;                 // features
constexpr int TR = 32;                 // rows (edges) per wave tile
constexpr int NW = 4;                  // waves per workgroup
constexpr int FRAG = 512;              // bf16 per 32x32x16 operand fragment (64 lanes x 8)
constexpr int LFR = 32;                // fragments per layer: 4 out-tiles x 8 k-steps
constexpr int SLD = H + 8;             // scratch row stride (bf16): 272 B, 16-B aligned
constexpr int SROWS = 16;              // scratch rows (half a tile per pass)
constexpr size_t LDS_W = (size_t)4 * LFR * FRAG * 2;   // 128 KiB
constexpr size_t LDS_V = (size_t)5 * H * 4;             // 4 bias vectors + RMSNorm scale (fp32)
constexpr size_t LDS_S = (size_t)NW * SROWS * SLD * 2;  // per-wave transpose scratch
constexpr size_t LDS_TOTAL = LDS_W + LDS_V + LDS_S;

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// feature index of accumulator register r of out-tile t, lane half h
__device__ __forceinline__ int dcol(int t, int r, int h) { return 32 * t + 8 * (r >> 2) + 4 * h + (r & 3); }

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Prefetch discipline: the compiler counts vector-memory waits exactly only within one loop
// iteration; a register loaded in iteration k and first read in iteration k+1 gets a full
// vmcnt(0) wait there (which also waits for the stores and prefetches issued since). So every
// prefetched register is "used" by an empty asm at the END of the iteration that issued it: the
// wait lands there, counted exactly, long after the load was issued.
template <class T>
__device__ __forceinline__ void pin(const T& v) { asm volatile("" ::"v"(v)); }

// 8 bytes = 4 bf16 at p (4 consecutive features), as floats
__device__ __forceinline__ f4 ld4bf(const __bf16* p) {
    const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
    return f4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}

// Stage the four layers' weight fragments in LDS: fragment (l, t, S), lane (r, h), element j =
// W_l[32t + r][16S + 8(j>>2) + 4h + (j&3)]  (fwd)   or   W_lᵀ likewise (bwd: out = in-feature).
// Sources are libmgn's 16x16x32 packed fragments (mgn_pack_weights), in which 4 consecutive k of
// one row (fwd pack) / 4 consecutive n of one column (transposed pack) are 8 contiguous bytes.
__device__ __forceinline__ void stage_weights(__bf16* W, const __bf16* pack, const int64_t* woff, const int* wks,
                                              bool transposed) {
    // Linear walk over the packed 16x16x32 fragments (16-byte loads, fully coalesced): a source
    // chunk is 8 consecutive reduction indices (k of the fwd pack, n of the transposed pack) of one
    // A-operand row a; its two 4-element halves land in two (k-step, lane half, element group)
    // slots of the chain image. Per layer 8 row tiles x 4 k-steps x 64 lanes = 2048 chunks.
    constexpr int PER = 4 * 2048 / (NW * 64);  // 32 chunks per thread, all in flight
    u32x4 v[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int it = threadIdx.x + u * NW * 64;
        const int l = it >> 11, c = it & 2047;
        const int tile = c >> 6, lane16 = c & 63;  // tile = rt*4 + ks (rt: 16-row tile of a)
        const int rt = tile >> 2, ks = tile & 3;
        const int ksl = transposed ? 4 : wks[l];
        v[u] = *reinterpret_cast<const u32x4*>(pack + woff[l] + ((int64_t)(rt * ksl + ks) * 64 + lane16) * 8);
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int it = threadIdx.x + u * NW * 64;
        const int l = it >> 11, c = it & 2047;
        const int tile = c >> 6, lane16 = c & 63;
        const int rt = tile >> 2, ks = tile & 3;
        const int a = rt * 16 + (lane16 & 15);             // A-operand row
        const int t = a >> 5, r = a & 31;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const int b = 32 * ks + 8 * (lane16 >> 4) + 4 * half;  // first of 4 reduction indices
            const int S = b >> 4, jg = (b >> 3) & 1, h = (b >> 2) & 1;
            const u32x2 w = {v[u][2 * half], v[u][2 * half + 1]};
            *reinterpret_cast<u32x2*>(W + ((size_t)((l * 4 + t) * 8 + S) * 64 + r + 32 * h) * 8 + jg * 4) = w;
        }
    }
}

__device__ __forceinline__ bf16x8 wfrag(const __bf16* W, int l, int t, int S, int lane) {
    return *reinterpret_cast<const bf16x8*>(W + ((size_t)((l * 4 + t) * 8 + S) * 64 + lane) * 8);
}

// acc[t] = Σ_S W(l, t, S) · B[S]
__device__ __forceinline__ void chain_gemm(f32x16 (&acc)[4], const __bf16* W, int l, const bf16x8 (&B)[8], int lane,
                                           bool skip = false) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
    if (skip) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][r] = (float)B[2 * t + (r >> 3)][r & 7];
        return;
    }
#pragma unroll
    for (int S = 0; S < 8; ++S)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = mfma32(wfrag(W, l, t, S, lane), B[S], acc[t]);
}

// Write the wave's 32x128 tile of values v (D layout) as bf16 into an R8 matrix [RP][128], rows
// [32*tile, 32*tile + 32): two passes of 16 rows through the wave's scratch.
__device__ __forceinline__ void store_r8(const f32x16 (&v)[4], __bf16* scr, __bf16* dst, int64_t tile, int lane,
                                         int ablate = 0) {
    if (ablate & 2) return;
    const int m = lane & 31, h = lane >> 5;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        if ((m >> 4) == u) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const bf16x4 w = {(__bf16)v[t][4 * g], (__bf16)v[t][4 * g + 1], (__bf16)v[t][4 * g + 2],
                                      (__bf16)v[t][4 * g + 3]};
                    *reinterpret_cast<bf16x4*>(scr + (m & 15) * SLD + 32 * t + 8 * g + 4 * h) = w;
                }
        }
        lds_fence();
        // item = (row octet o of this half, 4 columns c4): 8 rows x 8 B -> 4 R8 chunks of 16 B
        const int o = lane >> 5, c4 = lane & 31;
        bf16x4 rv[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) rv[q] = *reinterpret_cast<const bf16x4*>(scr + (8 * o + q) * SLD + 4 * c4);
        __bf16* p = dst + (((int64_t)tile * 4 + 2 * u + o) * H + 4 * c4) * 8;
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
            bf16x8 w;
#pragma unroll
            for (int q = 0; q < 8; ++q) w[q] = rv[q][cc];
            *reinterpret_cast<bf16x8*>(p + cc * 8) = w;
        }
        lds_fence();
    }
}

// Write the wave's tile of values v (D layout) as bf16 rows into a row-major [M][128] matrix
// (rows >= M skipped), as coalesced 16-byte row chunks through the scratch.
__device__ __forceinline__ void store_rows(const f32x16 (&v)[4], __bf16* scr, __bf16* dst, int64_t tile, int64_t M,
                                           int lane, int ablate = 0) {
    if (ablate & 8) return;
    const int m = lane & 31, h = lane >> 5;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        if ((m >> 4) == u) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const bf16x4 w = {(__bf16)v[t][4 * g], (__bf16)v[t][4 * g + 1], (__bf16)v[t][4 * g + 2],
                                      (__bf16)v[t][4 * g + 3]};
                    *reinterpret_cast<bf16x4*>(scr + (m & 15) * SLD + 32 * t + 8 * g + 4 * h) = w;
                }
        }
        lds_fence();
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int rr = 4 * p + (lane >> 4), c = (lane & 15) * 8;
            const u32x4 w = *reinterpret_cast<const u32x4*>(scr + rr * SLD + c);
            const int64_t row = (int64_t)tile * TR + 16 * u + rr;
            if (row < M) *reinterpret_cast<u32x4*>(dst + row * H + c) = w;
        }
        lds_fence();
    }
}

// ------------------------------------------------------------------------------------ forward
struct FwdIn {
    bf16x8 eb[8];   // layer-0 B operand: e[row][16S + 8(j>>2) + 4h + (j&3)]; also the residual
};
struct FwdProj {
    f4 pi[16];      // P_i[dst(row)][dcol(t, 4g, h) ..+3], index t*4 + g
    f4 pj[16];
};

// Loads are unconditional: rows past M read row M-1 (no branch, so no per-load wait); those rows'
// results are never stored row-major, and their saved R8/mask entries meet dZ = 0 in the backward.
__device__ __forceinline__ int64_t clamp_row(const int64_t row, int64_t M) { return row < M ? row : M - 1; }

__device__ __forceinline__ void fwd_load(FwdIn& in, const ChainFwdArgs& a, int64_t tile, int lane) {
    if (a.ablate & 1) tile = 0;  // diagnostics: every tile reads tile 0 (cache-resident)
    const int m = lane & 31, h = lane >> 5;
    const int64_t row = clamp_row(tile * TR + m, a.M);
    const __bf16* e = a.e + row * H + 4 * h;
#pragma unroll
    for (int S = 0; S < 8; ++S) {
        const u32x2 lo = *reinterpret_cast<const u32x2*>(e + 16 * S);
        const u32x2 hi = *reinterpret_cast<const u32x2*>(e + 16 * S + 8);
        u32x4 w = {lo[0], lo[1], hi[0], hi[1]};
        in.eb[S] = __builtin_bit_cast(bf16x8, w);
    }
}

// node-projection gathers of the tile (issued at tile start: the layer-0 GEMM covers their latency)
__device__ __forceinline__ void fwd_proj(FwdProj& in, const ChainFwdArgs& a, int64_t tile, int di, int dj, int lane) {
    const int h = lane >> 5;
    const float* pi = a.proj + (int64_t)di * (2 * H) + 4 * h;
    const float* pj = a.proj + (int64_t)dj * (2 * H) + H + 4 * h;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int off = 32 * (q >> 2) + 8 * (q & 3);
        in.pi[q] = *reinterpret_cast<const f4*>(pi + off);
        in.pj[q] = *reinterpret_cast<const f4*>(pj + off);
    }
}

__device__ __forceinline__ void fwd_idx(const ChainFwdArgs& a, int64_t tile, int lane, int& di, int& dj) {
    if (a.ablate & 1) tile = 0;
    const int64_t row = clamp_row(tile * TR + (lane & 31), a.M);
    di = a.proj_i[row];
    dj = a.proj_j[row];
}

// w = 2w + (v > 0): v_cmp to VCC, then add-with-carry — two instructions, no bit constants. After
// 32 pushes, element k of the word sits at bit 31 - k.
__device__ __forceinline__ unsigned push_bit(unsigned w, float v) {
    unsigned r;
    asm("v_cmp_lt_f32 vcc, 0, %2\n\tv_addc_co_u32 %0, vcc, %1, %1, vcc" : "=v"(r) : "v"(w), "v"(v) : "vcc");
    return r;
}

// all-ones if element k (0..31, pushed k-th) of w is set, else 0
__device__ __forceinline__ int bit_sel(unsigned w, int k) { return (int)(w << k) >> 31; }

// hidden-layer epilogue: v = relu(acc + bias), or relu(acc + P_i + P_j) for layer 0 (the node
// projection P_i carries b0); mask bits; next B operand.
__device__ __forceinline__ void fwd_hidden(f32x16 (&acc)[4], const float* bias, const FwdProj* in, bf16x8 (&B)[8],
                                           uint2& bits, int lane) {
    const int h = lane >> 5;
    unsigned w[2] = {0u, 0u};
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const f4 b = in ? in->pi[4 * t + g] + in->pj[4 * t + g]
                            : *reinterpret_cast<const f4*>(bias + 32 * t + 8 * g + 4 * h);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = 4 * g + i, k = 16 * t + r;
                const float v = fmaxf(acc[t][r] + b[i], 0.f);
                acc[t][r] = v;
                w[k >> 5] = push_bit(w[k >> 5], v);
                B[2 * t + (r >> 3)][r & 7] = (__bf16)v;
            }
        }
    bits = make_uint2(w[0], w[1]);
}

__global__ __launch_bounds__(NW * 64) void chain_fwd_kernel(ChainFwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __bf16* W = reinterpret_cast<__bf16*>(smem);
    float* vec = reinterpret_cast<float*>(smem + LDS_W);  // bias[4][H], scale[H]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __bf16* scr = reinterpret_cast<__bf16*>(smem + LDS_W + LDS_V) + wave * SROWS * SLD;
    const int m = lane & 31, h = lane >> 5;
    const int64_t stride = (int64_t)gridDim.x * NW;
    int64_t tile = (int64_t)blockIdx.x * NW + wave;
    const int64_t last = a.ntiles - 1;  // prefetch targets past the end are clamped (unconditional loads)
    // the first tile's inputs are in flight while the weights are staged
    FwdIn nxt;
    int di, dj;
    fwd_idx(a, min(tile, last), lane, di, dj);
    fwd_load(nxt, a, min(tile, last), lane);
    stage_weights(W, a.wpack, a.woff, a.wks, false);
    for (int i = threadIdx.x; i < 5 * H; i += NW * 64) vec[i] = i < 4 * H ? a.bias[i / H][i % H] : a.scale[i - 4 * H];
    __syncthreads();
    if (a.ablate & 16) return;  // diagnostics: staging only
    if (tile >= a.ntiles) return;
#pragma unroll
    for (int S = 0; S < 8; ++S) pin(nxt.eb[S]);
    pin(di);
    pin(dj);
    for (; tile < a.ntiles; tile += stride) {
        const FwdIn in = nxt;
        FwdProj pr;
        fwd_proj(pr, a, tile, di, dj, lane);

        int ndi, ndj;
        fwd_idx(a, min(tile + stride, last), lane, ndi, ndj);
        fwd_load(nxt, a, min(tile + stride, last), lane);
        const int64_t row = tile * TR + m;
        f32x16 accs[1][4];
        bf16x8 B[8];
        uint2 bits;
        // layer 0: e·W0aᵀ + P_i[dst] + P_j[src] + b0
        chain_gemm(accs[0], W, 0, in.eb, lane, a.ablate & 4);
        fwd_hidden(accs[0], vec, &pr, B, bits, lane);
        reinterpret_cast<uint2*>(a.mask)[tile * 64 + lane] = bits;
        store_r8(accs[0], scr, a.act8 + a.act_off[1], tile, lane, a.ablate);
#pragma unroll
        for (int l = 1; l < 3; ++l) {
            chain_gemm(accs[0], W, l, B, lane, a.ablate & 4);
            fwd_hidden(accs[0], vec + l * H, nullptr, B, bits, lane);
            reinterpret_cast<uint2*>(a.mask)[l * a.mask_stride + tile * 64 + lane] = bits;
            store_r8(accs[0], scr, a.act8 + a.act_off[l + 1], tile, lane, a.ablate);
        }
        // layer 3 + RMSNorm + residual
        f32x16 (&acc)[4] = accs[0];
        chain_gemm(acc, W, 3, B, lane, a.ablate & 4);
        float ss = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f4 b = *reinterpret_cast<const f4*>(vec + 3 * H + 32 * t + 8 * g + 4 * h);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float z = acc[t][4 * g + i] + b[i];
                    acc[t][4 * g + i] = z;
                    ss += z * z;
                }
            }
        ss += __shfl_xor(ss, 32);
        const float q = sqrtf(ss) * a.dinv + RMS_EPS;
        const float rq = __builtin_amdgcn_rcpf(q);  // bf16 outputs: z·(1/q) is within 2 fp32 ulp of z/q
        if (h == 0 && row < a.M) a.rden_save[row] = q;
        store_rows(acc, scr, a.z_save, tile, a.M, lane, a.ablate);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f4 s = *reinterpret_cast<const f4*>(vec + 4 * H + 32 * t + 8 * g + 4 * h);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int r = 4 * g + i;
                    acc[t][r] = fmaf(s[i], acc[t][r] * rq, (float)in.eb[2 * t + (r >> 3)][r & 7]);
                }
            }
        store_rows(acc, scr, a.out, tile, a.M, lane, a.ablate);
#pragma unroll
        for (int S = 0; S < 8; ++S) pin(nxt.eb[S]);
        pin(ndi);
        pin(ndj);
        di = ndi;
        dj = ndj;
    }
}

// ------------------------------------------------------------------------------------ backward
struct BwdIn {   // raw bf16: features dcol(t, 4g, h)..+3, index t*4 + g
    u32x2 d[16];    // de_out[row]
    u32x2 g[16];    // d_aggr[dst(row)]
    u32x2 z[16];    // z[row]
    float q;
    uint2 mask[3];     // ReLU bits of hidden layers 0..2 (forward layout)
};

__device__ __forceinline__ f4 bf4(u32x2 v) {
    const bf16x4 b = __builtin_bit_cast(bf16x4, v);
    return f4{(float)b[0], (float)b[1], (float)b[2], (float)b[3]};
}

__device__ __forceinline__ void bwd_load(BwdIn& in, const ChainBwdArgs& a, int64_t tile, int gi, int lane) {
    if (a.ablate & 1) tile = 0;  // diagnostics: every tile reads tile 0 (cache-resident)
    const int m = lane & 31, h = lane >> 5;
    const int64_t row = clamp_row(tile * TR + m, a.M);
    const __bf16* d = a.dout + row * H + 4 * h;
    const __bf16* g = a.gath + (int64_t)gi * H + 4 * h;
    const __bf16* z = a.z_save + row * H + 4 * h;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int off = 32 * (q >> 2) + 8 * (q & 3);
        in.d[q] = *reinterpret_cast<const u32x2*>(d + off);
        in.g[q] = *reinterpret_cast<const u32x2*>(g + off);
        in.z[q] = *reinterpret_cast<const u32x2*>(z + off);
    }
    in.q = a.rden_save[row];
#pragma unroll
    for (int l = 0; l < 3; ++l) in.mask[l] = reinterpret_cast<const uint2*>(a.mask)[l * a.mask_stride + tile * 64 + lane];
}

__device__ __forceinline__ int bwd_idx(const ChainBwdArgs& a, int64_t tile, int lane) {
    if (a.ablate & 1) tile = 0;
    return a.gath_idx[clamp_row(tile * TR + (lane & 31), a.M)];
}

__global__ __launch_bounds__(NW * 64) void chain_bwd_kernel(ChainBwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __bf16* W = reinterpret_cast<__bf16*>(smem);
    float* vec = reinterpret_cast<float*>(smem + LDS_W);  // scale[H], then dscale reduction [NW][H]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __bf16* scr = reinterpret_cast<__bf16*>(smem + LDS_W + LDS_V) + wave * SROWS * SLD;
    const int m = lane & 31, h = lane >> 5;
    const int64_t stride = (int64_t)gridDim.x * NW;
    int64_t tile = (int64_t)blockIdx.x * NW + wave;
    const int64_t last = a.ntiles - 1;  // prefetch targets past the end are clamped (unconditional loads)
    // the first tile's inputs are in flight while the weights are staged
    const int gi0 = bwd_idx(a, min(tile, last), lane);
    stage_weights(W, a.wtpack, a.woff, a.wks, true);
    BwdIn nxt;
    bwd_load(nxt, a, min(tile, last), gi0, lane);
    for (int i = threadIdx.x; i < H; i += NW * 64) vec[i] = a.scale[i];
    __syncthreads();
    if (a.ablate & 16) return;  // diagnostics: staging only

    f4 dsc[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) dsc[q] = f4{0.f, 0.f, 0.f, 0.f};
    int ngi = 0;
    if (tile < a.ntiles) {
        ngi = bwd_idx(a, min(tile + stride, last), lane);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            pin(nxt.d[q]);
            pin(nxt.g[q]);
            pin(nxt.z[q]);
        }
        pin(nxt.q);
#pragma unroll
        for (int l = 0; l < 3; ++l) pin(nxt.mask[l]);
        pin(ngi);
    }
    for (; tile < a.ntiles; tile += stride) {
        const int64_t row = tile * TR + m;
        const bool ok = row < a.M;
        // RMSNorm backward (layers.py:59-74): dz = s·dy/q − z·(Σ s·dy·z)/(q²·rms)·(1/H), from the
        // prefetched tile; its registers are then free for the next tile's prefetch.
        f32x16 accs[1][4];
        f32x16 (&acc)[4] = accs[0];  // dy, then dz
        float dot = 0.f;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const f4 dy = bf4(nxt.d[q]) + bf4(nxt.g[q]);
            const f4 z = bf4(nxt.z[q]);
            const f4 sc = *reinterpret_cast<const f4*>(vec + 32 * (q >> 2) + 8 * (q & 3) + 4 * h);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                acc[q >> 2][4 * (q & 3) + i] = dy[i];
                dot += sc[i] * dy[i] * z[i];
            }
        }
        dot += __shfl_xor(dot, 32);
        const float qd = nxt.q;
        const float rq = __builtin_amdgcn_rcpf(qd);  // bf16 dZ: ·(1/q) within 2 fp32 ulp of /q
        const float rms = qd - RMS_EPS;
        const float coef = rms > 0.f ? dot / (qd * qd * rms) * (a.dinv * a.dinv) : 0.f;
        bf16x8 B[8];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const f4 z = bf4(nxt.z[q]);
            const f4 sc = *reinterpret_cast<const f4*>(vec + 32 * (q >> 2) + 8 * (q & 3) + 4 * h);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int t = q >> 2, r = 4 * (q & 3) + i;
                const float dy = acc[t][r];
                const float dz = ok ? fmaf(-z[i], coef, sc[i] * dy * rq) : 0.f;
                dsc[q][i] = fmaf(ok ? dy * z[i] : 0.f, rq, dsc[q][i]);
                acc[t][r] = dz;
                B[2 * t + (r >> 3)][r & 7] = (__bf16)dz;
            }
        }
        u32x2 dcur[16];  // de_out of this tile, for the layer-0 residual
#pragma unroll
        for (int q = 0; q < 16; ++q) dcur[q] = nxt.d[q];
        uint2 mcur[3];
#pragma unroll
        for (int l = 0; l < 3; ++l) mcur[l] = ok ? nxt.mask[l] : make_uint2(0u, 0u);
        __builtin_amdgcn_sched_barrier(0);
        bwd_load(nxt, a, min(tile + stride, last), ngi, lane);
        const int ngi2 = bwd_idx(a, min(tile + 2 * stride, last), lane);
        store_r8(acc, scr, a.dz8 + 3 * a.RP * H, tile, lane, a.ablate);
        // layers 3..1: dZ_{l-1} = (dZ_l · W_l) ⊙ [A_l > 0]
#pragma unroll
        for (int l = 3; l >= 1; --l) {
            f32x16 (&c)[4] = accs[0];
            chain_gemm(c, W, l, B, lane, a.ablate & 4);
            const unsigned bw[2] = {mcur[l - 1].x, mcur[l - 1].y};
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int k = 16 * t + r;  // bit -> all-ones / zero lane mask (v_bfe_i32), then AND
                    const int sel = bit_sel(bw[k >> 5], k & 31);
                    const float v = __int_as_float(__float_as_int(c[t][r]) & sel);
                    c[t][r] = v;
                    B[2 * t + (r >> 3)][r & 7] = (__bf16)v;
                }
            store_r8(c, scr, a.dz8 + (int64_t)(l - 1) * a.RP * H, tile, lane, a.ablate);
            if (l == 1) store_rows(c, scr, a.dz0, tile, a.M, lane, a.ablate);
        }
        // layer 0, e block: de = de_out + dZ0 · W0a
        chain_gemm(acc, W, 0, B, lane, a.ablate & 4);
        // rows past M are not stored
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f4 o = bf4(dcur[4 * t + g]);
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[t][4 * g + i] = o[i] + acc[t][4 * g + i];
            }
        store_rows(acc, scr, a.de, tile, a.M, lane, a.ablate);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            pin(nxt.d[q]);
            pin(nxt.g[q]);
            pin(nxt.z[q]);
        }
        pin(nxt.q);
#pragma unroll
        for (int l = 0; l < 3; ++l) pin(nxt.mask[l]);
        pin(ngi2);
        ngi = ngi2;
    }
    // dscale partials: sum over the 32 rows of each lane half, then over the waves
#pragma unroll
    for (int q = 0; q < 16; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float v = dsc[q][i];
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) v += __shfl_xor(v, o);
            dsc[q][i] = v;
        }
    __syncthreads();
    float* red = vec + H;  // [NW][H]
    if (m == 0) {
#pragma unroll
        for (int q = 0; q < 16; ++q) *reinterpret_cast<f4*>(red + wave * H + 32 * (q >> 2) + 8 * (q & 3) + 4 * h) = dsc[q];
    }
    __syncthreads();
    if (threadIdx.x < H) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) t += red[w * H + threadIdx.x];
        a.dscale_part[(int64_t)blockIdx.x * H + threadIdx.x] = t;
    }
}

int set_lds_once(const void* fn, size_t bytes) {
    static std::mutex mu;
    static bool done[2] = {false, false};
    std::lock_guard<std::mutex> lk(mu);
    const int slot = fn == (const void*)chain_fwd_kernel ? 0 : 1;
    if (done[slot]) return 0;
    MGN_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    done[slot] = true;
    return 0;
}

// diagnostics only: MGN_ABLATE (results are wrong when nonzero)
int ablate_env() {
    const char* e = getenv("MGN_ABLATE");
    return e ? atoi(e) : 0;
}

int chain_grid(int64_t ntiles) {
    const int cus = device_cus();
    const int64_t groups = cdiv64(ntiles, NW);
    return (int)(groups < cus ? groups : cus);
}

void layer_offsets(const mgn_mlp* m, int64_t* woff, int* wks) {
    int64_t o = 0;
    for (int l = 0; l < 4; ++l) {
        int n, k;
        mlp_layer_shape(*m, l, &n, &k);
        woff[l] = o;
        wks[l] = cdiv(k, 32);
        o += linear_pack_elems(n, k, MGN_BF16);
    }
}

}  // namespace

bool chain_eligible(const mgn_mlp* m) {
    return m->dtype == MGN_BF16 && m->hidden == H && m->in_dim == 3 * H && m->out_dim == H && m->n_layers == 4 &&
           m->has_norm;
}

int chain_edge_forward(const mgn_mlp* m, const void* e, const float* proj, const int32_t* pi, const int32_t* pj,
                       int64_t M, void* out, mgn_mlp_saved* sv, hipStream_t st) {
    ChainFwdArgs a;
    memset(&a, 0, sizeof(a));
    a.e = reinterpret_cast<const __bf16*>(e);
    a.proj = proj;
    a.proj_i = pi;
    a.proj_j = pj;
    a.wpack = reinterpret_cast<const __bf16*>(m->wpack);
    layer_offsets(m, a.woff, a.wks);
    for (int l = 0; l < 4; ++l) a.bias[l] = m->bias[l];
    a.scale = m->scale;
    a.dinv = (float)(1.0 / sqrt((double)H));
    a.M = M;
    a.ntiles = rows_pad(M) / TR;  // every padded row: R8 saves and masks cover rows_pad(M)
    a.out = reinterpret_cast<__bf16*>(out);
    a.z_save = reinterpret_cast<__bf16*>(sv->z);
    a.rden_save = sv->rden;
    a.act8 = reinterpret_cast<__bf16*>(sv->act);
    for (int l = 0; l < 4; ++l) a.act_off[l] = act_off(*m, M, l, 1);
    a.mask = reinterpret_cast<unsigned long long*>(sv->mask);
    a.mask_stride = mask_words_per_layer(*m, M);
    a.ablate = ablate_env();
    if (a.ntiles == 0) return 0;
    if (int e2 = set_lds_once((const void*)chain_fwd_kernel, LDS_TOTAL)) return e2;
    ProfScope ps(PROF_FWD_EDGE, st);
    hipLaunchKernelGGL(chain_fwd_kernel, dim3(chain_grid(a.ntiles)), dim3(NW * 64), LDS_TOTAL, st, a);
    MGN_LAUNCH_CHECK();
    return 0;
}

int chain_edge_backward(const mgn_mlp* m, int64_t M, const mgn_mlp_saved* sv, const void* dout, const void* gath,
                        const int32_t* gath_idx, void* dz8, float* dscale_part, int* nparts, void* de, void* dz0,
                        hipStream_t st) {
    ChainBwdArgs a;
    memset(&a, 0, sizeof(a));
    a.dout = reinterpret_cast<const __bf16*>(dout);
    a.gath = reinterpret_cast<const __bf16*>(gath);
    a.gath_idx = gath_idx;
    a.z_save = reinterpret_cast<const __bf16*>(sv->z);
    a.rden_save = sv->rden;
    a.scale = m->scale;
    a.dinv = (float)(1.0 / sqrt((double)H));
    a.mask = reinterpret_cast<const unsigned long long*>(sv->mask);
    a.mask_stride = mask_words_per_layer(*m, M);
    a.wtpack = reinterpret_cast<const __bf16*>(m->wtpack);
    layer_offsets(m, a.woff, a.wks);
    a.M = M;
    a.ntiles = rows_pad(M) / TR;  // every padded row: R8 saves and masks cover rows_pad(M)
    a.dz8 = reinterpret_cast<__bf16*>(dz8);
    a.RP = rows_pad(M);
    a.dscale_part = dscale_part;
    a.de = reinterpret_cast<__bf16*>(de);
    a.dz0 = reinterpret_cast<__bf16*>(dz0);
    a.ablate = ablate_env();
    *nparts = 0;
    if (a.ntiles == 0) return 0;
    if (int e2 = set_lds_once((const void*)chain_bwd_kernel, LDS_TOTAL)) return e2;
    const int grid = chain_grid(a.ntiles);
    *nparts = grid;
    ProfScope ps(PROF_BWD_EDGE, st);
    hipLaunchKernelGGL(chain_bwd_kernel, dim3(grid), dim3(NW * 64), LDS_TOTAL, st, a);
    MGN_LAUNCH_CHECK();
    return 0;
}

size_t chain_lds_bytes() { return LDS_TOTAL; }

// 16 (default): mgn_chain16.hip, 16-row tiles, two waves per SIMD. 32: the 32x32x16 kernels above
// (one wave per SIMD), kept for A/B measurement. Read once: forward and backward must agree on the
// ReLU-mask layout.
int chain_variant() {
    static const int v = [] {
        const char* e = getenv("MGN_CHAIN");
        return e && atoi(e) == 32 ? 32 : 16;
    }();
    return v;
}
