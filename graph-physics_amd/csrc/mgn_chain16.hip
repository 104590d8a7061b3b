// Register-chained edge-MLP kernels on 16-row tiles (v_mfma_f32_16x16x32_bf16), bf16, h=128.
//
// One wave runs the whole 4-Linear chain of its edges (weights resident in LDS, accumulators
// chained as the next layer's B operand), on 16x16x32 tiles: a wave
// owns 16 edges, its accumulator is 8 f32x4 (32 VGPRs) instead of 64, so TWO waves fit per SIMD
// (8 waves per workgroup share one 128 KiB weight image) and one wave's epilogue VALU overlaps the
// other's MFMAs and memory traffic.
//
// Lane l: edge m = l&15, group g = l>>4. Accumulator tile t (16 features): lane holds features
// 16t + 4g + r, r = 0..3. B operand k-step s (32 features): element j of lane group g is feature
// 32s + 16(j>>2) + 4g + (j&3) = accumulator (t = 2s + (j>>2), r = j&3): the next layer's operand
// is the accumulator with no data movement, given weights staged in that permuted k order.
// ReLU masks: 32 bits per lane (bit 4t + r) per tile and layer; the backward has the same map.
#include <cmath>
#include <utility>
#include <cstring>
#include <mutex>
#include <type_traits>

#include "mgn_chain.h"
#include "mgn_chain16_dev.h"

// Diagnostics builds only (-DMGN_ABLATE=bits, results wrong when nonzero; see mgn_mlp.hip): edge
// forward 1 = P gathers from row 0 (cache-resident), 2 = no P loads, 4 = no weight-staging loads,
// 8 = no stores of outputs / saves; node forward 16 = no aggregation gathers; node kernels 32 = every
// global weight fragment read from fragment 0 (L1-hot: the cost of streaming them from L2), 64 = the
// same for the hand-off's projection fragments only
#ifndef MGN_ABLATE
#define MGN_ABLATE 0
#endif
#ifndef MGN_DIRECT_ROWS
#define MGN_DIRECT_ROWS 0
#endif


#ifndef MGN_PROJ_HANDOFF
#define MGN_PROJ_HANDOFF 1  // A/B builds: 0 = the tile wave computes the next block's projections itself
#endif

#ifndef MGN_BWD_HANDOFF
#define MGN_BWD_HANDOFF 1  // A/B builds: 0 = the node backward's tile wave computes d_aggr itself
#endif

#ifndef MGN_NODE_AG
#define MGN_NODE_AG 6  // in-edges gathered per round trip by the node-MLP aggregation (8 spills)
#endif

namespace {

constexpr int SLD = H + 8;             // scratch row stride (bf16)
constexpr int SROWS = 8;               // scratch rows (one R8 octet per pass)
constexpr size_t LDS_W = (size_t)4 * LFR * FRAG * 2;   // 128 KiB
constexpr size_t LDS_V = (size_t)6 * H * 4;             // 4 bias vectors + scale (+ edge scale: node MLP)
constexpr size_t LDS_S = (size_t)NW * SROWS * SLD * 2;  // per-wave transpose scratch
constexpr size_t LDS_R = (size_t)NW * H * 4;            // backward: per-wave dscale partials
constexpr size_t LDS_TOTAL = LDS_W + LDS_V + LDS_S + LDS_R;

// edge kernels, per waves-per-workgroup NWK (8: two waves per SIMD; 12: three): forward = weights |
// bias[4] + scale | scratch, backward = weights | scale | scratch | dscale partials (12 waves: 160 KiB)
constexpr size_t LDS_VF = (size_t)5 * H * 4, LDS_VB = (size_t)H * 4;
constexpr size_t lds_fwd(int nwk) { return LDS_W + LDS_VF + (size_t)nwk * SROWS * SLD * 2; }
constexpr size_t lds_bwd(int nwk) { return LDS_W + LDS_VB + (size_t)nwk * SROWS * SLD * 2 + (size_t)nwk * H * 4; }
static_assert(lds_bwd(12) <= 163840, "12-wave edge backward exceeds 160 KiB of LDS");
static_assert(SROWS * SLD * 2 >= 64 * 32, "a wave scratch holds half a 16-row bf16 B operand (partner hand-offs)");

// Diagnostics (build with -DMGN_STAMPS, e.g. MGN_STAMPS=1 python __graft_entry__.py): per-phase
// s_memtime deltas of wave 0 of workgroup 0, printed once per launch. Not in normal builds.
#ifdef MGN_STAMPS
#define STAMP_DECL                                                                                      \
    unsigned long long st_prev = __builtin_amdgcn_s_memtime(), st_ph[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}
#define STAMP(i)                                                                                        \
    do {                                                                                                \
        __builtin_amdgcn_sched_barrier(0);                                                              \
        unsigned long long st_t;                                                                        \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_t)::"memory");                   \
        __builtin_amdgcn_sched_barrier(0);                                                              \
        st_ph[i] += st_t - st_prev;                                                                     \
        st_prev = st_t;                                                                                 \
    } while (0)
#define STAMP_PRINT(name)                                                                               \
    if (blockIdx.x == 0 && threadIdx.x == 0)                                                            \
    printf("%s %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu\n", name, st_ph[0], st_ph[1],  \
           st_ph[2], st_ph[3], st_ph[4], st_ph[5], st_ph[6], st_ph[7], st_ph[8], st_ph[9], st_ph[10], st_ph[11])
// per-wave start / end (s_memrealtime, 100 MHz, one clock for the whole device) of the last launch
// of each chained kernel kind, read back by mgn_debug_wave_times (the launch's spread of wave ends)
__device__ unsigned long long g_wave_t[4][4096][2];
#define WAVE_T0 const unsigned long long wave_t0 = __builtin_amdgcn_s_memrealtime()
#define WAVE_REC(k)                                                                                     \
    do {                                                                                                \
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();                                \
        const int wi = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);                            \
        if ((threadIdx.x & 63) == 0 && wi < 4096) {                                                    \
            g_wave_t[k][wi][0] = wave_t0;                                                              \
            g_wave_t[k][wi][1] = t1;                                                                   \
        }                                                                                               \
    } while (0)
#else
#define STAMP_DECL
#define STAMP(i)
#define STAMP_PRINT(name)
#define WAVE_T0
#define WAVE_REC(k)
#endif



template <class T>
__device__ __forceinline__ void pin(const T& v) { asm volatile("" ::"v"(v)); }


// the 4 components of v summed over the 16 lanes of a DPP row, transposing as it goes: lane m
// returns the total of component 2(m&1) + ((m>>1)&1) (pairs m^1 trade two components, pairs m^2
// one, then rotations by 4 and 8 add the four lanes holding the same component): 6 DPP adds for
// four sums instead of 16
__device__ __forceinline__ float row16_sum4(const f4& v, int m) {
    const bool odd = m & 1, b1 = (m >> 1) & 1;
    const float s0 = odd ? v[0] : v[2], s1 = odd ? v[1] : v[3];
    float k0 = odd ? v[2] : v[0], k1 = odd ? v[3] : v[1];
    k0 += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s0), 0xB1, 0xF, 0xF, false));
    k1 += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s1), 0xB1, 0xF, 0xF, false));
    const float sb = b1 ? k0 : k1;
    float k = b1 ? k1 : k0;
    k += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(sb), 0x4E, 0xF, 0xF, false));
    k += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(k), 0x124, 0xF, 0xF, false));  // row_ror:4
    k += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(k), 0x128, 0xF, 0xF, false));  // row_ror:8
    return k;
}

__device__ __forceinline__ int64_t clamp_row(int64_t row, int64_t M) { return row < M ? row : M - 1; }

// w = 2w + (v > 0): v_cmp sets vcc, v_addc shifts it in (2 instructions, no constants)
__device__ __forceinline__ unsigned push_bit(unsigned w, float v) {
    unsigned r;
    asm("v_cmp_lt_f32 vcc, 0, %2\n\tv_addc_co_u32 %0, vcc, %1, %1, vcc" : "=v"(r) : "v"(w), "v"(v) : "vcc");
    return r;
}
__device__ __forceinline__ int bit_sel(unsigned w, int k) { return (int)(w << k) >> 31; }

// acc (tile layout, element 4t + r) &= sign-extended bit 31 - (4t + r) of w: one v_bfe_i32 + v_and
// per element (left to the compiler, the select becomes v_cmp + v_cndmask with SGPR-hazard s_nops)
template <int K>
__device__ __forceinline__ int bfe_sel(unsigned w) {
    int r;
    asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(r) : "v"(w), "n"(31 - K));
    return r;
}
template <int... K>
__device__ __forceinline__ void relu_mask_seq(f4 (&acc)[8], unsigned w, std::integer_sequence<int, K...>) {
    ((acc[K >> 2][K & 3] = __int_as_float(__float_as_int(acc[K >> 2][K & 3]) & bfe_sel<K>(w))), ...);
}
__device__ __forceinline__ void relu_mask(f4 (&acc)[8], unsigned w) {
    relu_mask_seq(acc, w, std::make_integer_sequence<int, 32>{});
}


// One layer's GEMM that also stores its B operand (= the layer's input, bf16) as R8 octets and/or
// row-major rows through the wave's 8-row scratch, with the LDS round trips placed between the
// k-steps so they run under the MFMAs: write octet 0 | k0 | read 0 | k1 | store 0, write octet 1 |
// k2 | read 1 | k3 | store 1. The fences only order the wave's own scratch writes and reads.
struct StoreDst {
    __bf16* r8;    // R8 [RP][128] (octets 2*tile, 2*tile+1) or nullptr
    __bf16* rows;  // row-major [M][128] (rows >= M skipped) or nullptr
};

__device__ __forceinline__ void gemm16_st(f4 (&acc)[8], const __bf16* W, int l, const bf16x8 (&B)[4], int lane,
                                          __bf16* scr, StoreDst d, int64_t tile, int64_t M,
                                          const float* bias = nullptr) {
    const int m = lane & 15, g = lane >> 4;
    acc_init(acc, bias, lane);
    u32x2 rv[8];
    u32x4 rw[2];
    auto write = [&](int u) {
        if ((m >> 3) == u) {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const u32x4 b = __builtin_bit_cast(u32x4, B[t >> 1]);
                const u32x2 w = (t & 1) ? u32x2{b[2], b[3]} : u32x2{b[0], b[1]};
                *reinterpret_cast<u32x2*>(scr + (m & 7) * SLD + 16 * t + 4 * g) = w;
            }
        }
    };
    auto read = [&]() {
        if (d.r8) {
#pragma unroll
            for (int q = 0; q < 8; ++q) rv[q][0] = *reinterpret_cast<const unsigned*>(scr + q * SLD + 2 * lane);
        }
        if (d.rows) {
#pragma unroll
            for (int p = 0; p < 2; ++p)
                rw[p] = *reinterpret_cast<const u32x4*>(scr + (4 * p + (lane >> 4)) * SLD + (lane & 15) * 8);
        }
    };
    auto store = [&](int u) {
        if (MGN_ABLATE & 8) return;
        if (d.r8) {
            bf16x8 c0, c1;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const bf16x2 p = __builtin_bit_cast(bf16x2, rv[q][0]);
                c0[q] = p[0];
                c1[q] = p[1];
            }
            __bf16* p = d.r8 + (((int64_t)tile * 2 + u) * H + 2 * lane) * 8;
            *reinterpret_cast<bf16x8*>(p) = c0;
            *reinterpret_cast<bf16x8*>(p + 8) = c1;
        }
        if (d.rows) {
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                const int64_t row = tile * TR + 8 * u + 4 * p + (lane >> 4);
                if (row < M) *reinterpret_cast<u32x4*>(d.rows + row * H + (lane & 15) * 8) = rw[p];
            }
        }
    };
    auto kstep = [&](int s) {
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = mfma16(wfrag(W, l, t, s, lane), B[s], acc[t]);
        __builtin_amdgcn_sched_barrier(0);
    };
    write(0);
    kstep(0);
    lds_fence();
    read();
    kstep(1);
    store(0);
    lds_fence();  // octet 0's reads are back before octet 1 overwrites the scratch
    write(1);
    kstep(2);
    lds_fence();
    read();
    kstep(3);
    store(1);
    lds_fence();  // scratch free for the next user
}



// write this lane's 32 values of row m (&7) of one octet into the scratch (P2: pair layout)
template <bool P2 = false>
__device__ __forceinline__ void scr_write(const f4 (&v)[8], __bf16* scr, int lane) {
    const int m = lane & 15, g = lane >> 4;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const bf16x4 w = {(__bf16)v[t][0], (__bf16)v[t][1], (__bf16)v[t][2], (__bf16)v[t][3]};
        *reinterpret_cast<bf16x4*>(scr + (m & 7) * SLD + col_of<P2>(t, g)) = w;
    }
}

// The wave's 16x128 tile (D layout) as bf16 into an R8 matrix [RP][128], octets 2*tile, 2*tile+1.
__device__ __forceinline__ void store_r8(const f4 (&v)[8], __bf16* scr, __bf16* dst, int64_t tile, int lane) {
    const int m = lane & 15;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        if ((m >> 3) == u) scr_write(v, scr, lane);
        lds_fence();
        // lane = column pair: 8 rows x 4 B -> 2 R8 chunks (32 contiguous bytes per lane)
        u32x2 rv[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) rv[q][0] = *reinterpret_cast<const unsigned*>(scr + q * SLD + 2 * lane);
        bf16x8 c0, c1;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const bf16x2 p = __builtin_bit_cast(bf16x2, rv[q][0]);
            c0[q] = p[0];
            c1[q] = p[1];
        }
        __bf16* p = dst + (((int64_t)tile * 2 + u) * H + 2 * lane) * 8;
        if (!(MGN_ABLATE & 8)) {
            *reinterpret_cast<bf16x8*>(p) = c0;
            *reinterpret_cast<bf16x8*>(p + 8) = c1;
        }
        lds_fence();
    }
}

// The wave's tile as bf16 rows of a row-major [M][128] matrix (rows >= M skipped), 16-byte stores
// (P2: each row in the pair layout).
template <bool P2 = false>
__device__ __forceinline__ void store_rows(const f4 (&v)[8], __bf16* scr, __bf16* dst, int64_t tile, int64_t M,
                                           int lane, int64_t ld = H) {
    const int m = lane & 15;
#if MGN_DIRECT_ROWS
    // straight from the accumulator layout: 8 stores of 8 B per lane (each wave instruction writes
    // 32 contiguous bytes of 16 rows; the rows complete in L2), no LDS round trip or fence
    (void)scr;
    const int64_t row = tile * TR + m;
    if (row < M && !(MGN_ABLATE & 8)) {
        __bf16* p = dst + row * ld;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const bf16x4 w = {(__bf16)v[t][0], (__bf16)v[t][1], (__bf16)v[t][2], (__bf16)v[t][3]};
            *reinterpret_cast<bf16x4*>(p + col_of<P2>(t, lane >> 4)) = w;
        }
    }
    return;
#endif
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        if ((m >> 3) == u) scr_write<P2>(v, scr, lane);
        lds_fence();
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int rr = 4 * p + (lane >> 4), c = (lane & 15) * 8;
            const u32x4 w = *reinterpret_cast<const u32x4*>(scr + rr * SLD + c);
            const int64_t row = tile * TR + 8 * u + rr;
            if (row < M && !(MGN_ABLATE & 8)) *reinterpret_cast<u32x4*>(dst + row * ld + c) = w;
        }
        lds_fence();
    }
}

int chain16_grid(int64_t ntiles, int nwk = NW) {
    const int cus = device_cus();
    const int64_t groups = cdiv64(ntiles, nwk);
    return (int)(groups < cus ? groups : cus);
}

// waves per workgroup of the edge kernels: 12 (three per SIMD) for both. Cfg B: forward 40.9 vs
// 42.5 us at 8; backward 47.9 vs 50.6 us, with its d_aggr gather loaded by the tile instead of
// prefetched (prefetched, the 168-VGPR cap spills 17 registers: 54.7 us). Compile-time (A/B builds:
// -DMGN_EDGE_WAVES=8 / -DMGN_EDGE_BWD_WAVES=8); no runtime switch.
#ifndef MGN_EDGE_WAVES
#define MGN_EDGE_WAVES 12
#endif
#ifndef MGN_EDGE_BWD_WAVES
#define MGN_EDGE_BWD_WAVES 12
#endif
static_assert((MGN_EDGE_WAVES == 8 || MGN_EDGE_WAVES == 12) && (MGN_EDGE_BWD_WAVES == 8 || MGN_EDGE_BWD_WAVES == 12),
              "edge kernels run 8 or 12 waves per workgroup");
constexpr int edge_waves() { return MGN_EDGE_WAVES; }
constexpr int edge_bwd_waves() { return MGN_EDGE_BWD_WAVES; }


// ------------------------------------------------------------------------------------ forward
struct In16 {
    bf16x8 eb[4];  // layer-0 B operand = e[row][32s + 16(j>>2) + 4g + (j&3)]; also the residual
};

__device__ __forceinline__ void load_e(In16& in, const ChainFwdArgs& a, int64_t tile, int lane) {
    const int64_t row = clamp_row(tile * TR + (lane & 15), a.M);
    const __bf16* e = a.e + row * H + 4 * (lane >> 4);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const u32x2 lo = *reinterpret_cast<const u32x2*>(e + 32 * s);
        const u32x2 hi = *reinterpret_cast<const u32x2*>(e + 32 * s + 16);
        const u32x4 w = {lo[0], lo[1], hi[0], hi[1]};
        in.eb[s] = __builtin_bit_cast(bf16x8, w);
    }
}

__device__ __forceinline__ void load_idx(const ChainFwdArgs& a, int64_t tile, int lane, int& di, int& dj) {
    const int64_t row = clamp_row(tile * TR + (lane & 15), a.M);
    di = a.proj_i[row];
    dj = a.proj_j[row];
}

// EdgeAgg (round 6): the dst of the rows adjoining the tile — lane 0 gets row 16·tile − 1's, lane 15 row
// 16·tile + 16's (-1 where there is none); the other lanes' values are unused
__device__ __forceinline__ int load_nb(const int32_t* dst, int64_t M, int64_t tile, int lane) {
    const int m = lane & 15;
    const int64_t r = m == 0 ? tile * TR - 1 : tile * TR + TR;
    const bool ok = r >= 0 && r < M && (m == 0 || m == 15);
    const int v = dst[ok ? r : 0];
    return ok ? v : -1;
}

// EdgeAgg: the per-edge terms v = z / q (this lane's row m, features 16t + 4g + r; the fp32 z the output
// is made of — the RMSNorm scale s multiplies the sum in the node forward) summed over each run of equal
// dst among the tile's 16 rows, and the sum stored as one fp32 row: a segment that starts and ends in this
// tile into agg_full[dst], the run continuing from the previous tile into agg_head[tile], the one
// continuing into the next tile into agg_tail[tile] (rows sorted by dst: at most one of each per tile).
// The runs are found from a ballot of lanes whose dst differs from the previous row's (wave-uniform: the
// four DPP rows of lane groups g hold the same rows), and each run is reduced over the 16 lanes with a
// transposing butterfly — xor 1 and xor 2 (quad_perm) exchange half of the lane's values each, rotations
// by 4 and 8 add the quads — after which lane m < 4 holds the run's features 16t + 4g .. +3 for t = m and
// m + 4: two 16-byte stores per lane, one 512-byte row per run (store instructions, not bytes, are what
// this kernel pays for). Fixed order: deterministic; the node forward adds a segment's rows in tile order.
#ifndef MGN_EAGG_ABL
#define MGN_EAGG_ABL 0  // diagnostics builds only (results wrong): 1 no partial stores, 4 nothing
#endif
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {  // within-row permutes only: every source lane is valid
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
// one run (lanes [r0, r1] of each row; all = the whole tile) reduced as above: half h of the lane's values
// (t = 4h .. 4h + 3) into u (t = 4h + (m & 3)); halves one at a time keep the temporaries at 12 registers
template <bool ALL, class V>
__device__ __forceinline__ f4 run_reduce_half(const V& v, int h, int m, int r0, int r1) {
    const bool in = ALL || (m >= r0 && m <= r1);
    const bool o1 = m & 1, o2 = (m >> 1) & 1;
    f4 u1[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float a0 = in ? v(4 * h + 2 * j, r) : 0.f, a1 = in ? v(4 * h + 2 * j + 1, r) : 0.f;
            u1[j][r] = (o1 ? a1 : a0) + dpp_f<0xB1>(o1 ? a0 : a1);  // xor 1: t parity
        }
    f4 u;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float w = (o2 ? u1[1][r] : u1[0][r]) + dpp_f<0x4E>(o2 ? u1[0][r] : u1[1][r]);  // xor 2: t bit 1
        w += dpp_f<0x124>(w);                                                            // row_ror:4
        u[r] = w + dpp_f<0x128>(w);                                                      // row_ror:8
    }
    return u;
}
struct AggOut {
    float *full, *head, *tail;
    int64_t M;
};
// v(t, r): the lane's term of feature 16t + 4g + r
template <class V>
__device__ __forceinline__ void edge_agg_store(const V& v, int di, int nb, int64_t tile, int lane, const AggOut& a) {
    if (MGN_EAGG_ABL & 4) return;
    const int m = lane & 15, g = lane >> 4;
    // the last tile's clamped rows (row >= M) form a run of their own (dst -2) that is not stored
    if (tile * TR + m >= a.M) di = -2;
    const int dprev = __builtin_amdgcn_update_dpp(-1, di, 0x111, 0xF, 0xF, false);  // row_shr:1 (m = 0 keeps -1)
    // run starts of row 0 (the other rows are the same rows); wave-uniform
    uint32_t starts = (uint32_t)__builtin_amdgcn_ballot_w64(m == 0 || dprev != di) & 0xFFFFu;
    const int nb0 = __builtin_amdgcn_readlane(nb, 0), nb15 = __builtin_amdgcn_readlane(nb, 15);
    const bool live = tile * TR < a.M;
    auto dst_of = [&](int d, bool first, bool last) -> float* {
        const bool sb = first && nb0 == d, ca = last && nb15 == d;
        return sb ? a.head + tile * H : ca ? a.tail + tile * H : a.full + (int64_t)d * H;
    };
    const bool st = m < 4 && live && !(MGN_EAGG_ABL & 1);
    if (starts == 1u) {  // one run (the common case at high in-degree)
        const int d = __builtin_amdgcn_readfirstlane(di);
        if (d < 0) return;
        float* dst = dst_of(d, true, true);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const f4 u = run_reduce_half<true>(v, h, m, 0, 15);
            if (st) *reinterpret_cast<f4*>(dst + 16 * (m + 4 * h) + 4 * g) = u;
        }
        return;
    }
    int r0 = 0;
    starts &= ~1u;
#pragma unroll 1
    while (true) {
        const int r1 = starts ? __builtin_ctz(starts) - 1 : 15;  // wave-uniform run [r0, r1]
        const int d = __builtin_amdgcn_readlane(di, r0);
        if (d >= 0) {  // (the padding run is not stored)
            float* dst = dst_of(d, r0 == 0, r1 == 15);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const f4 u = run_reduce_half<false>(v, h, m, r0, r1);
                if (st) *reinterpret_cast<f4*>(dst + 16 * (m + 4 * h) + 4 * g) = u;
            }
        }
        if (!starts) break;
        r0 = r1 + 1;
        starts &= starts - 1;
    }
}

// SAVE = false: inference (no autograd): only z and rden (the node MLP's aggregation inputs) are
// written — no R8 layer inputs, no ReLU masks (≈ 40 % of the training forward's HBM bytes).
// P is in the pair layout; ZP2: z too (the chained node MLP and the chained backward read it so;
// false: row-major, for a generic node MLP)
// SACT = false (with SAVE): ReLU masks, z, rden but no R8 layer inputs (their weight gradients recompute
// them: chain16_rew_kernel)
// EAGG (round 6, with SAVE): also the edge-side aggregation of the messages (edge_agg_store)
template <bool SAVE, int NWK, bool ZP2, bool SACT = true, bool EAGG = false>
__global__ __launch_bounds__(NWK * 64) void chain16_fwd_kernel(ChainFwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __bf16* W = reinterpret_cast<__bf16*>(smem);
    float* vec = reinterpret_cast<float*>(smem + LDS_W);  // bias[4][H], scale[H]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __bf16* scr = reinterpret_cast<__bf16*>(smem + LDS_W + LDS_VF) + wave * SROWS * SLD;
    const int m = lane & 15, g = lane >> 4;
    const int64_t stride = (int64_t)gridDim.x * NWK;
    int64_t tile = (int64_t)blockIdx.x * NWK + wave;
    const int64_t last = a.ntiles - 1;
    STAMP_DECL;
    WAVE_T0;
    In16 nxt;
    int di, dj, nb = -1;
    load_idx(a, min(tile, last), lane, di, dj);
    if (EAGG) nb = load_nb(a.proj_i, a.M, min(tile, last), lane);
    load_e(nxt, a, min(tile, last), lane);
    stage16<4, NWK * 64>(W, a.wpack, a.woff, a.wks, false);
    for (int i = threadIdx.x; i < 5 * H; i += NWK * 64) vec[i] = i < 4 * H ? a.bias[i / H][i % H] : a.scale[i - 4 * H];
    __syncthreads();
    if (tile >= a.ntiles) return;
#pragma unroll
    for (int s = 0; s < 4; ++s) pin(nxt.eb[s]);
    pin(di);
    pin(dj);
    if (EAGG) pin(nb);
    STAMP(0);
    for (; tile < a.ntiles; tile += stride) {
        const In16 in = nxt;
        // node projections of this tile (b0 folded into P_i); the layer-0 GEMM covers their latency
        u32x2 pi[8], pj[8];  // bf16 P_i[dst], P_j[src]: features 16t + 4g .. +3
        if (MGN_ABLATE & 2) {
#pragma unroll
            for (int t = 0; t < 8; ++t) pi[t] = pj[t] = u32x2{0u, 0u};
        } else {
            load_p2(pi, a.proj + (int64_t)((MGN_ABLATE & 1) ? 0 : di) * (2 * H), g);
            load_p2(pj, a.proj + (int64_t)((MGN_ABLATE & 1) ? 0 : dj) * (2 * H) + H, g);
        }
        int ndi, ndj, nnb = -1;
        load_idx(a, min(tile + stride, last), lane, ndi, ndj);
        if (EAGG) nnb = load_nb(a.proj_i, a.M, min(tile + stride, last), lane);
        load_e(nxt, a, min(tile + stride, last), lane);
        const int64_t row = tile * TR + m;
        f4 acc[8];
        bf16x8 B[4];
        STAMP(1);
#pragma unroll
        for (int l = 0; l < 3; ++l) {
            if (l == 0)
                gemm16(acc, W, 0, in.eb, lane);
            else if (SAVE && SACT)
                gemm16_st(acc, W, l, B, lane, scr, StoreDst{a.act8 + a.act_off[l], nullptr}, tile, a.M, vec + l * H);
            else
                gemm16(acc, W, l, B, lane, vec + l * H);
            STAMP(2);
            unsigned bits = 0u;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                // layer 0: + P_i[dst] + P_j[src] (b0 folded into P_i); layers 1, 2: the bias is in acc
                const f4 b = l == 0 ? bf4(pi[t]) + bf4(pj[t]) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float v = fmaxf(l == 0 ? acc[t][r] + b[r] : acc[t][r], 0.f);
                    acc[t][r] = v;
                    bits = push_bit(bits, v);
                }
            }
            to_operand(acc, B);
            if (SAVE) a.mask32[l * a.mask_stride * 2 + tile * 64 + lane] = bits;
            STAMP(3);
        }
        // layer 3 (stores its input, the R8 save of layer 3) + RMSNorm + residual
        if (SAVE && SACT)
            gemm16_st(acc, W, 3, B, lane, scr, StoreDst{a.act8 + a.act_off[3], nullptr}, tile, a.M, vec + 3 * H);
        else
            gemm16(acc, W, 3, B, lane, vec + 3 * H);
        STAMP(4);
        float ss = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) ss = fmaf(acc[t][r], acc[t][r], ss);  // z = acc (bias included)
        ss += __shfl_xor(ss, 16);
        ss += __shfl_xor(ss, 32);
        const float q = sqrtf(ss) * a.dinv + RMS_EPS;
        const float rq = __builtin_amdgcn_rcpf(q);  // bf16 outputs: z·(1/q) is within 2 fp32 ulp of z/q
        if (g == 0 && row < a.M) a.rden_save[row] = q;
        store_rows<ZP2>(acc, scr, a.z_save, tile, a.M, lane);
        STAMP(5);
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[t][r] *= rq;  // z / q: the output's term and (EAGG) the message
        if (EAGG)
            edge_agg_store([&](int t, int r) { return acc[t][r]; }, di, nb, tile, lane,
                           AggOut{a.agg_full, a.agg_head, a.agg_tail, a.M});
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const f4 s = *reinterpret_cast<const f4*>(vec + 4 * H + 16 * t + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; ++r)
                acc[t][r] = fmaf(s[r], acc[t][r], (float)in.eb[t >> 1][4 * (t & 1) + r]);
        }
        store_rows(acc, scr, a.out, tile, a.M, lane);
        STAMP(6);
#pragma unroll
        for (int s = 0; s < 4; ++s) pin(nxt.eb[s]);
        pin(ndi);
        pin(ndj);
        di = ndi;
        dj = ndj;
        if (EAGG) {
            pin(nnb);
            nb = nnb;
        }
        STAMP(7);
    }
    STAMP_PRINT("fwd16");
    WAVE_REC(0);
}

// ------------------------------------------------------------------------------------ backward
struct BIn16 {  // raw bf16: features 16t + 4g .. +3
    u32x2 d[8];     // de_out[row]
    u32x2 ga[8];    // d_aggr[dst(row)]
    u32x2 z[8];
    float q;
    unsigned mask[3];
};

// ZD: de_out is identically zero (the processor's last block: EncodeProcessDecode returns nodes only)
// PGA: prefetch the d_aggr gather with the rest (false: the tile loads it itself, 16 VGPRs fewer)
// a row in the accumulator layout: features 16t + 4g .. +3 (P2: stored in the pair layout)
template <bool P2>
__device__ __forceinline__ void load_acc_row(u32x2 (&o)[8], const __bf16* row, int g) {
    if (P2) {
        load_p2(o, row, g);
    } else {
#pragma unroll
        for (int t = 0; t < 8; ++t) o[t] = *reinterpret_cast<const u32x2*>(row + 16 * t + 4 * g);
    }
}

// P2: z and the d_aggr rows in the pair layout (written by the chained node MLP kernels);
// DIN2: de_out too (written by the next block's edge backward)
template <bool ZD, bool P2, bool DIN2, bool PGA = true>
__device__ __forceinline__ void bload(BIn16& in, const ChainBwdArgs& a, int64_t tile, int gi, int lane) {
    const int64_t row = clamp_row(tile * TR + (lane & 15), a.M);
    const int g = lane >> 4;
    if (ZD) {
#pragma unroll
        for (int t = 0; t < 8; ++t) in.d[t] = u32x2{0u, 0u};
    } else {
        load_acc_row<DIN2>(in.d, a.dout + row * H, g);
    }
    if (PGA) load_acc_row<P2>(in.ga, a.gath + (int64_t)gi * H, g);
    load_acc_row<P2>(in.z, a.z_save + row * H, g);
    in.q = a.rden_save[row];
#pragma unroll
    for (int l = 0; l < 3; ++l) in.mask[l] = a.mask32[l * a.mask_stride * 2 + tile * 64 + lane];
}

__device__ __forceinline__ int bidx(const ChainBwdArgs& a, int64_t tile, int lane) {
    return a.gath_idx[clamp_row(tile * TR + (lane & 15), a.M)];
}

template <bool PGA = true, class S>
__device__ __forceinline__ void pin_in(const S& in) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        pin(in.d[t]);
        if (PGA) pin(in.ga[t]);
        pin(in.z[t]);
    }
    pin(in.q);
#pragma unroll
    for (int l = 0; l < 3; ++l) pin(in.mask[l]);
}

// DOUT2: de in the pair layout (for the previous block's edge backward)
// EAGG (round 6): also the dst-direction segment sums of dZ0 (node_grad's dP_i) per tile run, as the
// forward's edge-side aggregation (edge_agg_store)
template <bool ZD, int NWK, bool P2, bool DIN2, bool DOUT2, bool EAGG = false>
__global__ __launch_bounds__(NWK * 64) void chain16_bwd_kernel(ChainBwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __bf16* W = reinterpret_cast<__bf16*>(smem);
    float* vec = reinterpret_cast<float*>(smem + LDS_W);  // scale[H]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __bf16* scr = reinterpret_cast<__bf16*>(smem + LDS_W + LDS_VB) + wave * SROWS * SLD;
    float* red = reinterpret_cast<float*>(smem + LDS_W + LDS_VB + (size_t)NWK * SROWS * SLD * 2);  // [NWK][H]
    const int m = lane & 15, g = lane >> 4;
    const int r4 = 2 * (m & 1) + ((m >> 1) & 1);  // row16_sum4's component in lane m
    const int64_t stride = (int64_t)gridDim.x * NWK;
    int64_t tile = (int64_t)blockIdx.x * NWK + wave;
    const int64_t last = a.ntiles - 1;
    STAMP_DECL;
    WAVE_T0;
    constexpr bool PGA = NWK < 12;  // three waves per SIMD: the gather is not prefetched (VGPR cap)
    const int gi0 = bidx(a, min(tile, last), lane);
    int gcur = gi0;
    int nb = EAGG ? load_nb(a.gath_idx, a.M, min(tile, last), lane) : -1;
    stage16<4, NWK * 64>(W, a.wtpack, a.woff, a.wks, true);
    BIn16 nxt;
    bload<ZD, P2, DIN2, PGA>(nxt, a, min(tile, last), gi0, lane);
    for (int i = threadIdx.x; i < H; i += NWK * 64) vec[i] = a.scale[i];
    __syncthreads();
    // RMSNorm-scale gradient partials of this wave: red[wave][H], one tile at a time (row sums
    // over the tile's 16 edges, then the 4 lane-group leaders add their features; fixed order)
    for (int i = lane; i < H; i += 64) red[wave * H + i] = 0.f;
    int ngi = 0;
    u32x2 gac[8];       // !PGA: d_aggr[dst] of the current tile
    bool gpre = false;  // gac already loaded (by the previous iteration)
    if (tile < a.ntiles) {
        ngi = bidx(a, min(tile + stride, last), lane);
        pin_in<PGA>(nxt);
        pin(ngi);
        if (EAGG) pin(nb);
    }
    STAMP(0);
    for (; tile < a.ntiles; tile += stride) {
        const int64_t row = tile * TR + m;
        const bool ok = row < a.M;
        // RMSNorm backward (layers.py:59-74) from the prefetched tile
        f4 acc[8];
        float dot = 0.f;
        if (!PGA && !gpre) {  // first tile: its gather now; later tiles': issued under the de stores
            if (P2) {
                load_p2(gac, a.gath + (int64_t)gcur * H, g);
            } else {
                const __bf16* gp = a.gath + (int64_t)gcur * H + 4 * g;
#pragma unroll
                for (int t = 0; t < 8; ++t) gac[t] = *reinterpret_cast<const u32x2*>(gp + 16 * t);
            }
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const f4 dy = bf4(nxt.d[t]) + bf4(PGA ? nxt.ga[t] : gac[t]);
            const f4 z = bf4(nxt.z[t]);
            const f4 sc = *reinterpret_cast<const f4*>(vec + 16 * t + 4 * g);
            acc[t] = dy;
#pragma unroll
            for (int r = 0; r < 4; ++r) dot = fmaf(sc[r] * dy[r], z[r], dot);
        }
        dot += __shfl_xor(dot, 16);
        dot += __shfl_xor(dot, 32);
        const float qd = nxt.q;
        const float rq = __builtin_amdgcn_rcpf(qd);
        const float rms = qd - RMS_EPS;
        const float coef = rms > 0.f ? dot / (qd * qd * rms) * (a.dinv * a.dinv) : 0.f;
        // rows past the end (last tile) are zeroed by a bit mask: a select on `ok` compiles to one
        // exec-masked branch per element (8x the VALU work of this phase)
        const int okm = ok ? -1 : 0;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const f4 z = bf4(nxt.z[t]);
            const f4 sc = *reinterpret_cast<const f4*>(vec + 16 * t + 4 * g);
            f4 ds;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float dy = acc[t][r];
                acc[t][r] = __int_as_float(__float_as_int(fmaf(-z[r], coef, sc[r] * dy * rq)) & okm);
                ds[r] = __int_as_float(__float_as_int(dy * z[r] * rq) & okm);
            }
            const float dsum = row16_sum4(ds, m);  // component r4(m) summed over the tile's 16 rows
            if (m < 4) atomicAdd(red + wave * H + 16 * t + 4 * g + r4, dsum);  // no-return LDS add
        }
        unsigned mcur[3];
#pragma unroll
        for (int l = 0; l < 3; ++l) mcur[l] = ok ? nxt.mask[l] : 0u;
        STAMP(1);
        bload<ZD, P2, DIN2, PGA>(nxt, a, min(tile + stride, last), ngi, lane);
        const int ngi2 = bidx(a, min(tile + 2 * stride, last), lane);
        const int nnb = EAGG ? load_nb(a.gath_idx, a.M, min(tile + stride, last), lane) : -1;
        bf16x8 B[4];
        to_operand(acc, B);
        STAMP(2);
        // layers 3..1: dZ_{l-1} = (dZ_l · W_l) ⊙ [A_l > 0]
        u32x2 dre[8];  // de_out of this tile again (cache-hot), for the layer-0 residual
#pragma unroll
        for (int l = 3; l >= 1; --l) {
            if (l == 1 && !ZD && !EAGG) load_acc_row<DIN2>(dre, a.dout + clamp_row(row, a.M) * H, g);
            // stores its B operand dZ_l (R8) under the MFMAs
            gemm16_st(acc, W, l, B, lane, scr, StoreDst{a.dz8 + (int64_t)l * a.RP * H, nullptr}, tile, a.M);
            STAMP(3);
            relu_mask(acc, mcur[l - 1]);
            to_operand(acc, B);
            if (EAGG && l == 1) {  // dZ0's bf16 operand (node_grad's terms; rows >= M are 0), acc free meanwhile
                edge_agg_store([&](int t, int r) { return (float)B[t >> 1][4 * (t & 1) + r]; }, gcur, nb, tile, lane,
                               AggOut{a.agg_full, a.agg_head, a.agg_tail, a.M});
                if (!ZD) load_acc_row<DIN2>(dre, a.dout + clamp_row(row, a.M) * H, g);  // after: fewer live registers
            }
            STAMP(4);
        }
        // layer 0, e block: de = de_out + dZ0 · W0a (stores dZ0 row-major under the MFMAs, every
        // padded row too: the weight-gradient ring reads it as its dZ operand, node_grad as rows)
        gemm16_st(acc, W, 0, B, lane, scr, StoreDst{nullptr, a.dz0}, tile, a.RP);
        STAMP(6);
#pragma unroll
        for (int t = 0; t < 8; ++t)
            if (!ZD) acc[t] += bf4(dre[t]);
        if constexpr (!PGA) {  // the next tile's gather, under this tile's de stores
            if (P2) {
                load_p2(gac, a.gath + (int64_t)ngi * H, g);
            } else {
                const __bf16* gp = a.gath + (int64_t)ngi * H + 4 * g;
#pragma unroll
                for (int t = 0; t < 8; ++t) gac[t] = *reinterpret_cast<const u32x2*>(gp + 16 * t);
            }
            gpre = true;
        }
        store_rows<DOUT2>(acc, scr, a.de, tile, a.M, lane);
        STAMP(7);
        pin_in<PGA>(nxt);
        pin(ngi2);
        gcur = ngi;
        ngi = ngi2;
        if (EAGG) {
            pin(nnb);
            nb = nnb;
        }
        STAMP(8);
    }
    STAMP_PRINT("bwd16");
    WAVE_REC(1);
    // dscale partials of the workgroup: the waves' rows in wave order
    __syncthreads();
    if (threadIdx.x < H) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < NWK; ++w) s += red[w * H + threadIdx.x];
        a.dscale_part[(int64_t)blockIdx.x * H + threadIdx.x] = s;
    }
}


// ------------------------------------------------------------------------------------ node MLP
// A-operand fragment (chain k order) read from a 16x16x32 pack in global memory (L2-resident):
// source tile `tile` (relative to the layer base); two 8-byte pieces per lane.
// Buffer loads: the lane part of the address is one 32-bit VGPR (gfrag_voff) and the tile part a
// scalar offset, so the compiler cannot hoist 64 per-fragment 64-bit addresses out of the tile
// loop (with global loads it did, and the node kernels spilled).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gfrag_rsrc(const __bf16* pack) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(pack), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ int gfrag_voff(int lane) {
    const int r = lane & 15, g = lane >> 4;
    return (r * 8 + 4 * (g & 1) + 16 * (g >> 1) * 8) * 2;  // bytes
}
template <int ABL = 32>
__device__ __forceinline__ bf16x8 gfrag(__amdgpu_buffer_rsrc_t rs, int voff, int tile) {
    const int so = (MGN_ABLATE & ABL) ? 0 : tile * 64 * 8 * 2;  // bytes (ablation: one L1-hot fragment)
    const u32x2 lo = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, so, 0));
    const u32x2 hi = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, so + 2 * 16 * 8 * 2, 0));
    const u32x4 w = {lo[0], lo[1], hi[0], hi[1]};
    return __builtin_bit_cast(bf16x8, w);
}

// acc += the 128-column K block of a packed weight matrix whose fragments are read from global
// memory (L2-resident), source tiles at tile_of(t, s); k-step s+1's fragments load while s computes
template <class TileFn>
__device__ __forceinline__ void gemm16_global(f4 (&acc)[8], const bf16x8 (&Ba)[4], const __bf16* pack, TileFn tile_of,
                                              int lane) {
    const __amdgpu_buffer_rsrc_t rs = gfrag_rsrc(pack);
    const int vo = gfrag_voff(lane);
    bf16x8 fr[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) fr[t] = gfrag(rs, vo, tile_of(t, 0));
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        bf16x8 nf[8];
        if (s + 1 < 4) {
#pragma unroll
            for (int t = 0; t < 8; ++t) nf[t] = gfrag(rs, vo, tile_of(t, s + 1));
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = mfma16(fr[t], Ba[s], acc[t]);
        if (s + 1 < 4) {
#pragma unroll
            for (int t = 0; t < 8; ++t) fr[t] = nf[t];
        }
    }
}

// node layer 0 = x block (LDS image, layer slot 0) + aggr block (global fragments)
template <class TileFn>
__device__ __forceinline__ void gemm16_layer0(f4 (&acc)[8], const __bf16* W, const bf16x8 (&Bx)[4],
                                              const bf16x8 (&Ba)[4], const __bf16* pack, TileFn tile_of, int lane,
                                              const float* bias = nullptr) {
    gemm16(acc, W, 0, Bx, lane, bias);
    gemm16_global(acc, Ba, pack, tile_of, lane);
}

// The next block's node projections P = [x·W0bᵀ + b0 ‖ x·W0cᵀ] of node tile `tile`, by a wave other
// than the one that computed x_out (chain16_node_fwd_kernel's hand-off): half 0's 32 weight fragments
// (k-steps 4..7 of the next edge MLP's layer-0 pack) are loaded BEFORE waiting for the tile, half
// 1's stream in under half 0's MFMAs. x_out's bf16 B operand (the bits the tile wave stores) comes
// through LDS: k-steps 0-1 from the tile wave's scratch, 2-3 from this wave's own (round 4: instead of
// re-reading the stored x_out rows from L2 after the tile wave waited for its stores to complete —
// node forward 27.0 -> see DESIGN.md).
__device__ __forceinline__ void node_proj_partner(const ChainNodeFwdArgs& a, int64_t tile, unsigned* flag,
                                                  const __bf16* tscr, __bf16* scr, int lane) {
    const int g = lane >> 4;
    const __amdgpu_buffer_rsrc_t rs = gfrag_rsrc(a.pn_pack);
    const int vo = gfrag_voff(lane), kst = a.pn_kst;
    bf16x8 fr[4][8];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < 8; ++t) fr[s][t] = gfrag<64>(rs, vo, t * kst + 4 + s);
    while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) __builtin_amdgcn_s_sleep(2);
    // B operand of x_out rows (as load_e): lane (m, g), k-step s: features 32s + 4g.. and 32s + 16 + 4g..
    const bf16x8* h0 = reinterpret_cast<const bf16x8*>(tscr);
    const bf16x8* h1 = reinterpret_cast<const bf16x8*>(scr);
    const bf16x8 Bx[4] = {h0[2 * lane], h0[2 * lane + 1], h1[2 * lane], h1[2 * lane + 1]};
    lds_fence();  // (own scratch reads back before store_rows reuses it)
    (void)g;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        f4 pacc[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) pacc[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
            for (int t = 0; t < 8; ++t) pacc[t] = mfma16(fr[s][t], Bx[s], pacc[t]);
            if (half == 0) {  // this k-step's registers now take half 1's fragments
#pragma unroll
                for (int t = 0; t < 8; ++t) fr[s][t] = gfrag<64>(rs, vo, t * kst + 8 + s);
            }
        }
        if (half == 0) {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const float* b = a.pn_b0 + 16 * t + 4 * g;  // 4-byte aligned only
                pacc[t] += f4{b[0], b[1], b[2], b[3]};
            }
        }
        store_rows<true>(pacc, scr, a.pn_out + half * H, tile, a.M, lane, 2 * H);
    }
}

// SAVE = false: inference — no aggregate, R8, mask, z or rden saves
// EAGG (round 6): the aggregate from the edge forward's per-tile partial rows of z/q (edge_agg_store)
// instead of every in-edge's z: s ⊙ (agg_full[v], or agg_tail[tb] + agg_head[tb + 1] + ... + agg_head[te]
// in tile order)
template <bool SAVE, bool EAGG = false>
__global__ __launch_bounds__(NW * 64) void chain16_node_fwd_kernel(ChainNodeFwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __bf16* W = reinterpret_cast<__bf16*>(smem);
    float* vec = reinterpret_cast<float*>(smem + LDS_W);  // bias[4][H], scale[H], edge scale[H]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __bf16* scr = reinterpret_cast<__bf16*>(smem + LDS_W + LDS_V) + wave * SROWS * SLD;
    const int m = lane & 15, g = lane >> 4;
    const int64_t stride = (int64_t)gridDim.x * NW;
    int64_t tile = (int64_t)wave * gridDim.x + blockIdx.x;
    // the first tile's segment bounds load under the weight staging (most waves own at most one
    // node tile: its chain of dependent loads is most of the kernel's time)
    // Phase A of a tile (memory-bound, no weights): x rows (layer-0 B operand of the x block, and
    // the residual) and the aggregation over the node's in-edges (target-sorted: one contiguous
    // segment), in the accumulator layout: the lane sums its 32 features of every message
    // s_e ⊙ z_k / q_k, in edge order. Groups of AG edges: every load of a group is issued before
    // the first add (one memory round trip per group; edges past the segment end reload its last
    // edge and add 0 · z). The edge RMSNorm scale s comes from the wave's scratch (a private copy,
    // so phase A needs nothing the workgroup stages).
    auto phase_a = [&](int64_t tl, bf16x8 (&xb)[4], f4 (&agg)[8]) {
        const int64_t row = tl * TR + m;
        const int64_t v = clamp_row(row, a.M);
        const int kb = a.seg_ptr[v];
        const int ke = row < a.M ? a.seg_ptr[v + 1] : kb;
        const __bf16* xp = a.x + v * H + 4 * g;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const u32x2 lo = *reinterpret_cast<const u32x2*>(xp + 32 * s);
            const u32x2 hi = *reinterpret_cast<const u32x2*>(xp + 32 * s + 16);
            const u32x4 w = {lo[0], lo[1], hi[0], hi[1]};
            xb[s] = __builtin_bit_cast(bf16x8, w);
        }
        if (EAGG) {
#pragma unroll
            for (int t = 0; t < 8; ++t) agg[t] = f4{0.f, 0.f, 0.f, 0.f};
            if (kb < ke) {
                const int tb = kb >> 4, te = (ke - 1) >> 4;
                const float* p0 = tb == te ? a.agg_full + v * H : a.agg_tail + (int64_t)tb * H;
#pragma unroll
                for (int t = 0; t < 8; ++t) agg[t] = *reinterpret_cast<const f4*>(p0 + 16 * t + 4 * g);
                // the head rows of the tiles after tb, two per round trip (the second clamped, added as 0)
#pragma unroll 1
                for (int T = tb + 1; T <= te; T += 2) {
                    const int T2 = T + 1 <= te ? T + 1 : T;
                    f4 h0[8], h1[8];
#pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        h0[t] = *reinterpret_cast<const f4*>(a.agg_head + (int64_t)T * H + 16 * t + 4 * g);
                        h1[t] = *reinterpret_cast<const f4*>(a.agg_head + (int64_t)T2 * H + 16 * t + 4 * g);
                    }
#pragma unroll
                    for (int t = 0; t < 8; ++t) agg[t] += h0[t];
                    if (T + 1 <= te) {
#pragma unroll
                        for (int t = 0; t < 8; ++t) agg[t] += h1[t];
                    }
                }
                // the edge RMSNorm scale s, factored out of the partial sums (Σ s ⊙ z/q = s ⊙ Σ z/q)
#pragma unroll
                for (int t = 0; t < 8; ++t) agg[t] *= *reinterpret_cast<const f4*>(a.agg_scale + 16 * t + 4 * g);
            }
            return;
        }
        float* scv = reinterpret_cast<float*>(scr);  // [H] edge scale, private to the wave
        scv[2 * lane] = a.agg_scale[2 * lane];
        scv[2 * lane + 1] = a.agg_scale[2 * lane + 1];
        lds_fence();
        constexpr int AG = MGN_NODE_AG;
#pragma unroll
        for (int t = 0; t < 8; ++t) agg[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
        for (int k = kb; k < ((MGN_ABLATE & 16) ? kb : ke); k += AG) {  // ablation 16: no aggregation
            u32x2 zz[AG][8];
            float rr[AG];
#pragma unroll
            for (int u = 0; u < AG; ++u) {
                const int ku = k + u < ke ? k + u : ke - 1;
                load_p2(zz[u], a.agg_z + (int64_t)ku * H, g);  // the edge forward's z: pair layout
                rr[u] = a.agg_rden[ku];
            }
#pragma unroll
            for (int u = 0; u < AG; ++u) {
                const float r = k + u < ke ? __builtin_amdgcn_rcpf(rr[u]) : 0.f;
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const f4 sc = *reinterpret_cast<const f4*>(scv + 16 * t + 4 * g);
                    agg[t] += sc * (bf4(zz[u][t]) * r);
                }
            }
        }
        lds_fence();  // scratch reads done before store_rows reuses it
    };
    auto fill_vec = [&](int tid, int nt) {
        for (int i = tid; i < 5 * H; i += nt) vec[i] = i < 4 * H ? a.bias[i / H][i % H] : a.scale[i - 4 * H];
    };
    // Most launches have at most one tile per wave of the first half (N/16 <= 4 x CUs): then the
    // second half of each workgroup stages the weights WHILE the first half runs its tile's phase A
    // (the staging burst hides behind the aggregation's gathers instead of preceding them).
    const bool split = a.ntiles <= (int64_t)gridDim.x * (NW / 2);
    // Projection hand-off (split launches with a chained next block): the NEXT block's node
    // projections of tile-wave w's tile are computed by its partner w + NW/2, which idles after the
    // staging otherwise. The partner loads its weight fragments (L2) while the tile wave runs phase A
    // and the MLP, then waits for the tile's x_out (an LDS word the tile wave sets once its x_out
    // stores have completed), reads those rows back (agent-scope loads: L2) and runs the 64 MFMAs —
    // the fragment stream leaves the tile's critical path. Same fragments, same k order: P is
    // bit-identical to the tile wave computing it.
    const bool handoff = MGN_PROJ_HANDOFF && split && a.pn_out != nullptr;
    unsigned* flags = reinterpret_cast<unsigned*>(smem + LDS_W + LDS_V + LDS_S);  // [NW/2] (the R region)
    bf16x8 xb[4];
    f4 agg[8];
    STAMP_DECL;
    WAVE_T0;
    if (split) {
        if (threadIdx.x < NW / 2) flags[threadIdx.x] = 0u;
        if (wave >= NW / 2) {
#ifdef MGN_STAMPS
            const unsigned long long s0 = __builtin_amdgcn_s_memtime();
#endif
            stage16<4, NW / 2 * 64>(W, a.wpack, a.woff, a.wks, false, threadIdx.x - NW / 2 * 64);
            fill_vec(threadIdx.x - NW / 2 * 64, NW / 2 * 64);
#ifdef MGN_STAMPS
            lds_fence();
            if (blockIdx.x == 0 && threadIdx.x == NW / 2 * 64)
                printf("nfwd16_stage %llu\n", __builtin_amdgcn_s_memtime() - s0);
#endif
        } else if (tile < a.ntiles) {
            phase_a(tile, xb, agg);
        }
    } else {
        stage16(W, a.wpack, a.woff, a.wks, false);
        fill_vec(threadIdx.x, NW * 64);
    }
    STAMP(4);  // wave 0: its phase A (split launches)
    __syncthreads();
    STAMP(0);
    if (handoff && wave >= NW / 2) {
        const int pw = wave - NW / 2;
        const int64_t pt = (int64_t)pw * gridDim.x + blockIdx.x;  // the partner's (only) tile
        if (pt < a.ntiles) node_proj_partner(a, pt, flags + pw, scr - (NW / 2) * SROWS * SLD, scr, lane);
        WAVE_REC(2);
        return;
    }
    for (const int64_t first = tile; tile < a.ntiles; tile += stride) {
        if (!split || tile != first) phase_a(tile, xb, agg);
        const int64_t row = tile * TR + m;
        const bool ok = row < a.M;
        STAMP(1);
        if (SAVE) store_rows(agg, scr, a.aggr_save, tile, a.M, lane);
        bf16x8 Ba[4];
        to_operand(agg, Ba);
        f4 acc[8];
        bf16x8 B[4];
#pragma unroll
        for (int l = 0; l < 3; ++l) {
            if (l == 0)
                gemm16_layer0(acc, W, xb, Ba, a.wpack + a.woff[0],
                              [](int t, int s) { return t * 8 + 4 + s; }, lane, vec);
            else if (SAVE)  // stores its input (the R8 save of layer l) under the MFMAs
                gemm16_st(acc, W, l, B, lane, scr, StoreDst{a.act8 + a.act_off[l], nullptr}, tile, a.M, vec + l * H);
            else
                gemm16(acc, W, l, B, lane, vec + l * H);
            unsigned bits = 0u;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float val = fmaxf(acc[t][r], 0.f);  // bias in the accumulator
                    acc[t][r] = val;
                    bits = push_bit(bits, val);
                }
            }
            to_operand(acc, B);
            if (SAVE) a.mask32[l * a.mask_stride * 2 + tile * 64 + lane] = bits;
        }
        if (SAVE)
            gemm16_st(acc, W, 3, B, lane, scr, StoreDst{a.act8 + a.act_off[3], nullptr}, tile, a.M, vec + 3 * H);
        else
            gemm16(acc, W, 3, B, lane, vec + 3 * H);
        STAMP(2);
        float ss = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) ss = fmaf(acc[t][r], acc[t][r], ss);  // z = acc (bias included)
        ss += __shfl_xor(ss, 16);
        ss += __shfl_xor(ss, 32);
        const float q = sqrtf(ss) * a.dinv + RMS_EPS;
        const float rq = __builtin_amdgcn_rcpf(q);
        if (SAVE) {
            if (g == 0 && ok) a.rden_save[row] = q;
            store_rows<true>(acc, scr, a.z_save, tile, a.M, lane);  // read back by the node backward only
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const f4 sc = *reinterpret_cast<const f4*>(vec + 4 * H + 16 * t + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; ++r)
                acc[t][r] = fmaf(sc[r], acc[t][r] * rq, (float)xb[t >> 1][4 * (t & 1) + r]);
        }
        store_rows(acc, scr, a.out, tile, a.M, lane);
        if (handoff) {
            // x_out's bf16 B operand to the partner through LDS: k-steps 0-1 in this wave's scratch
            // (free again after store_rows), 2-3 in the partner's (idle until it has read them)
            bf16x8 Bx[4];
            to_operand(acc, Bx);
            bf16x8* h0 = reinterpret_cast<bf16x8*>(scr);
            bf16x8* h1 = reinterpret_cast<bf16x8*>(scr + (NW / 2) * SROWS * SLD);
            h0[2 * lane] = Bx[0];
            h0[2 * lane + 1] = Bx[1];
            h1[2 * lane] = Bx[2];
            h1[2 * lane + 1] = Bx[3];
            lds_fence();
            if (lane == 0) __hip_atomic_store(flags + wave, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if (a.pn_out) {
            // the NEXT block's node projections from this tile's x_out (bf16, the bits just stored):
            // P = [x·W0bᵀ + b0 ‖ x·W0cᵀ] of the next edge MLP (its layer-0 k-steps 4..7 / 8..11,
            // fragments from L2) — what node_proj_kernel would compute in a launch of its own
            bf16x8 Bx[4];
            to_operand(acc, Bx);
#pragma unroll 1
            for (int half = 0; half < 2; ++half) {
                f4 pacc[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) pacc[t] = f4{0.f, 0.f, 0.f, 0.f};
                const int kst = a.pn_kst, k0 = 4 + 4 * half;
                gemm16_global(pacc, Bx, a.pn_pack, [kst, k0](int t, int s) { return t * kst + k0 + s; }, lane);
                if (half == 0) {
#pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        const float* b = a.pn_b0 + 16 * t + 4 * g;  // 4-byte aligned only
                        pacc[t] += f4{b[0], b[1], b[2], b[3]};
                    }
                }
                store_rows<true>(pacc, scr, a.pn_out + half * H, tile, a.M, lane, 2 * H);
            }
        }
        STAMP(3);
    }
    STAMP_PRINT("nfwd16");
    WAVE_REC(2);
}

// The wave's bf16 B operand (a 16-row tile, k-steps 0..3) as R8 octets 2*tile, 2*tile+1 of dst, through
// the wave's scratch (the store path of gemm16_st without its GEMM)
__device__ __forceinline__ void store_operand_r8(const bf16x8 (&B)[4], __bf16* scr, __bf16* dst, int64_t tile,
                                                 int lane) {
    const int m = lane & 15, g = lane >> 4;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        if ((m >> 3) == u) {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const u32x4 b = __builtin_bit_cast(u32x4, B[t >> 1]);
                const u32x2 w = (t & 1) ? u32x2{b[2], b[3]} : u32x2{b[0], b[1]};
                *reinterpret_cast<u32x2*>(scr + (m & 7) * SLD + 16 * t + 4 * g) = w;
            }
        }
        lds_fence();
        u32x2 rv[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) rv[q][0] = *reinterpret_cast<const unsigned*>(scr + q * SLD + 2 * lane);
        bf16x8 c0, c1;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const bf16x2 p = __builtin_bit_cast(bf16x2, rv[q][0]);
            c0[q] = p[0];
            c1[q] = p[1];
        }
        __bf16* p = dst + (((int64_t)tile * 2 + u) * H + 2 * lane) * 8;
        *reinterpret_cast<bf16x8*>(p) = c0;
        *reinterpret_cast<bf16x8*>(p + 8) = c1;
        lds_fence();
    }
}

// The aggregate half of node tile `tile`'s layer-0 backward, d_aggr = dZ0·W0aᵀ, and the dZ0 save, by the
// partner wave of the tile wave that ran layers 3..1 (chain16_node_bwd_kernel's hand-off; the tile wave
// keeps the LDS half, dx_part): the 32 weight fragments (global, L2) are loaded BEFORE waiting, so their
// round trips run under the tile wave's layers; then dZ0's operand comes from LDS (k-steps 0-1 from the
// tile wave's scratch, 2-3 from this wave's own). Same operations in the same order: bit-identical.
__device__ __forceinline__ void node_aggr_partner(const ChainNodeBwdArgs& a, int64_t tile, unsigned* flag,
                                                  const __bf16* tscr, __bf16* scr, int lane) {
    const __amdgpu_buffer_rsrc_t rs = gfrag_rsrc(a.wtpack + a.woff[0]);
    const int vo = gfrag_voff(lane);
    bf16x8 fr[4][8];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < 8; ++t) fr[s][t] = gfrag(rs, vo, (8 + t) * 4 + s);
    while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) __builtin_amdgcn_s_sleep(2);
    const bf16x8* h0 = reinterpret_cast<const bf16x8*>(tscr);
    const bf16x8* h1 = reinterpret_cast<const bf16x8*>(scr);
    const bf16x8 B[4] = {h0[2 * lane], h0[2 * lane + 1], h1[2 * lane], h1[2 * lane + 1]};
    lds_fence();  // (own scratch reads back before the stores below reuse it)
    f4 acc[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = mfma16(fr[s][t], B[s], acc[t]);
    store_rows<true>(acc, scr, a.d_aggr, tile, a.M, lane);  // gathered by the chained edge backward
    store_operand_r8(B, scr, a.dz8, tile, lane);            // dZ0 (R8): the weight-gradient ring's operand
}

// DIN2: dx_out in the pair layout (written by the next block's node_grad)
template <bool DIN2>
__global__ __launch_bounds__(NW * 64) void chain16_node_bwd_kernel(ChainNodeBwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __bf16* W = reinterpret_cast<__bf16*>(smem);
    float* vec = reinterpret_cast<float*>(smem + LDS_W);  // scale[H]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __bf16* scr = reinterpret_cast<__bf16*>(smem + LDS_W + LDS_V) + wave * SROWS * SLD;
    float* red = reinterpret_cast<float*>(smem + LDS_W + LDS_V + LDS_S);  // [NW][H]
    const int m = lane & 15, g = lane >> 4;
    const int r4 = 2 * (m & 1) + ((m >> 1) & 1);  // row16_sum4's component in lane m
    const int64_t stride = (int64_t)gridDim.x * NW;
    int64_t tile = (int64_t)wave * gridDim.x + blockIdx.x;
    for (int i = lane; i < H; i += 64) red[wave * H + i] = 0.f;  // the wave's own dscale row
    // Phase A of a tile (loads + RMSNorm backward, layers.py:59-74; no weights): dY = dx_out, the
    // scale from a private copy in the wave's scratch. Returns dZ of the last layer in acc, the
    // tile's dx_out rows (the residual) in d and the ReLU mask words in mk.
    auto phase_a = [&](int64_t tl, f4 (&acc)[8], u32x2 (&d)[8], unsigned (&mk)[3]) {
        const int64_t row = tl * TR + m;
        const bool ok = row < a.M;
        const int64_t v = clamp_row(row, a.M);
        u32x2 zr[8];
        load_acc_row<DIN2>(d, a.dout + v * H, g);
        load_p2(zr, a.z_save + v * H, g);  // the node forward's z: pair layout
        const float qd = a.rden_save[v];
#pragma unroll
        for (int l = 0; l < 3; ++l) mk[l] = ok ? a.mask32[l * a.mask_stride * 2 + tl * 64 + lane] : 0u;
        float* scv = reinterpret_cast<float*>(scr);  // [H] RMSNorm scale, private to the wave
        scv[2 * lane] = a.scale[2 * lane];
        scv[2 * lane + 1] = a.scale[2 * lane + 1];
        lds_fence();
        float dot = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const f4 dy = bf4(d[t]);
            const f4 z = bf4(zr[t]);
            const f4 sc = *reinterpret_cast<const f4*>(scv + 16 * t + 4 * g);
            acc[t] = dy;
#pragma unroll
            for (int r = 0; r < 4; ++r) dot = fmaf(sc[r] * dy[r], z[r], dot);
        }
        dot += __shfl_xor(dot, 16);
        dot += __shfl_xor(dot, 32);
        const float rq = __builtin_amdgcn_rcpf(qd);
        const float rms = qd - RMS_EPS;
        const float coef = rms > 0.f ? dot / (qd * qd * rms) * (a.dinv * a.dinv) : 0.f;
        const int okm = ok ? -1 : 0;  // bit mask, not a select (see chain16_bwd_kernel)
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const f4 z = bf4(zr[t]);
            const f4 sc = *reinterpret_cast<const f4*>(scv + 16 * t + 4 * g);
            f4 ds;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float dy = acc[t][r];
                acc[t][r] = __int_as_float(__float_as_int(fmaf(-z[r], coef, sc[r] * dy * rq)) & okm);
                ds[r] = __int_as_float(__float_as_int(dy * z[r] * rq) & okm);
            }
            const float dsum = row16_sum4(ds, m);  // component r4(m) summed over the tile's 16 rows
            if (m < 4) atomicAdd(red + wave * H + 16 * t + 4 * g + r4, dsum);  // no-return LDS add
        }
        lds_fence();  // scratch reads done before the GEMMs' stores reuse it
    };
    // as the node forward: with at most one tile per first-half wave, the second half stages the
    // weights while the first half runs phase A
    const bool split = a.ntiles <= (int64_t)gridDim.x * (NW / 2);
    // layer-0 hand-off (split launches): the partner w + NW/2 of tile wave w, idle after the staging,
    // runs the aggregate half of the tile's layer 0 (global weight fragments) and the dZ0 save once w
    // has put dZ0's operand in LDS (w's scratch and the partner's: no extra LDS); w keeps the LDS half
    const bool handoff = MGN_BWD_HANDOFF && split;
    unsigned* flags = reinterpret_cast<unsigned*>(vec + H);  // [NW/2], in the vector region's spare
    f4 acc[8];
    u32x2 d[8];
    unsigned mk[3];
    STAMP_DECL;
    WAVE_T0;
    if (split) {
        if (threadIdx.x < NW / 2) flags[threadIdx.x] = 0u;
        if (wave >= NW / 2)
            stage16<4, NW / 2 * 64>(W, a.wtpack, a.woff, a.wks, true, threadIdx.x - NW / 2 * 64);
        else if (tile < a.ntiles)
            phase_a(tile, acc, d, mk);
    } else {
        stage16(W, a.wtpack, a.woff, a.wks, true);
    }
    STAMP(7);  // wave 0: its phase A (split launches)
    __syncthreads();
    STAMP(0);
    if (handoff && wave >= NW / 2) {
        const int pw = wave - NW / 2;
        const int64_t pt = (int64_t)pw * gridDim.x + blockIdx.x;  // the partner's (only) tile
        if (pt < a.ntiles) node_aggr_partner(a, pt, flags + pw, scr - (NW / 2) * SROWS * SLD, scr, lane);
        tile = a.ntiles;  // no tile loop; the workgroup's dscale reduction below still needs this wave
    }
    for (const int64_t first = tile; tile < a.ntiles; tile += stride) {
        if (!split || tile != first) phase_a(tile, acc, d, mk);
        STAMP(1);
        bf16x8 B[4];
        to_operand(acc, B);
        // each GEMM stores its B operand dZ_l (R8) under its MFMAs
#pragma unroll
        for (int l = 3; l >= 1; --l) {
            gemm16_st(acc, W, l, B, lane, scr, StoreDst{a.dz8 + (int64_t)l * a.RP * H, nullptr}, tile, a.M);
            relu_mask(acc, mk[l - 1]);
            to_operand(acc, B);
        }
        STAMP(3);
        if (handoff) {  // dZ0's operand to the partner (k-steps 0-1: this scratch, 2-3: the partner's)
            bf16x8* h0 = reinterpret_cast<bf16x8*>(scr);
            bf16x8* h1 = reinterpret_cast<bf16x8*>(scr + (NW / 2) * SROWS * SLD);
            h0[2 * lane] = B[0];
            h0[2 * lane + 1] = B[1];
            h1[2 * lane] = B[2];
            h1[2 * lane + 1] = B[3];
            if (lane == 0) __hip_atomic_store(flags + wave, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            // the LDS half: dx_part = dx_out + dZ0·W0xᵀ, stored straight from the accumulator layout
            // (the scratch now belongs to the partner; the partner writes the dZ0 save)
            gemm16(acc, W, 0, B, lane);
            const int64_t row = tile * TR + m;
            if (row < a.M) {
                __bf16* p = a.dx_part + row * H;
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const f4 v = acc[t] + bf4(d[t]);
                    *reinterpret_cast<bf16x4*>(p + 16 * t + 4 * g) = bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2],
                                                                            (__bf16)v[3]};
                }
            }
            continue;  // (one tile per wave: the loop ends)
        }
        // layer 0: dx_part = dx_out + dZ0·W0x (LDS image), d_aggr = dZ0·W0a (global fragments)
        gemm16_st(acc, W, 0, B, lane, scr, StoreDst{a.dz8, nullptr}, tile, a.M);
        STAMP(4);
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] += bf4(d[t]);
        store_rows(acc, scr, a.dx_part, tile, a.M, lane);
        STAMP(5);
        {
            const __amdgpu_buffer_rsrc_t rs = gfrag_rsrc(a.wtpack + a.woff[0]);
            const int vo = gfrag_voff(lane);
#pragma unroll
            for (int t = 0; t < 8; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                bf16x8 fr[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) fr[t] = gfrag(rs, vo, (8 + t) * 4 + s);
#pragma unroll
                for (int t = 0; t < 8; ++t) acc[t] = mfma16(fr[t], B[s], acc[t]);
            }
        }
        STAMP(6);
        store_rows<true>(acc, scr, a.d_aggr, tile, a.M, lane);  // gathered by the chained edge backward
        STAMP(2);
    }
    STAMP_PRINT("nbwd16");
    WAVE_REC(3);
    __syncthreads();
    if (threadIdx.x < H) {
        float s2 = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) s2 += red[w * H + threadIdx.x];
        a.dscale_part[(int64_t)blockIdx.x * H + threadIdx.x] = s2;
    }
}

// ------------------------------------------------------------------------------------ dense MLP (encoders)
// build_mlp(in_dim ≤ 32, 128, 128, 4) + RMSNorm with no residual: the node and edge encoders
// (reference processors.py:72-82, applied at 127-128). Layer 0 is ONE 16x16x32 k-step per output
// tile (input columns zero-padded to 32; weights from the LDS image's slot 0, k-step 0); layers 1-3
// and the RMSNorm as in the block kernels. Saves follow the generic DENSE layout (R8 inputs of every
// layer incl. the padded layer-0 input, z, rden), so the generic weight-gradient kernel consumes
// them; the ReLU masks are the chained lane words (forward and backward are both chained whenever
// chain_dense_eligible(m), so the two always agree).
struct ChainDenseFwdArgs {
    const void* in;             // [*][in_ld] fp32 or bf16 MLP input
    const int32_t* in_rows;     // optional row gather
    int64_t in_ld;
    int32_t K0, in_f32, out_f32, pad;
    const __bf16* wpack;
    int64_t woff[4];
    int32_t wks[4];
    const float* bias[4];
    const float* scale;
    float dinv;
    int64_t M, ntiles;
    void* out;                  // [M][128] bf16 or fp32
    __bf16* z_save;
    float* rden_save;
    __bf16* act8;
    int64_t act_off[4];         // act_off(m, M, l, 0): layer 0 = R8 [RP][32]
    unsigned* mask32;
    int64_t mask_stride;        // 64-bit words per layer
};

struct ChainDenseBwdArgs {
    const void* dout;           // [M][128] bf16 or fp32 (template F32D)
    const __bf16* z_save;
    const float* rden_save;
    const float* scale;
    float dinv;
    const unsigned* mask32;
    int64_t mask_stride;
    const __bf16* wtpack;
    int64_t woff[4];
    int32_t wks[4];
    int64_t M, ntiles;
    __bf16* dz8;                // R8 [4][RP][128]: dZ of every layer
    int64_t RP;
    float* dscale_part;         // [grid][128]
    void* din;                  // optional [M][din_ld] gradient w.r.t. the (gathered) input rows
    int32_t din_f32, K0;
    int64_t din_ld;
};

// layer-0 B operand of a 16-row tile: lane (m, g) element j = input feature 16(j>>2) + 4g + (j&3)
// of row m (0 past K0 and past the last row)
__device__ __forceinline__ bf16x8 dense_in(const ChainDenseFwdArgs& a, int64_t tile, int lane) {
    const int64_t row = tile * TR + (lane & 15);
    const bool ok = row < a.M;
    const int64_t r = clamp_row(row, a.M);
    const int64_t src = a.in_rows ? (int64_t)a.in_rows[r] : r;
    const int g = lane >> 4;
    bf16x8 b;
    if (a.in_f32) {
        const float* p = reinterpret_cast<const float*>(a.in) + src * a.in_ld;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int f = 16 * (j >> 2) + 4 * g + (j & 3);
            b[j] = (__bf16)(ok && f < a.K0 ? p[f] : 0.f);
        }
    } else {
        const __bf16* p = reinterpret_cast<const __bf16*>(a.in) + src * a.in_ld;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int f = 16 * (j >> 2) + 4 * g + (j & 3);
            b[j] = ok && f < a.K0 ? p[f] : (__bf16)0.f;
        }
    }
    return b;
}

__global__ __launch_bounds__(NW * 64) void chain16_dense_fwd_kernel(ChainDenseFwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __bf16* W = reinterpret_cast<__bf16*>(smem);
    float* vec = reinterpret_cast<float*>(smem + LDS_W);  // bias[4][H], scale[H]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __bf16* scr = reinterpret_cast<__bf16*>(smem + LDS_W + LDS_V) + wave * SROWS * SLD;
    const int m = lane & 15, g = lane >> 4;
    const int64_t stride = (int64_t)gridDim.x * NW;
    int64_t tile = (int64_t)blockIdx.x * NW + wave;
    const int64_t last = a.ntiles - 1;
    bf16x8 nxt = dense_in(a, min(tile, last), lane);
    // layer 0's pack has one k-step per output tile: slot 0's k-steps 1..3 receive in-bounds bytes
    // of the rest of its region that no GEMM reads
    stage16(W, a.wpack, a.woff, a.wks, false);
    for (int i = threadIdx.x; i < 5 * H; i += NW * 64) vec[i] = i < 4 * H ? a.bias[i / H][i % H] : a.scale[i - 4 * H];
    __syncthreads();
    if (tile >= a.ntiles) return;
    pin(nxt);
    for (; tile < a.ntiles; tile += stride) {
        const bf16x8 in0 = nxt;
        nxt = dense_in(a, min(tile + stride, last), lane);
        const int64_t row = tile * TR + m;
        // padded layer-0 input as R8 [RP][32] (operand of W0's weight gradient): the tile's 16 x 32
        // block through the scratch, then lane (u, c) stores rows 8u..8u+7 of column c (16 bytes)
        {
            constexpr int LD0 = 40;
            const u32x4 w = __builtin_bit_cast(u32x4, in0);
            *reinterpret_cast<u32x2*>(scr + m * LD0 + 4 * g) = u32x2{w[0], w[1]};
            *reinterpret_cast<u32x2*>(scr + m * LD0 + 16 + 4 * g) = u32x2{w[2], w[3]};
            lds_fence();
            const int u = lane >> 5, c = lane & 31;
            bf16x8 o;
#pragma unroll
            for (int q = 0; q < 8; ++q) o[q] = scr[(8 * u + q) * LD0 + c];
            lds_fence();  // scratch free for the layer saves below
            *reinterpret_cast<bf16x8*>(a.act8 + a.act_off[0] + (((int64_t)tile * 2 + u) * 32 + c) * 8) = o;
        }
        f4 acc[8];
        bf16x8 B[4];
#pragma unroll
        for (int l = 0; l < 3; ++l) {
            if (l == 0) {
                acc_init(acc, vec, lane);
#pragma unroll
                for (int t = 0; t < 8; ++t) acc[t] = mfma16(wfrag(W, 0, t, 0, lane), in0, acc[t]);
            } else {
                gemm16_st(acc, W, l, B, lane, scr, StoreDst{a.act8 + a.act_off[l], nullptr}, tile, a.M, vec + l * H);
            }
            unsigned bits = 0u;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float v = fmaxf(acc[t][r], 0.f);  // bias in the accumulator
                    acc[t][r] = v;
                    bits = push_bit(bits, v);
                }
            }
            to_operand(acc, B);
            a.mask32[l * a.mask_stride * 2 + tile * 64 + lane] = bits;
        }
        gemm16_st(acc, W, 3, B, lane, scr, StoreDst{a.act8 + a.act_off[3], nullptr}, tile, a.M, vec + 3 * H);
        float ss = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) ss = fmaf(acc[t][r], acc[t][r], ss);  // z = acc (bias included)
        ss += __shfl_xor(ss, 16);
        ss += __shfl_xor(ss, 32);
        const float q = sqrtf(ss) * a.dinv + RMS_EPS;
        const float rq = __builtin_amdgcn_rcpf(q);
        if (g == 0 && row < a.M) a.rden_save[row] = q;
        store_rows(acc, scr, a.z_save, tile, a.M, lane);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const f4 s = *reinterpret_cast<const f4*>(vec + 4 * H + 16 * t + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[t][r] = s[r] * (acc[t][r] * rq);
        }
        if (a.out_f32) {
            if (row < a.M) {
                float* o = reinterpret_cast<float*>(a.out) + row * H + 4 * g;
#pragma unroll
                for (int t = 0; t < 8; ++t) *reinterpret_cast<f4*>(o + 16 * t) = acc[t];
            }
        } else {
            store_rows(acc, scr, reinterpret_cast<__bf16*>(a.out), tile, a.M, lane);
        }
        pin(nxt);
    }
}

template <bool F32D>
struct DIn16 {
    typename std::conditional<F32D, f4, u32x2>::type d[8];  // dout[row]: fp32, or raw bf16 pairs
    u32x2 z[8];
    float q;
    unsigned mask[3];
};

template <bool F32D>
__device__ __forceinline__ void dload(DIn16<F32D>& in, const ChainDenseBwdArgs& a, int64_t tile, int lane) {
    const int64_t row = clamp_row(tile * TR + (lane & 15), a.M);
    const int off = 4 * (lane >> 4);
    const __bf16* z = a.z_save + row * H + off;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        if constexpr (F32D)
            in.d[t] = *reinterpret_cast<const f4*>(reinterpret_cast<const float*>(a.dout) + row * H + off + 16 * t);
        else
            in.d[t] = *reinterpret_cast<const u32x2*>(reinterpret_cast<const __bf16*>(a.dout) + row * H + off + 16 * t);
        in.z[t] = *reinterpret_cast<const u32x2*>(z + 16 * t);
    }
    in.q = a.rden_save[row];
#pragma unroll
    for (int l = 0; l < 3; ++l) in.mask[l] = a.mask32[l * a.mask_stride * 2 + tile * 64 + lane];
}

template <bool F32D>
__device__ __forceinline__ void dpin(const DIn16<F32D>& in) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        pin(in.d[t]);
        pin(in.z[t]);
    }
    pin(in.q);
#pragma unroll
    for (int l = 0; l < 3; ++l) pin(in.mask[l]);
}

template <bool F32D>
__global__ __launch_bounds__(NW * 64) void chain16_dense_bwd_kernel(ChainDenseBwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __bf16* W = reinterpret_cast<__bf16*>(smem);
    float* vec = reinterpret_cast<float*>(smem + LDS_W);  // scale[H]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __bf16* scr = reinterpret_cast<__bf16*>(smem + LDS_W + LDS_V) + wave * SROWS * SLD;
    float* red = reinterpret_cast<float*>(smem + LDS_W + LDS_V + LDS_S);  // [NW][H]
    const int m = lane & 15, g = lane >> 4;
    const int r4 = 2 * (m & 1) + ((m >> 1) & 1);  // row16_sum4's component in lane m
    const int64_t stride = (int64_t)gridDim.x * NW;
    int64_t tile = (int64_t)blockIdx.x * NW + wave;
    const int64_t last = a.ntiles - 1;
    stage16(W, a.wtpack, a.woff, a.wks, true);
    DIn16<F32D> nxt;
    dload<F32D>(nxt, a, min(tile, last), lane);
    for (int i = threadIdx.x; i < H; i += NW * 64) vec[i] = a.scale[i];
    for (int i = lane; i < H; i += 64) red[wave * H + i] = 0.f;
    __syncthreads();
    if (tile < a.ntiles) dpin<F32D>(nxt);
    for (; tile < a.ntiles; tile += stride) {
        const int64_t row = tile * TR + m;
        const bool ok = row < a.M;
        // RMSNorm backward (layers.py:59-74), as chain16_bwd_kernel without the aggregate term
        f4 acc[8];
        float dot = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            f4 dy;
            if constexpr (F32D)
                dy = nxt.d[t];
            else
                dy = bf4(nxt.d[t]);
            const f4 z = bf4(nxt.z[t]);
            const f4 sc = *reinterpret_cast<const f4*>(vec + 16 * t + 4 * g);
            acc[t] = dy;
#pragma unroll
            for (int r = 0; r < 4; ++r) dot = fmaf(sc[r] * dy[r], z[r], dot);
        }
        dot += __shfl_xor(dot, 16);
        dot += __shfl_xor(dot, 32);
        const float qd = nxt.q;
        const float rq = __builtin_amdgcn_rcpf(qd);
        const float rms = qd - RMS_EPS;
        const float coef = rms > 0.f ? dot / (qd * qd * rms) * (a.dinv * a.dinv) : 0.f;
        const int okm = ok ? -1 : 0;  // bit mask, not a select (see chain16_bwd_kernel)
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const f4 z = bf4(nxt.z[t]);
            const f4 sc = *reinterpret_cast<const f4*>(vec + 16 * t + 4 * g);
            f4 ds;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float dy = acc[t][r];
                acc[t][r] = __int_as_float(__float_as_int(fmaf(-z[r], coef, sc[r] * dy * rq)) & okm);
                ds[r] = __int_as_float(__float_as_int(dy * z[r] * rq) & okm);
            }
            const float dsum = row16_sum4(ds, m);  // component r4(m) summed over the tile's 16 rows
            if (m < 4) atomicAdd(red + wave * H + 16 * t + 4 * g + r4, dsum);  // no-return LDS add
        }
        unsigned mcur[3];
#pragma unroll
        for (int l = 0; l < 3; ++l) mcur[l] = ok ? nxt.mask[l] : 0u;
        dload<F32D>(nxt, a, min(tile + stride, last), lane);
        bf16x8 B[4];
        to_operand(acc, B);
        // layers 3..1: dZ_{l-1} = (dZ_l · W_l) ⊙ [A_{l-1} > 0]; each GEMM stores its B operand dZ_l (R8)
#pragma unroll
        for (int l = 3; l >= 1; --l) {
            gemm16_st(acc, W, l, B, lane, scr, StoreDst{a.dz8 + (int64_t)l * a.RP * H, nullptr}, tile, a.M);
            relu_mask(acc, mcur[l - 1]);
            to_operand(acc, B);
        }
        store_r8(acc, scr, a.dz8, tile, lane);  // dZ0: operand of W0's weight gradient
        if (a.din) {
            // dA0 = dZ0 · W0 (transposed image slot 0): output tiles 0-1 = input features 0..31
            f4 d2[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int t = 0; t < 2; ++t) d2[t] = mfma16(wfrag(W, 0, t, s, lane), B[s], d2[t]);
            if (ok) {
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int k = 16 * t + 4 * g + r;
                        if (k < a.K0) {
                            if (a.din_f32)
                                reinterpret_cast<float*>(a.din)[row * a.din_ld + k] = d2[t][r];
                            else
                                reinterpret_cast<__bf16*>(a.din)[row * a.din_ld + k] = (__bf16)d2[t][r];
                        }
                    }
            }
        }
        dpin<F32D>(nxt);
    }
    // dscale partials of the workgroup: the waves' rows in wave order
    __syncthreads();
    if (threadIdx.x < H) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) s += red[w * H + threadIdx.x];
        a.dscale_part[(int64_t)blockIdx.x * H + threadIdx.x] = s;
    }
}

}  // namespace

// EdgeAgg scratch carve: full [N][128], head / tail [rows_pad(E)/16][128] (fp32, 256-byte aligned parts)
static size_t agg_al(size_t x) { return (x + 255) & ~(size_t)255; }
size_t chain16_edge_agg_bytes(int64_t N, int64_t E) {
    const int64_t nt = rows_pad(E) / TR;
    return agg_al((size_t)N * H * 4) + 2 * agg_al((size_t)nt * H * 4);
}
static void agg_carve(void* scratch, int64_t N, int64_t E, float** full, float** head, float** tail) {
    char* p = reinterpret_cast<char*>(scratch);
    *full = reinterpret_cast<float*>(p);
    p += agg_al((size_t)N * H * 4);
    *head = reinterpret_cast<float*>(p);
    p += agg_al((size_t)(rows_pad(E) / TR) * H * 4);
    *tail = reinterpret_cast<float*>(p);
}

void chain16_edge_agg_parts(void* scratch, int64_t N, int64_t E, float** full, float** head, float** tail) {
    agg_carve(scratch, N, E, full, head, tail);
}

int chain16_edge_forward(const mgn_mlp* m, const void* e, const void* proj, const int32_t* pi, const int32_t* pj,
                         int64_t M, void* out, mgn_mlp_saved* sv, hipStream_t st, bool z_p2, bool save_act, int64_t N,
                         void* agg_scratch) {
    ChainFwdArgs a;
    memset(&a, 0, sizeof(a));
    const bool eagg = agg_scratch != nullptr;
    if (eagg) agg_carve(agg_scratch, N, M, &a.agg_full, &a.agg_head, &a.agg_tail);
    a.e = reinterpret_cast<const __bf16*>(e);
    a.proj = reinterpret_cast<const __bf16*>(proj);
    a.proj_i = pi;
    a.proj_j = pj;
    a.wpack = reinterpret_cast<const __bf16*>(m->wpack);
    layer_offsets(m, a.woff, a.wks);
    for (int l = 0; l < 4; ++l) a.bias[l] = m->bias[l];
    a.scale = m->scale;
    a.dinv = norm_dinv(m);
    a.M = M;
    a.ntiles = rows_pad(M) / TR;  // every padded row: R8 saves and masks cover rows_pad(M)
    a.out = reinterpret_cast<__bf16*>(out);
    a.z_save = reinterpret_cast<__bf16*>(sv->z);
    a.rden_save = sv->rden;
    a.act8 = reinterpret_cast<__bf16*>(sv->act);
    for (int l = 0; l < 4; ++l) a.act_off[l] = act_off(*m, M, l, 1);
    a.mask32 = reinterpret_cast<unsigned*>(sv->mask);
    a.mask_stride = mask_words_per_layer(*m, M);
    if (a.ntiles == 0) return 0;
    const int nwk = edge_waves();
    // inference (no saves) always feeds the chained node MLP: z in the pair layout
    MGN_REQUIRE(sv->act || z_p2, "chained inference edge forward: z must be in the pair layout");
    MGN_REQUIRE(save_act || (sv->act && z_p2), "edge forward without R8 saves: the chained block path only");
    MGN_REQUIRE(!eagg || (sv->act && z_p2 && nwk == 12), "edge-side aggregation: the chained training forward only");
    const auto kern = eagg ? (save_act ? chain16_fwd_kernel<true, 12, true, true, true>
                                       : chain16_fwd_kernel<true, 12, true, false, true>)
                    : nwk == 12 ? (!sv->act   ? chain16_fwd_kernel<false, 12, true>
                                   : !save_act ? chain16_fwd_kernel<true, 12, true, false>
                                   : z_p2      ? chain16_fwd_kernel<true, 12, true>
                                               : chain16_fwd_kernel<true, 12, false>)
                                : (!sv->act   ? chain16_fwd_kernel<false, 8, true>
                                   : !save_act ? chain16_fwd_kernel<true, 8, true, false>
                                   : z_p2      ? chain16_fwd_kernel<true, 8, true>
                                               : chain16_fwd_kernel<true, 8, false>);
    const size_t lds = lds_fwd(nwk);
    if (int e2 = set_lds_once((const void*)kern, lds)) return e2;
    ProfScope ps(PROF_FWD_EDGE, st);
    hipLaunchKernelGGL(kern, dim3(chain16_grid(a.ntiles, nwk)), dim3(nwk * 64), lds, st, a);
    MGN_LAUNCH_CHECK();
    return 0;
}

int chain16_edge_backward(const mgn_mlp* m, int64_t M, const mgn_mlp_saved* sv, const void* dout, const void* gath,
                          const int32_t* gath_idx, void* dz8, float* dscale_part, int* nparts, void* de, void* dz0,
                          hipStream_t st, bool p2, bool din2, bool dout2, int64_t N, void* agg_scratch) {
    ChainBwdArgs a;
    memset(&a, 0, sizeof(a));
    const bool eagg = agg_scratch != nullptr;
    if (eagg) agg_carve(agg_scratch, N, M, &a.agg_full, &a.agg_head, &a.agg_tail);
    a.dout = reinterpret_cast<const __bf16*>(dout);
    a.gath = reinterpret_cast<const __bf16*>(gath);
    a.gath_idx = gath_idx;
    a.z_save = reinterpret_cast<const __bf16*>(sv->z);
    a.rden_save = sv->rden;
    a.scale = m->scale;
    a.dinv = norm_dinv(m);
    a.mask32 = reinterpret_cast<const unsigned*>(sv->mask);
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
    *nparts = 0;
    if (a.ntiles == 0) return 0;
    constexpr int nwk = edge_bwd_waves();
    MGN_REQUIRE(p2 || (!din2 && !dout2), "pair-layout de needs the chained node MLP");
    using K = void (*)(ChainBwdArgs);
    MGN_REQUIRE(!eagg || p2, "backward edge-side aggregation: the chained node MLP only");
    const K kern = eagg ? (!dout ? (dout2 ? (K)chain16_bwd_kernel<true, nwk, true, false, true, true>
                                          : (K)chain16_bwd_kernel<true, nwk, true, false, false, true>)
                           : din2 ? (dout2 ? (K)chain16_bwd_kernel<false, nwk, true, true, true, true>
                                           : (K)chain16_bwd_kernel<false, nwk, true, true, false, true>)
                                  : (dout2 ? (K)chain16_bwd_kernel<false, nwk, true, false, true, true>
                                           : (K)chain16_bwd_kernel<false, nwk, true, false, false, true>))
                   : !p2    ? (dout ? (K)chain16_bwd_kernel<false, nwk, false, false, false>
                                  : (K)chain16_bwd_kernel<true, nwk, false, false, false>)
                   : !dout ? (dout2 ? (K)chain16_bwd_kernel<true, nwk, true, false, true>
                                    : (K)chain16_bwd_kernel<true, nwk, true, false, false>)
                   : din2  ? (dout2 ? (K)chain16_bwd_kernel<false, nwk, true, true, true>
                                    : (K)chain16_bwd_kernel<false, nwk, true, true, false>)
                           : (dout2 ? (K)chain16_bwd_kernel<false, nwk, true, false, true>
                                    : (K)chain16_bwd_kernel<false, nwk, true, false, false>);
    const size_t lds = lds_bwd(nwk);
    if (int e2 = set_lds_once((const void*)kern, lds)) return e2;
    const int grid = chain16_edge_backward_parts(M);
    *nparts = grid;
    ProfScope ps(PROF_BWD_EDGE, st);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(nwk * 64), lds, st, a);
    MGN_LAUNCH_CHECK();
    return 0;
}

// node tiles are few (N/16): NODE_SPREAD 1 = one workgroup per CU, tiles spread wave-major over all
// of them; 0 = ceil(tiles / waves) workgroups, leaving the other CUs to a concurrent launch
#ifndef MGN_NODE_SPREAD
#define MGN_NODE_SPREAD 1  // measured: compact (0) fwd 27 -> 37.5 us, bwd 20 -> 23 us at Cfg B
#endif
static int node_grid(int64_t ntiles) {
    int cus = chain16_grid((int64_t)1 << 30);
    const int64_t want = MGN_NODE_SPREAD ? ntiles : cdiv64(ntiles, NW);
    return (int)(want < cus ? want : cus);
}

// dscale partial rows the backward launches write (= their grids): the weight-gradient half of a
// block backward (mgn_block_backward_wgrad) recomputes them from the sizes
int chain16_edge_backward_parts(int64_t M) { return M > 0 ? chain16_grid(rows_pad(M) / TR, edge_bwd_waves()) : 0; }
int chain16_node_backward_parts(int64_t M) { return M > 0 ? node_grid(rows_pad(M) / TR) : 0; }

bool chain_node_eligible(const mgn_mlp* m) {
    return m->dtype == MGN_BF16 && m->hidden == H && m->in_dim == 2 * H && m->out_dim == H && m->n_layers == 4 &&
           m->has_norm;
}

int chain16_node_forward(const mgn_mlp* m, const void* x, const mgn_topology* t, const mgn_mlp* edge,
                         const mgn_mlp_saved* edge_sv, int64_t M, void* x_out, void* aggr_save, mgn_mlp_saved* sv,
                         hipStream_t st, const mgn_mlp* next_edge, void* next_proj, void* agg_scratch) {
    ChainNodeFwdArgs a;
    memset(&a, 0, sizeof(a));
    if (agg_scratch) {
        float *full, *head, *tail;
        agg_carve(agg_scratch, t->num_nodes, t->num_edges, &full, &head, &tail);
        a.agg_full = full;
        a.agg_head = head;
        a.agg_tail = tail;
    }
    if (next_edge && next_proj) {
        a.pn_pack = reinterpret_cast<const __bf16*>(next_edge->wpack);  // layer 0 is the first pack
        a.pn_b0 = next_edge->bias[0];
        a.pn_out = reinterpret_cast<__bf16*>(next_proj);
        a.pn_kst = cdiv(next_edge->in_dim, 32);
    }
    a.x = reinterpret_cast<const __bf16*>(x);
    a.seg_ptr = t->col_ptr;
    a.agg_z = reinterpret_cast<const __bf16*>(edge_sv->z);
    a.agg_rden = edge_sv->rden;
    a.agg_scale = edge->scale;
    a.wpack = reinterpret_cast<const __bf16*>(m->wpack);
    layer_offsets(m, a.woff, a.wks);
    for (int l = 0; l < 4; ++l) a.bias[l] = m->bias[l];
    a.scale = m->scale;
    a.dinv = norm_dinv(m);
    a.M = M;
    a.ntiles = rows_pad(M) / TR;
    a.out = reinterpret_cast<__bf16*>(x_out);
    a.aggr_save = reinterpret_cast<__bf16*>(aggr_save);
    a.z_save = reinterpret_cast<__bf16*>(sv->z);
    a.rden_save = sv->rden;
    a.act8 = reinterpret_cast<__bf16*>(sv->act);
    for (int l = 0; l < 4; ++l) a.act_off[l] = act_off(*m, M, l, 1);
    a.mask32 = reinterpret_cast<unsigned*>(sv->mask);
    a.mask_stride = mask_words_per_layer(*m, M);
    if (M == 0) return 0;
    MGN_REQUIRE(!agg_scratch || sv->act, "edge-side aggregation: the chained training forward only");
    const auto kern = agg_scratch ? chain16_node_fwd_kernel<true, true>
                                  : sv->act ? chain16_node_fwd_kernel<true> : chain16_node_fwd_kernel<false>;
    if (int e2 = set_lds_once((const void*)kern, LDS_TOTAL)) return e2;
    ProfScope ps(PROF_FWD_NODE, st);
    hipLaunchKernelGGL(kern, dim3(node_grid(a.ntiles)), dim3(NW * 64), LDS_TOTAL, st, a);
    MGN_LAUNCH_CHECK();
    return 0;
}

int chain16_node_backward(const mgn_mlp* m, int64_t M, const mgn_mlp_saved* sv, const void* dout, void* dz8,
                          float* dscale_part, int* nparts, void* dx_part, void* d_aggr, hipStream_t st, bool din2) {
    ChainNodeBwdArgs a;
    memset(&a, 0, sizeof(a));
    a.dout = reinterpret_cast<const __bf16*>(dout);
    a.z_save = reinterpret_cast<const __bf16*>(sv->z);
    a.rden_save = sv->rden;
    a.scale = m->scale;
    a.dinv = norm_dinv(m);
    a.mask32 = reinterpret_cast<const unsigned*>(sv->mask);
    a.mask_stride = mask_words_per_layer(*m, M);
    a.wtpack = reinterpret_cast<const __bf16*>(m->wtpack);
    layer_offsets(m, a.woff, a.wks);
    a.M = M;
    a.ntiles = rows_pad(M) / TR;
    a.dz8 = reinterpret_cast<__bf16*>(dz8);
    a.RP = rows_pad(M);
    a.dscale_part = dscale_part;
    a.dx_part = reinterpret_cast<__bf16*>(dx_part);
    a.d_aggr = reinterpret_cast<__bf16*>(d_aggr);
    *nparts = 0;
    if (M == 0) return 0;
    const auto kern = din2 ? chain16_node_bwd_kernel<true> : chain16_node_bwd_kernel<false>;
    if (int e2 = set_lds_once((const void*)kern, LDS_TOTAL)) return e2;
    const int grid = chain16_node_backward_parts(M);
    *nparts = grid;
    ProfScope ps(PROF_BWD_NODE, st);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NW * 64), LDS_TOTAL, st, a);
    MGN_LAUNCH_CHECK();
    return 0;
}

// the encoders' shape on the chained kernels (compile-time -DMGN_CHAIN_DENSE=0: generic kernels, for
// A/B builds); forward and backward must agree on the ReLU-mask layout
#ifndef MGN_CHAIN_DENSE
#define MGN_CHAIN_DENSE 1
#endif
bool chain_dense_eligible(const mgn_mlp* m) {
    return MGN_CHAIN_DENSE && m->dtype == MGN_BF16 && m->hidden == H && m->out_dim == H && m->n_layers == 4 &&
           m->has_norm && m->in_dim >= 1 && m->in_dim <= 32;
}

// the GraphNetBlock edge MLP shape the chained edge kernels run: bf16, 3h -> h -> h -> h -> h + RMSNorm
bool chain_eligible(const mgn_mlp* m) {
    return m->dtype == MGN_BF16 && m->hidden == H && m->in_dim == 3 * H && m->out_dim == H && m->n_layers == 4 &&
           m->has_norm;
}

int chain16_dense_forward(const mgn_mlp* m, const void* in, int in_dtype, int64_t in_ld, const int32_t* in_rows,
                          int64_t M, void* out, int out_dtype, mgn_mlp_saved* sv, hipStream_t st) {
    ChainDenseFwdArgs a;
    memset(&a, 0, sizeof(a));
    a.in = in;
    a.in_rows = in_rows;
    a.in_ld = in_ld;
    a.K0 = m->in_dim;
    a.in_f32 = in_dtype == MGN_F32;
    a.out_f32 = out_dtype == MGN_F32;
    a.wpack = reinterpret_cast<const __bf16*>(m->wpack);
    layer_offsets(m, a.woff, a.wks);
    for (int l = 0; l < 4; ++l) a.bias[l] = m->bias[l];
    a.scale = m->scale;
    a.dinv = norm_dinv(m);
    a.M = M;
    a.ntiles = rows_pad(M) / TR;
    a.out = out;
    a.z_save = reinterpret_cast<__bf16*>(sv->z);
    a.rden_save = sv->rden;
    a.act8 = reinterpret_cast<__bf16*>(sv->act);
    for (int l = 0; l < 4; ++l) a.act_off[l] = act_off(*m, M, l, 0);
    a.mask32 = reinterpret_cast<unsigned*>(sv->mask);
    a.mask_stride = mask_words_per_layer(*m, M);
    if (a.ntiles == 0) return 0;
    if (int e2 = set_lds_once((const void*)chain16_dense_fwd_kernel, LDS_TOTAL)) return e2;
    ProfScope ps(PROF_FWD_DENSE, st);
    hipLaunchKernelGGL(chain16_dense_fwd_kernel, dim3(chain16_grid(a.ntiles)), dim3(NW * 64), LDS_TOTAL, st, a);
    MGN_LAUNCH_CHECK();
    return 0;
}

int chain16_dense_backward(const mgn_mlp* m, int64_t M, const mgn_mlp_saved* sv, const void* dout, int dout_dtype,
                           void* din, int din_dtype, int64_t din_ld, void* dz8, float* dscale_part, int* nparts,
                           hipStream_t st) {
    ChainDenseBwdArgs a;
    memset(&a, 0, sizeof(a));
    a.dout = dout;
    a.z_save = reinterpret_cast<const __bf16*>(sv->z);
    a.rden_save = sv->rden;
    a.scale = m->scale;
    a.dinv = norm_dinv(m);
    a.mask32 = reinterpret_cast<const unsigned*>(sv->mask);
    a.mask_stride = mask_words_per_layer(*m, M);
    a.wtpack = reinterpret_cast<const __bf16*>(m->wtpack);
    layer_offsets(m, a.woff, a.wks);
    a.M = M;
    a.ntiles = rows_pad(M) / TR;
    a.dz8 = reinterpret_cast<__bf16*>(dz8);
    a.RP = rows_pad(M);
    a.dscale_part = dscale_part;
    a.din = din;
    a.din_f32 = din_dtype == MGN_F32;
    a.K0 = m->in_dim;
    a.din_ld = din_ld;
    *nparts = 0;
    if (a.ntiles == 0) return 0;
    const auto kern = dout_dtype == MGN_F32 ? chain16_dense_bwd_kernel<true> : chain16_dense_bwd_kernel<false>;
    if (int e2 = set_lds_once((const void*)kern, LDS_TOTAL)) return e2;
    const int grid = chain16_grid(a.ntiles);
    *nparts = grid;
    ProfScope ps(PROF_BWD_DENSE, st);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NW * 64), LDS_TOTAL, st, a);
    MGN_LAUNCH_CHECK();
    return 0;
}

// Diagnostics (MGN_STAMPS builds only): per-wave [start, end] s_memrealtime ticks (100 MHz) of the last
// launch of a chained kernel kind (0 edge fwd, 1 edge bwd, 2 node fwd, 3 node bwd), n <= 4096 waves.
extern "C" int mgn_debug_wave_times(int32_t kind, uint64_t* out, int32_t n) {
#ifdef MGN_STAMPS
    if (kind < 0 || kind > 3 || n < 0 || n > 4096) return 1000;
    (void)hipDeviceSynchronize();
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_t), (size_t)n * 16, (size_t)kind * 4096 * 16,
                                    hipMemcpyDeviceToHost);
#else
    (void)kind;
    (void)out;
    (void)n;
    return 1000;
#endif
}
