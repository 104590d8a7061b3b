#include <vector>
#include <cstddef>
// Fused MLP kernels for the MeshGraphNet processor (gfx950).
//
// One workgroup (256 threads = 4 waves) owns a tile of BM rows (edges or nodes) and runs the
// WHOLE build_mlp chain on it (reference graphphysics/models/layers.py:77-113):
//   prologue  : stage the layer-0 input rows in LDS. EDGE mode gathers [e ‖ x[dst] ‖ x[src]]
//               (layers.py:689-690,717 — the `cat` is never materialised in HBM); NODE mode
//               builds [x ‖ Σ_in-edges m] with the segment sum over target-sorted edges
//               (PyG propagate aggr="add", layers.py:694-696,744).
//   layers    : MFMA GEMMs (16x16x32 bf16 or 16x16x4 f32), weights read as pre-packed
//               1-KiB-per-wave fragments from L2, activations ping-pong in LDS, bias+ReLU
//               epilogue in registers.
//   epilogue  : RMSNorm (layers.py:59-74) with a cross-wave row reduction, residual add
//               (layers.py:698-699), saved activations for the backward.
// Backward = data-gradient chain per tile (same structure, transposed weight fragments) +
// weight-gradient GEMMs over row chunks (K = rows) with a fixed-order partial-slab reduction.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>

#include "mgn_chain.h"
#include "mgn_common.h"

namespace {

enum { MODE_DENSE = 0, MODE_EDGE = 1, MODE_NODE = 2 };

#ifdef MGN_STAMPS  // diagnostics builds: per-phase s_memtime deltas of wave 0 of workgroup 0 (as mgn_chain16.hip)
#define F32C_STAMP_DECL unsigned long long st_prev = __builtin_amdgcn_s_memtime(), st_ph[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}
#define F32C_STAMP(i)                                                                     \
    do {                                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                \
        unsigned long long st_t;                                                          \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_t)::"memory");     \
        __builtin_amdgcn_sched_barrier(0);                                                \
        st_ph[i] += st_t - st_prev;                                                       \
        st_prev = st_t;                                                                   \
    } while (0)
#define F32C_STAMP_PRINT(name)                                                                                   \
    if (blockIdx.x == 0 && threadIdx.x == 0)                                                                     \
    printf("%s %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu\n", name, st_ph[0], st_ph[1], st_ph[2], \
           st_ph[3], st_ph[4], st_ph[5], st_ph[6], st_ph[7], st_ph[8], st_ph[9], st_ph[10], st_ph[11])
#else
#define F32C_STAMP_DECL
#define F32C_STAMP(i)
#define F32C_STAMP_PRINT(name)
#endif

template <int NT, int MT>
#ifndef MGN_F32_PD
#define MGN_F32_PD 8  // weight k-steps in flight in the generic fp32 GEMMs (A/B: 4 -> 86.8, 8 -> 90.0, 16 -> 88.5 steps/s)
#endif
#ifndef MGN_BF16_PD
#define MGN_BF16_PD 4  // the same for bf16 (one fragment = 4 VGPRs)
#endif

struct TileCfg {
    static constexpr int WN = NT < 4 ? NT : 4;
    static constexpr int NTW = NT / WN;
    static constexpr int WM = 4 / WN;
    static constexpr int MTW = (MT / WM) > 0 ? (MT / WM) : 1;
};

// One layer: acc[i][j] = D tile (n-tile nt0+i, row-tile mt0+j), A = packed fragments (global),
// B = LDS rows (row m, contiguous k).
template <class T, int NT, int MT>
struct Gemm {
    using C = TileCfg<NT, MT>;
    static constexpr int VEC = Mf<T>::VEC, KSTEP = Mf<T>::KSTEP;
    f4 acc[C::NTW][C::MTW];
    int nt0, mt0;
    bool active;

    // KS k-steps; fragment (n-tile t, k-step s) at wp + (t*kstride + s) fragments (kstride >= KS
    // lets a GEMM use a column block of a wider packed weight). accumulate: keep acc.
    __device__ __forceinline__ void run(const T* __restrict__ wp, int KS, const T* lds, int ldl, bool skip = false,
                                        int kstride = 0, bool accumulate = false) {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        const int wn = wave % C::WN, wm = wave / C::WN;
        nt0 = wn * C::NTW;
        mt0 = wm * C::MTW;
        active = mt0 < MT;
        if (!accumulate) {
#pragma unroll
            for (int i = 0; i < C::NTW; ++i)
#pragma unroll
                for (int j = 0; j < C::MTW; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
        }
        if (!active || skip) return;
        if (kstride <= 0) kstride = KS;
        const T* bp = lds + (size_t)(mt0 * 16 + (lane & 15)) * ldl + VEC * (lane >> 4);
        const T* ap = wp + ((size_t)nt0 * kstride * 64 + lane) * VEC;
        // weight fragments come from L2: keep PD k-steps of them in flight (register ring with
        // compile-time slots; the k loop is unrolled by PD so every ring index is static). An fp32
        // fragment is one VGPR (K = 4 per k-step), so fp32 keeps MGN_F32_PD k-steps in flight.
        constexpr int PD = sizeof(T) == 4 ? MGN_F32_PD : MGN_BF16_PD;
        typename Mf<T>::frag ring[PD][C::NTW];
#pragma unroll
        for (int u = 0; u < PD; ++u)
#pragma unroll
            for (int i = 0; i < C::NTW; ++i)
                if (u < KS) ring[u][i] = ld_frag(ap + ((size_t)i * kstride + u) * 64 * VEC);
        for (int k0 = 0; k0 < KS; k0 += PD) {
#pragma unroll
            for (int u = 0; u < PD; ++u) {
                const int ks = k0 + u;
                if (ks >= KS) break;
                typename Mf<T>::frag a[C::NTW], b[C::MTW];
#pragma unroll
                for (int i = 0; i < C::NTW; ++i) a[i] = ring[u][i];
                if (ks + PD < KS) {
#pragma unroll
                    for (int i = 0; i < C::NTW; ++i) ring[u][i] = ld_frag(ap + ((size_t)i * kstride + ks + PD) * 64 * VEC);
                }
#pragma unroll
                for (int j = 0; j < C::MTW; ++j) b[j] = ld_frag(bp + (size_t)j * 16 * ldl + ks * KSTEP);
#pragma unroll
                for (int i = 0; i < C::NTW; ++i)
#pragma unroll
                    for (int j = 0; j < C::MTW; ++j) acc[i][j] = Mf<T>::mma(a[i], b[j], acc[i][j]);
            }
        }
    }
    // The same GEMM with the weight fragments in LDS (WL kernels): groups of G k-steps whose A and B
    // fragments are all read before the group's MFMAs (one LDS round trip per group instead of one per
    // k-step: the runtime-KS loop above compiled to read -> wait -> MFMA per k-step, ~200 cycles each).
    // Same MFMA sequence per accumulator (k-steps ascending): bit-identical to run().
    __device__ __forceinline__ void run_lds(const T* wp, int KS, const T* lds, int ldl, int kstride = 0) {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        const int wn = wave % C::WN, wm = wave / C::WN;
        nt0 = wn * C::NTW;
        mt0 = wm * C::MTW;
        active = mt0 < MT;
#pragma unroll
        for (int i = 0; i < C::NTW; ++i)
#pragma unroll
            for (int j = 0; j < C::MTW; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
        if (!active) return;
        if (kstride <= 0) kstride = KS;
        const T* bp = lds + (size_t)(mt0 * 16 + (lane & 15)) * ldl + VEC * (lane >> 4);
        const T* ap = wp + ((size_t)nt0 * kstride * 64 + lane) * VEC;
        constexpr int G = sizeof(T) == 4 ? 8 : 4;
        for (int k0 = 0; k0 < KS; k0 += G) {
            typename Mf<T>::frag a[G][C::NTW], b[G][C::MTW];
#pragma unroll
            for (int u = 0; u < G; ++u) {
                const int ks = k0 + u < KS ? k0 + u : KS - 1;
#pragma unroll
                for (int i = 0; i < C::NTW; ++i) a[u][i] = ld_frag(ap + ((size_t)i * kstride + ks) * 64 * VEC);
#pragma unroll
                for (int j = 0; j < C::MTW; ++j) b[u][j] = ld_frag(bp + (size_t)j * 16 * ldl + ks * KSTEP);
            }
#pragma unroll
            for (int u = 0; u < G; ++u) {
                if (k0 + u >= KS) break;
#pragma unroll
                for (int i = 0; i < C::NTW; ++i)
#pragma unroll
                    for (int j = 0; j < C::MTW; ++j) acc[i][j] = Mf<T>::mma(a[u][i], b[u][j], acc[i][j]);
            }
        }
    }
    __device__ __forceinline__ int n_of(int i) const { return (nt0 + i) * 16 + ((threadIdx.x & 63) >> 4) * 4; }
    __device__ __forceinline__ int m_of(int j) const { return (mt0 + j) * 16 + (threadIdx.x & 15); }
};

// Weights in LDS (small MLPs, hidden <= 64): every layer's packed fragments the kernel reads (a
// contiguous prefix of the layer's pack) are copied into LDS by LDS-DMA at kernel start — one round
// trip that overlaps the input loads — instead of each layer's GEMM streaming them from L2 (which
// exposed one L2 round trip per 8 k-steps: measured, MGN_STAMPS, fp32 h=32 edge forward: 19.4k of
// 38k cycles in the GEMMs of layers 0-2). WlDesc: per layer, source element offset in the pack and
// element count; LDS copies are consecutive (layer l at wl_lo[l] elements).
#ifndef MGN_WL_BATCH
#define MGN_WL_BATCH 1  // A/B builds: 0 = the descriptor read field by field inside the layer loop
#endif
struct WlDesc {
    int32_t n;                      // layers staged (0: weights read from global memory)
    int32_t pad;
    int64_t src[MGN_MAX_LAYERS];    // element offset of the layer's prefix in the pack
    int32_t cnt[MGN_MAX_LAYERS];    // elements
    int32_t lo[MGN_MAX_LAYERS];     // element offset of its LDS copy
};

// issue the LDS-DMA copies (all waves; 16 bytes per lane, a wave instruction = 1 KiB); the caller
// waits vmcnt(0) and barriers before the first read
// The descriptor is copied whole (one batch of scalar loads) and the layer loop unrolled: a loop
// over d.n re-read d.cnt / d.src / d.lo from the kernel arguments layer by layer, one scalar-load
// round trip each before the layer's copies could issue (MGN_STAMPS: 4.3-5.6k cycles to issue the
// copies of a 4-layer MLP, ahead of every generic launch's first input load).
template <class T>
__device__ __forceinline__ void wl_issue(const WlDesc& d, const T* pack, T* lds) {
    const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int EPL = 16 / sizeof(T);  // elements per lane
#if MGN_WL_BATCH
    const WlDesc w = d;
#else
    const WlDesc& w = d;
#endif
#pragma unroll
    for (int l = 0; l < MGN_MAX_LAYERS; ++l) {
        if (l >= w.n) break;
        const int pieces = (w.cnt[l] + 64 * EPL - 1) / (64 * EPL);
        for (int pc = wave; pc < pieces; pc += nw) {
            const int e0 = pc * 64 * EPL;
            if (e0 + lane * EPL < w.cnt[l])
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(pack + w.src[l] + e0 + lane * EPL),
                    (__attribute__((address_space(3))) void*)(lds + w.lo[l] + e0), 16, 0, 0);
        }
    }
}

struct SrcSeg {
    const void* p;
    const int32_t* idx;
    int64_t ld;
    int32_t ncols, dtype, coff, pad;
};

template <class T>
constexpr int dtype_id() { return sizeof(T) == 4 ? MGN_F32 : MGN_BF16; }

// element (row, col) of a segment as float
__device__ __forceinline__ float seg_load(const SrcSeg& g, int64_t row, int col) {
    const int64_t r = g.idx ? (int64_t)g.idx[row] : row;
    return load_any(g.p, g.dtype, r * g.ld + col);
}

// Stage rows [row0, row0+BM) of the concatenated segments into LDS In[BM][ldi], zero padding
// rows >= M and columns [K0, KP).
template <class T, int BM>
__device__ void load_tile(T* In, int ldi, int K0, int KP, const SrcSeg* seg, int nseg,
                          int64_t row0, int64_t M) {
    constexpr int CH = 16 / sizeof(T);
    for (int s = 0; s < nseg; ++s) {
        const SrcSeg g = seg[s];
        const bool vec = g.dtype == dtype_id<T>() && g.ncols % CH == 0 && g.ld % CH == 0 &&
                         g.coff % CH == 0;
        if (vec) {
            const int cpr = g.ncols / CH;
            constexpr int B = 4;  // loads in flight per thread
            for (int base = threadIdx.x; base < BM * cpr; base += MGN_THREADS * B) {
                u32x4 v[B];
                int64_t sr[B];
#pragma unroll
                for (int q = 0; q < B; ++q) {
                    const int it = base + q * MGN_THREADS;
                    const int64_t row = row0 + it / cpr;
                    sr[q] = (it < BM * cpr && row < M) ? (g.idx ? (int64_t)g.idx[row] : row) : -1;
                }
#pragma unroll
                for (int q = 0; q < B; ++q) {
                    const int it = base + q * MGN_THREADS;
                    const int c = (it % cpr) * CH;
                    v[q] = u32x4{0u, 0u, 0u, 0u};
                    if (sr[q] >= 0) v[q] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const T*>(g.p) + sr[q] * g.ld + c);
                }
#pragma unroll
                for (int q = 0; q < B; ++q) {
                    const int it = base + q * MGN_THREADS;
                    if (it < BM * cpr) {
                        const int r = it / cpr, c = (it - r * cpr) * CH;
                        *reinterpret_cast<u32x4*>(In + (size_t)r * ldi + g.coff + c) = v[q];
                    }
                }
            }
        } else {
            for (int it = threadIdx.x; it < BM * g.ncols; it += MGN_THREADS) {
                const int r = it / g.ncols, c = it - r * g.ncols;
                const int64_t row = row0 + r;
                const float v = row < M ? seg_load(g, row, c) : 0.f;
                In[(size_t)r * ldi + g.coff + c] = from_f<T>(v);
            }
        }
    }
    const int padc = KP - K0;
    if (padc > 0)
        for (int it = threadIdx.x; it < BM * padc; it += MGN_THREADS) {
            const int r = it / padc, c = it - r * padc;
            In[(size_t)r * ldi + K0 + c] = from_f<T>(0.f);
        }
}

// Write an LDS tile (BM rows x cols, row-major, leading dim ldl) to an R8 matrix with `cols`
// columns, rows [row0, row0 + BM). One item = one (row octet, column) = 8 LDS reads, one 16/32-B store.
template <class T, int BM>
__device__ void copy_out_r8(const T* lds, int ldl, int cols, T* dst, int64_t row0) {
    constexpr int OCT = BM / 8;
    const int64_t o0 = row0 >> 3;
    if (sizeof(T) == 2 && (cols & 3) == 0 && (ldl & 3) == 0) {
        // item = (octet, 4 columns): 8 ds_read_b64 (one per row) -> 4 R8 chunks of 16 B
        const int c4 = cols >> 2;
        for (int it = threadIdx.x; it < OCT * c4; it += MGN_THREADS) {
            const int o = it / c4, c = (it - o * c4) * 4;
            bf16x4 rv[8];
#pragma unroll
            for (int q = 0; q < 8; ++q)
                rv[q] = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const __bf16*>(lds) + (size_t)(o * 8 + q) * ldl + c);
            __bf16* p = reinterpret_cast<__bf16*>(dst) + ((o0 + o) * cols + c) * 8;
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                bf16x8 w;
#pragma unroll
                for (int q = 0; q < 8; ++q) w[q] = rv[q][cc];
                *reinterpret_cast<bf16x8*>(p + cc * 8) = w;
            }
        }
        return;
    }
    for (int it = threadIdx.x; it < OCT * cols; it += MGN_THREADS) {
        const int o = it / cols, c = it - o * cols;
        float v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = to_f(lds[(size_t)(o * 8 + q) * ldl + c]);
        T* p = dst + ((o0 + o) * cols + c) * 8;
        if (sizeof(T) == 2) {
            Chunk<T>::store(p, v);
        } else {
            Chunk<T>::store(p, v);
            Chunk<T>::store(p + 4, v + 4);
        }
    }
}

// --------------------------------------------------------------------------- forward
struct FwdArgs {
    SrcSeg seg[3];
    int32_t nseg;
    int32_t L, K0, H, NOUT, has_norm, ldi, ldh;
    int32_t Kpack0, kstride0;  // layer-0 packed width (K0 < Kpack0: EDGE uses the e-column block)
    int64_t M;
    const void* wpack;
    // EDGE: node projections P [N][2H] fp32 (x·W0bᵀ ‖ x·W0cᵀ), added at rows proj_i/proj_j
    const float* proj;
    const int32_t* proj_i;
    const int32_t* proj_j;
    const float* bias[MGN_MAX_LAYERS];
    const float* scale;
    float dinv;
    // NODE mode aggregation of edge messages m_k = scale_e * (z_k / rden_k)
    const int32_t* seg_ptr;
    const void* agg_z;
    const float* agg_rden;
    const float* agg_scale;
    void* agg_save;
    // outputs
    void* out;
    int32_t out_dtype;
    int64_t out_ld;
    const void* resid;
    void* act8;                          // R8 saved layer inputs
    int64_t act_off[MGN_MAX_LAYERS];     // element offset of layer l's R8 block
    unsigned long long* mask;            // ReLU ballot words of hidden layers
    int64_t mask_stride;                 // words per hidden layer
    void* z_save;
    float* rden_save;
    int32_t ablate;  // diagnostics builds only (-DMGN_ABLATE=bits): 1 gather, 2 R8 saves, 4 MFMA, 8 epilogue stores
    int32_t r0_elems;  // LDS region 0 (layer-0 input / odd-layer activations / fp32 z staging), in T
    int32_t wl_elems;  // WL kernels: LDS element offset of the staged weights
    WlDesc wl;
    // chained fp32 node MLP: the NEXT block's node projections P = [x_out·W0bᵀ ‖ x_out·W0cᵀ] (fp32
    // [N][2H], what node_proj_kernel writes) from the next edge MLP's forward pack (nullptr: none)
    const float* pn_pack;
    float* pn_out;
};

// Diagnostic ablation mask for timing studies (results are wrong when nonzero): a compile-time
// define of diagnostics builds (MGN_ABLATE=bits python __graft_entry__.py), never a runtime switch.
#ifndef MGN_ABLATE
#define MGN_ABLATE 0
#endif
static int ablate_mask() { return MGN_ABLATE; }

// Last layer: bias, RMSNorm, residual. z is staged (fp32) in LDS `zf` ([BM][H+4], aliases the
// dead layer-0 input region), then one cooperative pass writes z, out = resid + scale*z/q and rden
// as coalesced 16-byte row chunks.
template <class T, int BM, class G>
__device__ __forceinline__ void fwd_last_epilogue(G& g, const FwdArgs& a, float* red, float* zf, int64_t row0) {
    using C = typename G::C;
    const int lane = threadIdx.x & 63;
    const int wn = (threadIdx.x >> 6) % C::WN;
    const float* b = a.bias[a.L - 1];
    if (a.has_norm) {
        const int H = a.H, ldz = a.H + 4;
        float ss[C::MTW];
#pragma unroll
        for (int j = 0; j < C::MTW; ++j) {
            ss[j] = 0.f;
#pragma unroll
            for (int i = 0; i < C::NTW; ++i) {
                const f4 bb = ld4u(b + g.n_of(i));
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float z = g.acc[i][j][r] + bb[r];
                    g.acc[i][j][r] = z;
                    ss[j] += z * z;
                }
            }
            ss[j] += __shfl_xor(ss[j], 16);
            ss[j] += __shfl_xor(ss[j], 32);
        }
        __syncthreads();  // every wave is done reading the GEMM input (zf may alias it)
        if (g.active) {
#pragma unroll
            for (int j = 0; j < C::MTW; ++j) {
                if (lane < 16) red[wn * BM + g.m_of(j)] = ss[j];
#pragma unroll
                for (int i = 0; i < C::NTW; ++i)
                    *reinterpret_cast<f4*>(zf + (size_t)g.m_of(j) * ldz + g.n_of(i)) = g.acc[i][j];
            }
        }
        __syncthreads();
        const int cpr = H / 8;
        for (int it = threadIdx.x; it < BM * cpr; it += MGN_THREADS) {
            const int r = it / cpr, c = (it - r * cpr) * 8;
            const int64_t row = row0 + r;
            if (row >= a.M) continue;
            float tot = 0.f;
#pragma unroll
            for (int w = 0; w < C::WN; ++w) tot += red[w * BM + r];
            const float q = sqrtf(tot) * a.dinv + RMS_EPS;
            if (c == 0) a.rden_save[row] = q;
            float z[8], y[8];
            const f4 z0 = *reinterpret_cast<const f4*>(zf + (size_t)r * ldz + c);
            const f4 z1 = *reinterpret_cast<const f4*>(zf + (size_t)r * ldz + c + 4);
            const f4 s0 = ld4u(a.scale + c), s1 = ld4u(a.scale + c + 4);
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                z[v] = z0[v];
                z[v + 4] = z1[v];
                y[v] = s0[v] * (z0[v] / q);
                y[v + 4] = s1[v] * (z1[v] / q);
            }
            if (a.resid) {
                float x[8];
                if constexpr (sizeof(T) == 2) {
                    Chunk<T>::load(reinterpret_cast<const T*>(a.resid) + row * H + c, x);
                } else {
                    Chunk<T>::load(reinterpret_cast<const T*>(a.resid) + row * H + c, x);
                    Chunk<T>::load(reinterpret_cast<const T*>(a.resid) + row * H + c + 4, x + 4);
                }
#pragma unroll
                for (int v = 0; v < 8; ++v) y[v] = x[v] + y[v];
            }
            T* zp = reinterpret_cast<T*>(a.z_save) + row * H + c;
            if constexpr (sizeof(T) == 2) {
                Chunk<T>::store(zp, z);
            } else {
                Chunk<T>::store(zp, z);
                Chunk<T>::store(zp + 4, z + 4);
            }
            if (a.out_dtype == MGN_BF16) {
                Chunk<__bf16>::store(reinterpret_cast<__bf16*>(a.out) + row * a.out_ld + c, y);
            } else {
                float* op = reinterpret_cast<float*>(a.out) + row * a.out_ld + c;
                Chunk<float>::store(op, y);
                Chunk<float>::store(op + 4, y + 4);
            }
        }
    } else {
        if (!g.active) return;
#pragma unroll
        for (int j = 0; j < C::MTW; ++j) {
            const int64_t row = row0 + g.m_of(j);
            if (row >= a.M) continue;
#pragma unroll
            for (int i = 0; i < C::NTW; ++i) {
                const int n = g.n_of(i);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (n + r >= a.NOUT) continue;
                    float y = g.acc[i][j][r] + b[n + r];
                    if (a.z_save) reinterpret_cast<T*>(a.z_save)[row * a.H + n + r] = from_f<T>(y);
                    if (a.rden_save && n + r == 0) a.rden_save[row] = 1.f;
                    if (a.resid) y = to_f(reinterpret_cast<const T*>(a.resid)[row * a.H + n + r]) + y;
                    if (a.out_dtype == MGN_F32)
                        reinterpret_cast<float*>(a.out)[row * a.out_ld + n + r] = y;
                    else
                        reinterpret_cast<__bf16*>(a.out)[row * a.out_ld + n + r] = (__bf16)y;
                }
            }
        }
    }
}

// in-edges per aggregation round trip of the generic node forward (A/B builds: 4 = groups of 4 and
// the remainder one edge at a time, the round-4 form's round-trip count is higher)
#ifndef MGN_GEN_AG
#define MGN_GEN_AG 8
#endif
template <class T, int H, int BM, int MODE, bool WL = false>
__global__ __launch_bounds__(MGN_THREADS) void mlp_fwd_kernel(FwdArgs a) {
    constexpr int KSTEP = Mf<T>::KSTEP;
    constexpr int NTH = H / 16, MT = BM / 16;
    constexpr int CH = 16 / sizeof(T);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int KP0 = rup(a.K0, KSTEP);
    T* In = reinterpret_cast<T*>(smem);
    T* P0 = In + a.r0_elems;
    T* P1 = In;  // In is dead after layer 0
    float* red = reinterpret_cast<float*>(P0 + BM * a.ldh);
    T* Wl = reinterpret_cast<T*>(smem) + a.wl_elems;  // WL: the staged weight prefixes
    const int64_t row0 = (int64_t)blockIdx.x * BM;

    F32C_STAMP_DECL;
    if (WL) wl_issue<T>(a.wl, reinterpret_cast<const T*>(a.wpack), Wl);
    if (!(a.ablate & 1)) load_tile<T, BM>(In, a.ldi, a.K0, KP0, a.seg, a.nseg, row0, a.M);
    if (MODE == MODE_NODE && !(a.ablate & 1)) {
        // aggregation: In[r][H + c] = sum over in-edges k of scale[c] * (z[k][c] / rden[k])
        constexpr int CPR = H / CH;
        const T* z = reinterpret_cast<const T*>(a.agg_z);
        for (int it = threadIdx.x; it < BM * CPR; it += MGN_THREADS) {
            const int r = it / CPR, c = (it - r * CPR) * CH;
            const int64_t row = row0 + r;
            float acc[CH];
#pragma unroll
            for (int v = 0; v < CH; ++v) acc[v] = 0.f;
            if (row < a.M) {
                float s[CH];
#pragma unroll
                for (int v = 0; v < CH; ++v) s[v] = a.agg_scale ? a.agg_scale[c + v] : 1.f;
                // groups of MGN_GEN_AG in-edges, every load of a group issued before its adds (one
                // round trip per group; edges past the segment end re-read its last edge and are not
                // added): the same sums in edge order as one edge at a time
                constexpr int AG = MGN_GEN_AG;
                const int kb = a.seg_ptr[row], ke = a.seg_ptr[row + 1];
                for (int k = kb; k < ke; k += AG) {
                    float zz[AG][CH], q[AG];
#pragma unroll
                    for (int u = 0; u < AG; ++u) {
                        const int ku = k + u < ke ? k + u : ke - 1;
                        Chunk<T>::load(z + (int64_t)ku * H + c, zz[u]);
                        q[u] = a.agg_rden[ku];
                    }
#pragma unroll
                    for (int u = 0; u < AG; ++u)
                        if (k + u < ke) {
#pragma unroll
                            for (int v = 0; v < CH; ++v) acc[v] += s[v] * (zz[u][v] / q[u]);
                        }
                }
                Chunk<T>::store(reinterpret_cast<T*>(a.agg_save) + row * H + c, acc);
            }
            Chunk<T>::store(In + (size_t)r * a.ldi + H + c, acc);
        }
    }
    if (WL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's weight copies landed
    __syncthreads();
    F32C_STAMP(0);
    // the layer-0 input of edge/node MLPs is re-gathered by the weight-gradient kernel
    if (MODE == MODE_DENSE && !(a.ablate & 2))
        copy_out_r8<T, BM>(In, a.ldi, KP0, reinterpret_cast<T*>(a.act8) + a.act_off[0], row0);
    F32C_STAMP(1);

    const T* wp = reinterpret_cast<const T*>(a.wpack);
    const T* cur = In;
    int ldc = a.ldi, KS = KP0 / KSTEP, K = a.Kpack0;
    for (int l = 0; l < a.L - 1; ++l) {
        Gemm<T, NTH, MT> g;
        if (WL)
            g.run_lds(Wl + a.wl.lo[l], KS, cur, ldc, l == 0 ? a.kstride0 : KS);
        else
            g.run(wp, KS, cur, ldc, a.ablate & 4, l == 0 ? a.kstride0 : KS);
        F32C_STAMP(2);
        T* nxt = (l & 1) ? P1 : P0;
        if (g.active) {
            const float* b = a.bias[l];
#pragma unroll
            for (int i = 0; i < Gemm<T, NTH, MT>::C::NTW; ++i) {
                const int n = g.n_of(i);
                const f4 bb = ld4u(b + n);
#pragma unroll
                for (int j = 0; j < Gemm<T, NTH, MT>::C::MTW; ++j) {
                    const int m = g.m_of(j);
                    f4 pp = {0.f, 0.f, 0.f, 0.f};
                    if (MODE == MODE_EDGE && l == 0 && a.proj && row0 + m < a.M) {
                        // [e ‖ x_i ‖ x_j]·W0ᵀ = e·W0aᵀ + (x·W0bᵀ)[dst] + (x·W0cᵀ)[src]
                        const f4 pi = *reinterpret_cast<const f4*>(a.proj + (int64_t)a.proj_i[row0 + m] * (2 * H) + n);
                        const f4 pj = *reinterpret_cast<const f4*>(a.proj + (int64_t)a.proj_j[row0 + m] * (2 * H) + H + n);
                        pp = pi + pj;
                    }
                    f4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = fmaxf(g.acc[i][j][r] + bb[r] + pp[r], 0.f);
                    st4(nxt + (size_t)m * a.ldh + n, v);
                    const int64_t mtile = (row0 >> 4) + g.mt0 + j;
                    unsigned long long* mw = a.mask + (int64_t)l * a.mask_stride + (mtile * NTH + g.nt0 + i) * 4;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const unsigned long long bits = __ballot(v[r] > 0.f);
                        if ((threadIdx.x & 63) == 0 && !(a.ablate & 8)) mw[r] = bits;
                    }
                }
            }
        }
        if (H % KSTEP != 0) {
            constexpr int padc = (H + KSTEP - 1) / KSTEP * KSTEP - H;
            for (int it = threadIdx.x; it < BM * padc; it += MGN_THREADS)
                nxt[(size_t)(it / padc) * a.ldh + H + it % padc] = from_f<T>(0.f);
        }
        __syncthreads();
        F32C_STAMP(3);
        if (!(a.ablate & 2))
            copy_out_r8<T, BM>(nxt, a.ldh, rup(H, KSTEP), reinterpret_cast<T*>(a.act8) + a.act_off[l + 1], row0);
        F32C_STAMP(4);
        wp += linear_pack_elems(H, K, dtype_id<T>());
        cur = nxt;
        ldc = a.ldh;
        KS = cdiv(H, KSTEP);
        K = H;
    }
    const T* wlast = WL ? Wl + a.wl.lo[a.L - 1] : wp;
    if (a.NOUT == H) {
        Gemm<T, NTH, MT> g;
        if (WL)
            g.run_lds(wlast, KS, cur, ldc);
        else
            g.run(wlast, KS, cur, ldc, a.ablate & 4);
        F32C_STAMP(5);
        if (a.ablate & 8) return;
        fwd_last_epilogue<T, BM>(g, a, red, reinterpret_cast<float*>(In), row0);
        F32C_STAMP(6);
        F32C_STAMP_PRINT(MODE == MODE_EDGE ? "gfe" : MODE == MODE_NODE ? "gfn" : "gfd");
    } else {
        Gemm<T, 1, MT> g;
        if (WL)
            g.run_lds(wlast, KS, cur, ldc);
        else
            g.run(wlast, KS, cur, ldc);
        fwd_last_epilogue<T, BM>(g, a, red, reinterpret_cast<float*>(In), row0);
    }
}

// --------------------------------------------------------------------------- backward (data)
struct BwdArgs {
    int64_t M;
    int32_t L, K0, H, NOUT, has_norm, ldh, mode;
    int32_t Kpack0;         // layer-0 packed width (EDGE: 3H, of which the e block K0 = H is used)
    float dinv;
    const void* wtpack;
    const float* scale;
    const unsigned long long* mask;  // ReLU ballot words (forward)
    int64_t mask_stride;
    const void* z_save;
    const float* rden_save;
    const void* dout;
    int32_t dout_dtype;
    int64_t dout_ld;
    const void* gath;       // EDGE: d_aggr [N][H] (T), added at gath_idx[row]
    const int32_t* gath_idx;
    void* dz8;              // [L] R8 blocks of [RP x H] (T): dZ of every layer, for the weight grads
    int64_t RP;
    float* dscale_part;     // [gridDim.x][NOUT]
    void* din;              // DENSE: [M][din_ld] (din_dtype), optional
    int32_t din_dtype;
    int64_t din_ld;
    void* o1;               // EDGE: de_in [M][H]; NODE: dx_part [M][H]  (T)
    void* o2;               // EDGE: dZ_0 [M][H] row-major; NODE: d_aggr [M][H]   (T)
    int32_t wl_elems;       // WL kernels: LDS element offset of the staged (transposed) weights
    WlDesc wl;
};

template <class T, int H, int BM, int MODE, bool WL = false>
__global__ __launch_bounds__(MGN_THREADS) void mlp_bwd_kernel(BwdArgs a) {
    constexpr int KSTEP = Mf<T>::KSTEP, VEC = Mf<T>::VEC;
    constexpr int NTH = H / 16, MT = BM / 16;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* D0 = reinterpret_cast<T*>(smem);
    T* D1 = D0 + BM * a.ldh;
    float* red = reinterpret_cast<float*>(D1 + BM * a.ldh);  // [256][4]
    T* Wl = reinterpret_cast<T*>(smem) + a.wl_elems;
    const int64_t row0 = (int64_t)blockIdx.x * BM;
    const int tid = threadIdx.x;
    const int NO = a.NOUT;
    const int KPN = rup(NO, KSTEP);
    if (WL) wl_issue<T>(a.wl, reinterpret_cast<const T*>(a.wtpack), Wl);

    // ---- dY -> dZ_last (RMSNorm backward), chunks of 4 columns; CPR lanes per row
    {
        const int CPR = cdiv(NO, 4);  // <= 64, divides 256 for NOUT in {H} or <= 16 rounded
        const int RPP = MGN_THREADS / CPR;  // rows per pass
        const int cc = (tid % CPR) * 4, rr = tid / CPR;
        f4 dsc = {0.f, 0.f, 0.f, 0.f};
        f4 s = {1.f, 1.f, 1.f, 1.f};
        if (a.has_norm) s = ld4u(a.scale + cc);
        // passes of RPP rows, 4 passes per batch: all loads of a batch are issued before use
        // batches of 4 passes until the tile's BM rows are covered (RPP = 4 at hidden 256: 4 batches of a
        // 32-row tile; 8+ rows per pass below)
        for (int p0 = 0; p0 * RPP < BM; p0 += 4) {
            f4 dy[4], z[4];
            float q[4];
            bool valid[4];
            int64_t gi[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int r = rr + (p0 + u) * RPP;
                valid[u] = r < BM && row0 + r < a.M;
                gi[u] = (MODE == MODE_EDGE && valid[u]) ? (int64_t)a.gath_idx[row0 + r] : 0;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t row = row0 + rr + (p0 + u) * RPP;
                dy[u] = f4{0.f, 0.f, 0.f, 0.f};
                z[u] = f4{0.f, 0.f, 0.f, 0.f};
                q[u] = 1.f;
                if (!valid[u]) continue;
                if (NO % 4 == 0) {
                    dy[u] = a.dout_dtype == MGN_F32
                                ? ld4(reinterpret_cast<const float*>(a.dout) + row * a.dout_ld + cc)
                                : ld4(reinterpret_cast<const __bf16*>(a.dout) + row * a.dout_ld + cc);
                } else {
#pragma unroll
                    for (int v = 0; v < 4; ++v)
                        dy[u][v] = cc + v < NO ? load_any(a.dout, a.dout_dtype, row * a.dout_ld + cc + v) : 0.f;
                }
                if (MODE == MODE_EDGE) {
                    const f4 g = ld4(reinterpret_cast<const T*>(a.gath) + gi[u] * H + cc);
#pragma unroll
                    for (int v = 0; v < 4; ++v) dy[u][v] += g[v];
                }
                if (a.has_norm) {
                    z[u] = ld4(reinterpret_cast<const T*>(a.z_save) + row * H + cc);
                    q[u] = a.rden_save[row];
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int r = rr + (p0 + u) * RPP;
                f4 dz = dy[u];
                if (a.has_norm) {
                    float dot = 0.f;
#pragma unroll
                    for (int v = 0; v < 4; ++v) dot += s[v] * dy[u][v] * z[u][v];
                    for (int o = 1; o < CPR; o <<= 1) dot += __shfl_xor(dot, o);
                    const float rms = q[u] - RMS_EPS;
                    const float coef = rms > 0.f ? dot / (q[u] * q[u] * rms) * (a.dinv * a.dinv) : 0.f;
#pragma unroll
                    for (int v = 0; v < 4; ++v) {
                        dz[v] = s[v] * dy[u][v] / q[u] - z[u][v] * coef;
                        dsc[v] += dy[u][v] * (z[u][v] / q[u]);
                    }
                }
                if (r < BM) st4(D0 + (size_t)r * a.ldh + cc, dz);
            }
        }
        // zero pad columns [NO4, max(KPN, H)) of D0
        const int NO4 = CPR * 4;
        const int padc = (KPN > H ? KPN : H) - NO4;
        if (padc > 0)
            for (int it = tid; it < BM * padc; it += MGN_THREADS) {
                const int r = it / padc, c = it - r * padc;
                D0[(size_t)r * a.ldh + NO4 + c] = from_f<T>(0.f);
            }
        if (a.has_norm) {
            *reinterpret_cast<f4*>(red + tid * 4) = dsc;
            __syncthreads();
            if (tid < CPR) {
                f4 t = {0.f, 0.f, 0.f, 0.f};
                for (int q2 = 0; q2 < RPP; ++q2) {
                    const f4 u = *reinterpret_cast<const f4*>(red + (q2 * CPR + tid) * 4);
                    t += u;
                }
#pragma unroll
                for (int v = 0; v < 4; ++v)
                    if (tid * 4 + v < NO) a.dscale_part[(int64_t)blockIdx.x * NO + tid * 4 + v] = t[v];
            }
        }
    }
    F32C_STAMP_DECL;
    if (WL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's weight copies landed
    __syncthreads();
    F32C_STAMP(0);
    copy_out_r8<T, BM>(D0, a.ldh, H, reinterpret_cast<T*>(a.dz8) + (int64_t)(a.L - 1) * a.RP * H, row0);
    F32C_STAMP(1);

    // ---- layers L-1 .. 1 : dZ_{l-1} = (dZ_l · W_l) ⊙ [A_{l-1} > 0]
    const T* wt = reinterpret_cast<const T*>(a.wtpack);
    int64_t off[MGN_MAX_LAYERS];
    {
        int64_t o = 0;
        for (int l = 0; l < a.L; ++l) {
            off[l] = o;
            const int n = l == a.L - 1 ? NO : H, k = l == 0 ? a.Kpack0 : H;
            o += linear_pack_elems(n, k, dtype_id<T>());
        }
    }
    T* cur = D0;
    T* nxt = D1;
    for (int l = a.L - 1; l >= 1; --l) {
        const int Nl = l == a.L - 1 ? NO : H;
        Gemm<T, NTH, MT> g;
        if (WL)
            g.run_lds(Wl + a.wl.lo[l], cdiv(Nl, KSTEP), cur, a.ldh);
        else
            g.run(wt + off[l], cdiv(Nl, KSTEP), cur, a.ldh);
        F32C_STAMP(2);
        if (g.active) {
            const int lane = tid & 63;
#pragma unroll
            for (int i = 0; i < Gemm<T, NTH, MT>::C::NTW; ++i) {
                const int k = g.n_of(i);
#pragma unroll
                for (int j = 0; j < Gemm<T, NTH, MT>::C::MTW; ++j) {
                    const int m = g.m_of(j);
                    const int64_t row = row0 + m;
                    const int64_t mtile = (row0 >> 4) + g.mt0 + j;
                    const unsigned long long* mw =
                        a.mask + (int64_t)(l - 1) * a.mask_stride + (mtile * NTH + g.nt0 + i) * 4;
                    f4 v = g.acc[i][j];
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = ((mw[r] >> lane) & 1ull) && row < a.M ? v[r] : 0.f;
                    st4(nxt + (size_t)m * a.ldh + k, v);
                }
            }
        }
        if (H % KSTEP != 0) {
            constexpr int padc = (H + KSTEP - 1) / KSTEP * KSTEP - H;
            for (int it = tid; it < BM * padc; it += MGN_THREADS)
                nxt[(size_t)(it / padc) * a.ldh + H + it % padc] = from_f<T>(0.f);
        }
        __syncthreads();
        F32C_STAMP(3);
        T* t = cur;
        cur = nxt;
        nxt = t;
        copy_out_r8<T, BM>(cur, a.ldh, H, reinterpret_cast<T*>(a.dz8) + (int64_t)(l - 1) * a.RP * H, row0);
        F32C_STAMP(4);
    }

    // ---- layer 0 : dA0 = dZ_0 · W_0, K0 columns in chunks of H
    if (MODE == MODE_DENSE && a.din == nullptr) return;
    if (MODE == MODE_EDGE) {
        // dZ_0 row-major for the node side: d(x·W0bᵀ)[v] = Σ_{dst(k)=v} dZ_0[k], likewise src
        constexpr int CH = 16 / sizeof(T);
        for (int it = tid; it < BM * (H / CH); it += MGN_THREADS) {
            const int r = it / (H / CH), cc = (it - r * (H / CH)) * CH;
            const int64_t row = row0 + r;
            if (row < a.M)
                *reinterpret_cast<u32x4*>(reinterpret_cast<T*>(a.o2) + row * H + cc) =
                    *reinterpret_cast<const u32x4*>(cur + (size_t)r * a.ldh + cc);
        }
    }
    const int KS0 = cdiv(a.L == 1 ? NO : H, KSTEP);
    const int nchunk = cdiv(cdiv(a.K0, 16), NTH);
    for (int c = 0; c < nchunk; ++c) {
        Gemm<T, NTH, MT> g;
        if (WL)
            g.run_lds(Wl + a.wl.lo[0] + c * NTH * KS0 * 64 * VEC, KS0, cur, a.ldh);
        else
            g.run(wt + off[0] + (int64_t)c * NTH * KS0 * 64 * VEC, KS0, cur, a.ldh);
        F32C_STAMP(5);
        if (MODE != MODE_DENSE) {
            // stage the chunk in the free LDS buffer, then write coalesced 16-byte row chunks
            if (g.active) {
#pragma unroll
                for (int i = 0; i < Gemm<T, NTH, MT>::C::NTW; ++i)
#pragma unroll
                    for (int j = 0; j < Gemm<T, NTH, MT>::C::MTW; ++j)
                        st4(nxt + (size_t)g.m_of(j) * a.ldh + g.n_of(i), g.acc[i][j]);
            }
            __syncthreads();
            constexpr int CH = 16 / sizeof(T);
            for (int it = tid; it < BM * (H / CH); it += MGN_THREADS) {
                const int r = it / (H / CH), cc = (it - r * (H / CH)) * CH;
                const int64_t row = row0 + r;
                if (row >= a.M) continue;
                float v[CH];
                Chunk<T>::load(nxt + (size_t)r * a.ldh + cc, v);
                if (c == 0) {
                    float d[CH];
                    Chunk<T>::load(reinterpret_cast<const T*>(a.dout) + row * a.dout_ld + cc, d);
#pragma unroll
                    for (int e = 0; e < CH; ++e) v[e] = d[e] + v[e];
                    Chunk<T>::store(reinterpret_cast<T*>(a.o1) + row * H + cc, v);
                } else if (MODE == MODE_NODE) {
                    Chunk<T>::store(reinterpret_cast<T*>(a.o2) + row * H + cc, v);
                }
            }
            __syncthreads();
            F32C_STAMP(6);
            if (c == nchunk - 1) F32C_STAMP_PRINT(MODE == MODE_EDGE ? "gbe" : "gbn");
            continue;
        }
        if (!g.active) continue;
#pragma unroll
        for (int i = 0; i < Gemm<T, NTH, MT>::C::NTW; ++i) {
            const int n = g.n_of(i);  // column within the chunk
#pragma unroll
            for (int j = 0; j < Gemm<T, NTH, MT>::C::MTW; ++j) {
                const int64_t row = row0 + g.m_of(j);
                if (row >= a.M) continue;
                const f4 v = g.acc[i][j];
                const int k = c * H + n;
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (k + r < a.K0) {
                        if (a.din_dtype == MGN_F32)
                            reinterpret_cast<float*>(a.din)[row * a.din_ld + k + r] = v[r];
                        else
                            reinterpret_cast<__bf16*>(a.din)[row * a.din_ld + k + r] = (__bf16)v[r];
                    }
            }
        }
    }
}

// --------------------------------------------------------------------------- weight gradients
// dW_l[n][k] = Σ_m dZ_l[m][n] · X_l[m][k], db_l[n] = Σ_m dZ_l[m][n]  (X_l = input of layer l).
// Both operands are R8 matrices written by the forward/backward kernels, so each MFMA fragment
// (VEC consecutive rows of one column) is a single 16-byte global load. A workgroup owns one
// (layer, 128-column block) output tile over a chunk of rows; partial tiles go to fp32 slabs that
// wgrad_reduce sums in a fixed order (deterministic, no atomics).
struct WgJob {
    int32_t layer, kb, n, k, kp, staged;  // staged: B operand re-gathered from seg[] through LDS
    int64_t w_off, b_off, act_off;        // b_off < 0: no bias for this job
    int32_t zl;                           // dZ operand = R8 block zl of dz8
    int32_t nb;                           // output-feature block: rows [nb*TW, nb*TW + TW) of dW (hidden > 128)
    // multi-MLP launches (WgArgs.multi): the job's own rows, operands, slabs and (staged) segment —
    // one launch then covers every weight gradient of a GraphNetBlock (edge MLP over edge rows, node
    // MLP and the edge W0's x blocks over node rows); blockIdx.x >= nchunks: idle workgroup
    int64_t RP, M;
    int32_t rows_per_chunk, nchunks;
    const void* dz8;
    const void* act8;
    float* part;
    int64_t G;
    SrcSeg seg;
};
struct WgArgs {
    int64_t RP, M;
    int32_t rows_per_chunk, H, njobs, gathered, nseg, multi;
    const void* dz8;
    const void* act8;
    SrcSeg seg[3];  // gathered != 0: layer-0 input segments (re-gathered, staged through LDS)
    WgJob job[12];
    float* part;
    int64_t G;
};

// Two groups of 4 waves per workgroup split the chunk's rows (alternate k-steps / stages) and
// combine their tiles through LDS in a fixed order: twice the resident waves of a 4-wave
// workgroup without more partial slabs.
constexpr int WG_GROUPS = 2;
// k-steps of R8 operands in flight in the weight-gradient kernel's direct (fp32) path (A/B builds:
// 0 = two, by unrolling) and workgroups per CU of its h <= 32 launches. Measured (Cfg A, fp32 h=32,
// weight-gradient launch per block): 2-deep / 4 per CU 30.7 us, 8-deep / 2 per CU 24.8 us (1,556 ->
// 1,611 steps/s), 8 / 1 38.1, 4 / 4 31.1, 16 / 1 45.1
#ifndef MGN_WG_PF
#define MGN_WG_PF 8
#endif
#ifndef MGN_WG_PER_CU32
#define MGN_WG_PER_CU32 2
#endif
// fp32 weight-gradient operands loaded as 16-byte row quads (A/B builds: 0 = one 4-byte fragment
// per k-step)
#ifndef MGN_WG_QUAD
#define MGN_WG_QUAD 1
#endif

// Output tile of a weight-gradient workgroup: TW x TW (TW = H up to 128). Hidden sizes above 128 (256:
// h = 129..256 zero-padded) split every dW into 128 x 128 tiles — job (kb, nb) = input columns
// [kb*TW, +TW) x output features [nb*TW, +TW) — so the h = 128 kernel's registers and LDS carry over.
template <int H>
constexpr int wg_tile() { return H > 128 ? 128 : H; }

template <class T, int H>
size_t wgrad_lds_bytes(bool staged) {
    constexpr int TW = wg_tile<H>();
    // re-gathered layer-0 input: [2][TW][64 + pad] per group; bf16 R8 input: [2][8 octets][TW] x 16 B
    const size_t stage = staged ? (size_t)WG_GROUPS * 2 * TW * (64 + 16 / sizeof(T)) * sizeof(T)
                                : (sizeof(T) == 2 ? (size_t)WG_GROUPS * 2 * 8 * TW * 16 : 0);
    const size_t red = (size_t)(TW * (TW + 4) + TW) * sizeof(float);  // canonical combine tile + bias row
    return stage > red ? stage : red;
}

template <class T, int H>
__global__ __launch_bounds__(MGN_THREADS * WG_GROUPS) void mlp_wgrad_kernel(WgArgs a) {
    constexpr int VEC = Mf<T>::VEC, KSTEP = Mf<T>::KSTEP;
    constexpr int TW = wg_tile<H>();            // output tile TW x TW (H: the dZ row width)
    constexpr int NT = TW / 16;
    constexpr int SR = 64;                      // rows per LDS stage
    constexpr int CH = 16 / sizeof(T);          // elements per 16-byte chunk
    constexpr int LDT = SR + CH;                // LDS row = one input column over SR rows (+pad)
    using C = TileCfg<NT, NT>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // group and wave index wave-uniform (readfirstlane): the row loops below then run on scalar
    // counters, without exec-masked exits
    const int grp = __builtin_amdgcn_readfirstlane(threadIdx.x / MGN_THREADS), tid = threadIdx.x % MGN_THREADS;
    T* AT = reinterpret_cast<T*>(smem) + (size_t)grp * 2 * TW * LDT;  // this group's [2][TW][LDT]
    F32C_STAMP_DECL;
    const WgJob job = a.job[blockIdx.y];
    const bool multi = a.multi != 0;
    if (multi && (int)blockIdx.x >= job.nchunks) return;  // uniform per workgroup, before any barrier
    const int64_t RP = multi ? job.RP : a.RP, Mrows = multi ? job.M : a.M, G = multi ? job.G : a.G;
    const int RPC = multi ? job.rows_per_chunk : a.rows_per_chunk;
    const void* dz8 = multi ? job.dz8 : a.dz8;
    const void* act8 = multi ? job.act8 : a.act8;
    float* const part0 = multi ? job.part : a.part;
    auto pick_seg = [&](int col0_) {
        if (multi) return job.seg;
        int s = 0;
        while (s + 1 < a.nseg && col0_ >= a.seg[s + 1].coff) ++s;
        return a.seg[s];
    };
    const int64_t r_begin = (int64_t)blockIdx.x * RPC;
    const int64_t r_end = r_begin + RPC < RP ? r_begin + RPC : RP;
    const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wn = wave % C::WN, wm = wave / C::WN;
    const int nt0 = wn * C::NTW, mt0 = wm * C::MTW;
    const bool active = mt0 < NT;
    const T* Z = reinterpret_cast<const T*>(dz8) + (int64_t)job.zl * RP * H;
    const T* X = reinterpret_cast<const T*>(act8) + job.act_off;
    const int col0 = job.kb * TW;
    const int n0 = job.nb * TW;  // first output feature (dZ column) of this tile
    const bool staged = job.staged != 0;
    bool kon[C::MTW];
#pragma unroll
    for (int j = 0; j < C::MTW; ++j) kon[j] = col0 + (mt0 + j) * 16 < job.kp;
    f4 acc[C::NTW][C::MTW];
#pragma unroll
    for (int i = 0; i < C::NTW; ++i)
#pragma unroll
        for (int j = 0; j < C::MTW; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    float bsum[C::NTW];
#pragma unroll
    for (int i = 0; i < C::NTW; ++i) bsum[i] = 0.f;
    const bool do_bias = job.b_off >= 0 && wm == 0 && active;
    const typename Mf<T>::frag zero{};
    auto bias_acc = [&](const typename Mf<T>::frag* fa) {
#pragma unroll
        for (int i = 0; i < C::NTW; ++i) {
            if constexpr (VEC == 1) {
                bsum[i] += to_f(fa[i]);
            } else {
#pragma unroll
                for (int v = 0; v < VEC; ++v) bsum[i] += (float)fa[i][v];
            }
        }
    };
    // Stage pipeline shared by the LDS-staged paths: the groups take alternate SR-row stages; the
    // next stage's X source loads AND its dZ fragments are issued before this stage's MFMAs, so a
    // stage exposes at most one memory latency (with two waves per SIMD the dZ loads issued inside
    // the k-loop used to expose one per k-step). Double-buffered LDS, one barrier per stage; every
    // group runs the same iteration count (a group past the end stages zeros) so all threads reach
    // each barrier. Loads past r_end are clamped to a valid stage and never consumed.
    constexpr int KS = SR / KSTEP;
    auto pipeline = [&](auto&& issue_x, auto&& commit_x, auto&& frag_b, auto&& frag_b4) {
      if constexpr (VEC == 1 && MGN_WG_QUAD && H <= 64) {
        // fp32: dZ as 16-byte row quads (see the direct path below) and the staged X read back as
        // the same quads (4 consecutive rows of a column in the [col][row] image: one ds_read_b128)
        constexpr int KQ = SR / 16;
        const int g4 = lane >> 4;
        f4 zq[KQ][C::NTW];
        auto issue_z = [&](int64_t m0) {
            const int64_t mc = m0 < r_end ? m0 : r_begin;
#pragma unroll
            for (int q = 0; q < KQ; ++q)
#pragma unroll
                for (int i = 0; i < C::NTW; ++i)
                    zq[q][i] = *reinterpret_cast<const f4*>(
                        reinterpret_cast<const float*>(Z) + (((mc + q * 16) >> 3) + (g4 >> 1)) * H * 8 +
                        (int64_t)(n0 + (nt0 + i) * 16 + (lane & 15)) * 8 + 4 * (g4 & 1));
        };
        issue_x(r_begin + grp * SR);
        issue_z(r_begin + grp * SR);
        for (int64_t base = r_begin; base < r_end; base += WG_GROUPS * SR) {
            const int64_t m0 = base + grp * SR;
            const int par = (int)((base - r_begin) / (WG_GROUPS * SR) & 1);
            commit_x(par);
            f4 za[KQ][C::NTW];
#pragma unroll
            for (int q = 0; q < KQ; ++q)
#pragma unroll
                for (int i = 0; i < C::NTW; ++i) za[q][i] = zq[q][i];
            __syncthreads();
            issue_x(m0 + WG_GROUPS * SR);
            issue_z(m0 + WG_GROUPS * SR);
            if (active && m0 < r_end) {
#pragma unroll
                for (int q = 0; q < KQ; ++q) {
                    f4 xb[C::MTW];
#pragma unroll
                    for (int j = 0; j < C::MTW; ++j) xb[j] = kon[j] ? frag_b4(par, q, j) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int v = 0; v < 4; ++v) {
                        typename Mf<T>::frag fa[C::NTW];
#pragma unroll
                        for (int i = 0; i < C::NTW; ++i) fa[i] = za[q][i][v];
#pragma unroll
                        for (int i = 0; i < C::NTW; ++i)
#pragma unroll
                            for (int j = 0; j < C::MTW; ++j) acc[i][j] = Mf<T>::mma(fa[i], xb[j][v], acc[i][j]);
                        if (do_bias) bias_acc(fa);
                    }
                }
            }
        }
      } else {
        typename Mf<T>::frag zn[KS][C::NTW];
        auto issue_z = [&](int64_t m0) {
            const int64_t mc = m0 < r_end ? m0 : r_begin;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
#pragma unroll
                for (int i = 0; i < C::NTW; ++i)
                    zn[ks][i] = ld_frag(Z + r8_index(mc + ks * KSTEP + VEC * (lane >> 4), n0 + (nt0 + i) * 16 + (lane & 15), H));
        };
        issue_x(r_begin + grp * SR);
        issue_z(r_begin + grp * SR);
        for (int64_t base = r_begin; base < r_end; base += WG_GROUPS * SR) {
            const int64_t m0 = base + grp * SR;
            const int par = (int)((base - r_begin) / (WG_GROUPS * SR) & 1);
            commit_x(par);
            typename Mf<T>::frag za[KS][C::NTW];
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
#pragma unroll
                for (int i = 0; i < C::NTW; ++i) za[ks][i] = zn[ks][i];
            __syncthreads();
            issue_x(m0 + WG_GROUPS * SR);
            issue_z(m0 + WG_GROUPS * SR);
            if (active && m0 < r_end) {
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) {
                    typename Mf<T>::frag fb[C::MTW];
#pragma unroll
                    for (int j = 0; j < C::MTW; ++j) fb[j] = kon[j] ? frag_b(par, ks, j) : zero;
#pragma unroll
                    for (int i = 0; i < C::NTW; ++i)
#pragma unroll
                        for (int j = 0; j < C::MTW; ++j) acc[i][j] = Mf<T>::mma(za[ks][i], fb[j], acc[i][j]);
                    if (do_bias) bias_acc(za[ks]);
                }
            }
        }
      }
    };
    auto no_b4 = [](int, int, int) { return f4{0.f, 0.f, 0.f, 0.f}; };  // bf16-only pipelines
    if (!staged && VEC == 8) {
        // R8 input: the 4 waves of a group all need the same 8 X fragments per k-step, so the
        // group copies each stage once (SR/8 octets x TW columns x 16 B, coalesced: in R8 an
        // octet's columns are contiguous) and the waves read their fragments from LDS (lanes 0-15
        // = 16 consecutive columns: conflict-free).
        constexpr int ITEMS = (SR / 8) * TW;
        constexpr int PER = (ITEMS + MGN_THREADS - 1) / MGN_THREADS;
        u32x4* img = reinterpret_cast<u32x4*>(smem) + (size_t)grp * 2 * ITEMS;
        u32x4 nxt[PER];
        pipeline(
            [&](int64_t m0) {
                const int64_t mc = m0 < r_end ? m0 : r_begin;
#pragma unroll
                for (int q = 0; q < PER; ++q) {
                    const int it = tid + q * MGN_THREADS;
                    const int o = it / TW, c = it % TW;
                    const int cc = col0 + c < job.kp ? col0 + c : 0;
                    nxt[q] = *reinterpret_cast<const u32x4*>(X + r8_index(mc + 8 * (it < ITEMS ? o : 0), cc, job.kp));
                    if (col0 + c >= job.kp) nxt[q] = u32x4{0u, 0u, 0u, 0u};
                }
            },
            [&](int par) {
                u32x4* buf = img + (size_t)par * ITEMS;
#pragma unroll
                for (int q = 0; q < PER; ++q)
                    if (tid + q * MGN_THREADS < ITEMS) buf[tid + q * MGN_THREADS] = nxt[q];
            },
            [&](int par, int ks, int j) {
                const u32x4* buf = img + (size_t)par * ITEMS;
                return ld_frag(reinterpret_cast<const T*>(buf + (ks * (KSTEP / 8) + (lane >> 4)) * TW + (mt0 + j) * 16 +
                                                          (lane & 15)));
            },
            no_b4);
    } else if (!staged && VEC == 1 && MGN_WG_QUAD) {
        if constexpr (VEC == 1) {
            // fp32 R8 operands as 16-byte quads: lane (g, f) = (lane >> 4, lane & 15) loads rows
            // 4g..4g+3 of a 16-row step of feature f (one f4: R8 keeps a feature's 8 rows contiguous),
            // so a wave's load is 1 KiB of whole 128-byte lines; k-step v of the quad then pairs
            // row 4g+v of dZ and X in lane (g, f). A 4-byte fragment load per k-step (lanes 32 B
            // apart) cost the texture addresser one cache access per lane: 64 per load, and the
            // launch was address-bound (Cfg A: 10.2M L1 accesses for 159k loads). Same products,
            // summed over the rows in another order. A ring of PQ quads per operand stays in flight.
            constexpr int PQ = H <= 32 ? 4 : H <= 64 ? 2 : 1;
            constexpr int64_t QSTEP = (int64_t)WG_GROUPS * 16;
            const int g4 = lane >> 4, fl = lane & 15;
            const int cz = fl < job.kp ? fl : 0;
            auto qidx = [&](int64_t m, int c, int64_t cols) {
                return ((m >> 3) + (g4 >> 1)) * cols * 8 + (int64_t)c * 8 + 4 * (g4 & 1);
            };
            f4 qa[PQ][C::NTW], qb[PQ][C::MTW];
            auto load = [&](int64_t m0, f4 (&fa)[C::NTW], f4 (&fb)[C::MTW]) {
                const int64_t m = m0 < r_end ? m0 : r_begin;
#pragma unroll
                for (int i = 0; i < C::NTW; ++i)
                    fa[i] = *reinterpret_cast<const f4*>(reinterpret_cast<const float*>(Z) + qidx(m, n0 + (nt0 + i) * 16 + fl, H));
#pragma unroll
                for (int j = 0; j < C::MTW; ++j)
                    fb[j] = *reinterpret_cast<const f4*>(reinterpret_cast<const float*>(X) +
                                                         qidx(m, kon[j] ? col0 + (mt0 + j) * 16 + fl : cz, job.kp));
            };
            const int64_t m_first = r_begin + grp * 16;
            if (active && m_first < r_end) {
                const int nq = (int)((r_end - m_first + QSTEP - 1) / QSTEP);
#pragma unroll
                for (int u = 0; u < PQ; ++u) load(m_first + u * QSTEP, qa[u], qb[u]);
                for (int q0 = 0; q0 < nq; q0 += PQ) {
#pragma unroll
                    for (int u = 0; u < PQ; ++u) {
                        const bool ok = q0 + u < nq;
                        f4 za[C::NTW], xb[C::MTW];
#pragma unroll
                        for (int i = 0; i < C::NTW; ++i) za[i] = ok ? qa[u][i] : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int j = 0; j < C::MTW; ++j) xb[j] = ok && kon[j] ? qb[u][j] : f4{0.f, 0.f, 0.f, 0.f};
                        load(m_first + (int64_t)(q0 + u + PQ) * QSTEP, qa[u], qb[u]);
#pragma unroll
                        for (int v = 0; v < 4; ++v) {
                            typename Mf<T>::frag fa[C::NTW];
#pragma unroll
                            for (int i = 0; i < C::NTW; ++i) fa[i] = za[i][v];
#pragma unroll
                            for (int i = 0; i < C::NTW; ++i)
#pragma unroll
                                for (int j = 0; j < C::MTW; ++j) acc[i][j] = Mf<T>::mma(fa[i], xb[j][v], acc[i][j]);
                            if (do_bias) bias_acc(fa);
                        }
                    }
                }
            }
        }
    } else if (!staged && MGN_WG_PF > 0) {
        // R8 operands straight from global memory (fp32: one VGPR per fragment): a register ring
        // keeps MGN_WG_PF k-steps of both operands in flight (the loop is unrolled by it so every
        // slot is static; loads past the chunk clamp to its first k-step and are never consumed).
        // Same MFMA sequence as one k-step at a time: bit-identical sums.
        constexpr int PF = MGN_WG_PF > 0 ? MGN_WG_PF : 1;
        constexpr int64_t STEP = (int64_t)WG_GROUPS * KSTEP;
        typename Mf<T>::frag ra[PF][C::NTW], rb[PF][C::MTW];
        auto load = [&](int64_t m0, typename Mf<T>::frag (&fa)[C::NTW], typename Mf<T>::frag (&fb)[C::MTW]) {
            const int64_t mr = (m0 < r_end ? m0 : r_begin) + VEC * (lane >> 4);
#pragma unroll
            for (int i = 0; i < C::NTW; ++i) fa[i] = ld_frag(Z + r8_index(mr, n0 + (nt0 + i) * 16 + (lane & 15), H));
            // unconditional loads (an inactive column block reads a valid column and is zeroed where
            // consumed): a load-or-zero join would again make the compiler copy the ring registers
            const int cz = (lane & 15) < job.kp ? (lane & 15) : 0;
#pragma unroll
            for (int j = 0; j < C::MTW; ++j)
                fb[j] = ld_frag(X + r8_index(mr, kon[j] ? col0 + (mt0 + j) * 16 + (lane & 15) : cz, job.kp));
        };
        const int64_t m_first = r_begin + grp * KSTEP;
        if (active && m_first < r_end) {
            // every slot of the ring is loaded and consumed unconditionally (a conditional exit
            // inside the unrolled ring made the compiler copy the ring registers, waiting on each
            // load right after issuing it: Cfg A's launch spent ~2k cycles per k-step); the steps
            // past the chunk's end (the count padded to a multiple of PF) multiply zeros (+0 to
            // every sum: same values)
            const int nsteps = (int)((r_end - m_first + STEP - 1) / STEP);
#pragma unroll
            for (int u = 0; u < PF; ++u) load(m_first + u * STEP, ra[u], rb[u]);
            for (int s0 = 0; s0 < nsteps; s0 += PF) {
#pragma unroll
                for (int u = 0; u < PF; ++u) {
                    const bool ok = s0 + u < nsteps;
                    typename Mf<T>::frag fa[C::NTW], fb[C::MTW];
#pragma unroll
                    for (int i = 0; i < C::NTW; ++i) fa[i] = ok ? ra[u][i] : zero;
#pragma unroll
                    for (int j = 0; j < C::MTW; ++j) fb[j] = ok && kon[j] ? rb[u][j] : zero;
                    load(m_first + (int64_t)(s0 + u + PF) * STEP, ra[u], rb[u]);
#pragma unroll
                    for (int i = 0; i < C::NTW; ++i)
#pragma unroll
                        for (int j = 0; j < C::MTW; ++j) acc[i][j] = Mf<T>::mma(fa[i], fb[j], acc[i][j]);
                    if (do_bias) bias_acc(fa);
                }
            }
        }
    } else if (!staged) {
#pragma unroll 2
        for (int64_t m0 = r_begin + grp * KSTEP; m0 < r_end; m0 += WG_GROUPS * KSTEP) {
            if (!active) break;
            const int64_t mr = m0 + VEC * (lane >> 4);
            typename Mf<T>::frag fa[C::NTW], fb[C::MTW];
#pragma unroll
            for (int i = 0; i < C::NTW; ++i) fa[i] = ld_frag(Z + r8_index(mr, n0 + (nt0 + i) * 16 + (lane & 15), H));
#pragma unroll
            for (int j = 0; j < C::MTW; ++j)
                fb[j] = kon[j] ? ld_frag(X + r8_index(mr, col0 + (mt0 + j) * 16 + (lane & 15), job.kp)) : zero;
#pragma unroll
            for (int i = 0; i < C::NTW; ++i)
#pragma unroll
                for (int j = 0; j < C::MTW; ++j) acc[i][j] = Mf<T>::mma(fa[i], fb[j], acc[i][j]);
            if (do_bias) bias_acc(fa);
        }
    } else if (VEC == 8 && TW == 128) {
        if constexpr (VEC == 8 && TW == 128) {
            // re-gathered layer-0 input, bf16 h=128: rows staged ROW-major (consecutive threads take
            // consecutive 16-byte chunks of one row: coalesced 256-byte row reads, one ds_write_b128
            // each) and the column-major B fragments read back with ds_read_b64_tr_b16 (two 4-row
            // blocks per fragment). Chunk ch of row r sits at slot ch ^ swz(r), which keeps both the
            // row writes and the transposed reads (a 32-lane half = two blocks 8 rows apart, same
            // columns) conflict-free.
            const SrcSeg g = pick_seg(col0);
            const T* src = reinterpret_cast<const T*>(g.p) + (col0 - g.coff);
            constexpr int CPR = TW / 8;                       // 16-byte chunks per row
            constexpr int ITEMS = SR * CPR;
            constexpr int PER = (ITEMS + MGN_THREADS - 1) / MGN_THREADS;
            char* img = smem + (size_t)grp * 2 * SR * TW * sizeof(T);
            auto slot = [](int r, int ch) { return r * (TW * (int)sizeof(T)) + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3))); };
            u32x4 nxt[PER];
            pipeline(
                [&](int64_t m0) {
    #pragma unroll
                    for (int q = 0; q < PER; ++q) {
                        const int it = tid + q * MGN_THREADS;
                        const int r = (it / CPR) % SR, ch = it % CPR;
                        const int64_t row = m0 + r;
                        const bool ok = it < ITEMS && m0 < r_end && row < Mrows;
                        const int64_t rc = ok ? row : 0;
                        const int64_t sr = g.idx ? (int64_t)g.idx[rc] : rc;
                        nxt[q] = *reinterpret_cast<const u32x4*>(src + sr * g.ld + ch * 8);
                        if (!ok) nxt[q] = u32x4{0u, 0u, 0u, 0u};
                    }
                },
                [&](int par) {
                    char* buf = img + (size_t)par * SR * TW * sizeof(T);
    #pragma unroll
                    for (int q = 0; q < PER; ++q) {
                        const int it = tid + q * MGN_THREADS;
                        if (it < ITEMS) *reinterpret_cast<u32x4*>(buf + slot(it / CPR, it % CPR)) = nxt[q];
                    }
                },
                [&](int par, int ks, int j) {
                    typedef short s4 __attribute__((ext_vector_type(4)));
                    typedef __attribute__((address_space(3))) s4 lds_s4;
                    const char* buf = img + (size_t)par * SR * TW * sizeof(T);
                    const int i = lane & 15, q = i >> 2, p = i & 3;
                    const int r0 = ks * KSTEP + 8 * (lane >> 4) + q;
                    const int ch = (mt0 + j) * 2 + (p >> 1);
                    const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(buf + slot(r0, ch) + 8 * (p & 1)));
                    const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(buf + slot(r0 + 4, ch) + 8 * (p & 1)));
                    typedef short s8 __attribute__((ext_vector_type(8)));
                    const s8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    return __builtin_bit_cast(typename Mf<T>::frag, v);
                },
                no_b4);
        }
    } else {
        // re-gathered layer-0 input: segment holding columns [col0, col0 + TW) (segments are H
        // wide); consecutive lanes take consecutive ROWS of one 16-byte column chunk, so the
        // transposed LDS writes (column-major AT[col][row]) hit consecutive 2-byte slots.
        const SrcSeg g = pick_seg(col0);
        const T* src = reinterpret_cast<const T*>(g.p);
        constexpr int ITEMS = SR * (TW / CH);
        constexpr int PER = (ITEMS + MGN_THREADS - 1) / MGN_THREADS;  // 16-byte chunks per thread
        u32x4 nxt[PER];
        pipeline(
            [&](int64_t m0) {
#pragma unroll
                for (int q = 0; q < PER; ++q) {
                    const int it = tid + q * MGN_THREADS;
                    const int r = it % SR, cc = (it / SR) * CH;
                    const int64_t row = m0 + r;
                    nxt[q] = u32x4{0u, 0u, 0u, 0u};
                    if (it < ITEMS && m0 < r_end && row < Mrows) {
                        const int64_t sr = g.idx ? (int64_t)g.idx[row] : row;
                        nxt[q] = *reinterpret_cast<const u32x4*>(src + sr * g.ld + (col0 - g.coff) + cc);
                    }
                }
            },
            [&](int par) {
                T* buf = AT + (size_t)par * TW * LDT;
#pragma unroll
                for (int q = 0; q < PER; ++q) {
                    const int it = tid + q * MGN_THREADS;
                    if (it >= ITEMS) continue;
                    const int r = it % SR, cc = (it / SR) * CH;
                    const T* v = reinterpret_cast<const T*>(&nxt[q]);
#pragma unroll
                    for (int e = 0; e < CH; ++e) buf[(size_t)(cc + e) * LDT + r] = v[e];
                }
            },
            [&](int par, int ks, int j) {
                const T* buf = AT + (size_t)par * TW * LDT;
                return ld_frag(buf + (size_t)((mt0 + j) * 16 + (lane & 15)) * LDT + ks * KSTEP + VEC * (lane >> 4));
            },
            [&](int par, int q, int j) {  // fp32 only: rows 16q + 4g .. +3 of the column
                const T* buf = AT + (size_t)par * TW * LDT;
                return *reinterpret_cast<const f4*>(buf + (size_t)((mt0 + j) * 16 + (lane & 15)) * LDT + q * 16 +
                                                    4 * (lane >> 4));
            });
    }
    F32C_STAMP(0);
    // Combine and store through a canonical [n][k] tile in LDS (row pitch TW+4 floats: the four
    // 16-lane groups of an accumulator write land 16 banks apart): group 1 deposits its tile,
    // group 0 adds its own, then all 512 threads store the slab rows with coalesced 16-byte stores
    // (the per-lane accumulator layout holds 4 rows x 1 column: scalar stores 4 rows apart).
    constexpr int LP = TW + 4;
    float* tile = reinterpret_cast<float*>(smem);
    float* btile = tile + TW * LP;
    float bt[C::NTW];
#pragma unroll
    for (int i = 0; i < C::NTW; ++i) {
        float t = bsum[i];
        t += __shfl_xor(t, 16);
        t += __shfl_xor(t, 32);
        bt[i] = t;
    }
    auto deposit = [&](bool add) {
#pragma unroll
        for (int i = 0; i < C::NTW; ++i) {
#pragma unroll
            for (int j = 0; j < C::MTW; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float* p = tile + ((nt0 + i) * 16 + (lane >> 4) * 4 + r) * LP + (mt0 + j) * 16 + (lane & 15);
                    *p = add ? *p + acc[i][j][r] : acc[i][j][r];
                }
            if (do_bias && lane < 16) {
                float* p = btile + (nt0 + i) * 16 + lane;
                *p = add ? *p + bt[i] : bt[i];
            }
        }
    };
    __syncthreads();  // staging buffers are dead
    if (grp == 1 && active) deposit(false);
    __syncthreads();
    if (grp == 0 && active) deposit(true);
    __syncthreads();
    float* part = part0 + (int64_t)blockIdx.x * G;
    constexpr int C4 = TW / 4;
    const bool vec = ((G | job.w_off | (int64_t)job.k) & 3) == 0;
    for (int it = threadIdx.x; it < TW * C4; it += MGN_THREADS * WG_GROUPS) {
        const int n = n0 + it / C4, k4 = (it % C4) * 4;
        const int kc = col0 + k4;
        if (n >= job.n || kc >= job.k) continue;
        const int nl = n - n0;
        const f4 v = *reinterpret_cast<const f4*>(tile + nl * LP + k4);
        float* dst = part + job.w_off + (int64_t)n * job.k + kc;
        if (vec && kc + 4 <= job.k) {
            *reinterpret_cast<f4*>(dst) = v;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (kc + e < job.k) dst[e] = v[e];
        }
    }
    if (job.b_off >= 0 && (int)threadIdx.x < job.n - n0 && (int)threadIdx.x < TW)
        part[job.b_off + n0 + threadIdx.x] = btile[threadIdx.x];
    F32C_STAMP(1);
    if (blockIdx.y == 0) F32C_STAMP_PRINT("gwg");
}

// Ring variant for bf16 h=128 (the hot configuration): the whole workgroup (8 waves as 4 n-groups
// x 2 k-groups, 2x4 16x16 tiles each) consumes one 32-row stage at a time from an 8-slot LDS ring
// filled by global_load_lds (LDS-DMA: no VGPR staging, so 7 stages = 112 KiB stay in flight per
// CU). A stage is the dZ block (R8: 8 KiB contiguous) and the X block (R8 octets, or re-gathered
// rows in the XOR-swizzled row image read by ds_read_b64_tr_b16; the swizzle is applied on the
// source addresses since LDS-DMA writes lane-linear). Each wave issues one 1 KiB piece of each per
// stage; a counted vmcnt + barrier publishes stage s while stages s+1..s+6 stay in flight. No group
// combine: every wave deposits its own tiles into the canonical LDS tile for the slab stores.
constexpr int RG_RS = 32;                 // rows per stage (one MFMA k-step)
constexpr int RG_NS = 8;                  // ring slots
constexpr int RG_SLOT = 2 * RG_RS * 128 * 2;  // dZ + X, bf16 h=128: 16 KiB
constexpr size_t RG_LDS = (size_t)RG_NS * RG_SLOT;

// A ring job is self-contained (its own dZ block, X source, row space, chunking and slab target),
// so one launch can cover several MLPs: WG b runs job j with wg0_j <= b < wg0_j + nchunks_j.
struct RgJob {
    const void* z;      // dZ: R8 [RP][128] block of this layer, or (zrm) row-major [RP][128] rows
    const void* x;      // X: R8 matrix (ld == 0, kp columns) or row-major rows (ld = row stride), both
                        // already offset to this job's first column
    int64_t ld, RP, M;
    float* part;        // slab base of the job's MLP; slab c at part + c * G
    int64_t G, w_off, b_off;
    int32_t n, k, kp, col0;
    int32_t rows_per_chunk, nchunks, wg0, zrm;  // zrm: dZ row-major (needs a row-major X: ld != 0)
};
struct RgArgs {
    int32_t njobs, pad;
    RgJob job[12];
};

#ifndef MGN_RG_JOBSCAN
#define MGN_RG_JOBSCAN 1  // A/B builds: 0 = the job found by a while loop over the arguments
#endif
// The job of this workgroup: the last j with wg0_j <= blockIdx.x (wg0 increases with j). The loop
// runs over the fixed-size array, unrolled, so every wg0's scalar load issues together; a while loop
// paid one dependent scalar-load round trip per job passed.
__device__ __forceinline__ int rg_job_index(const RgArgs& a) {
    int jn = 0;
#if MGN_RG_JOBSCAN
    constexpr int NJ = (int)(sizeof(a.job) / sizeof(a.job[0]));
#pragma unroll
    for (int j = 1; j < NJ; ++j)
        if (j < a.njobs && (int)blockIdx.x >= a.job[j].wg0) jn = j;
#else
    while (jn + 1 < a.njobs && (int)blockIdx.x >= a.job[jn + 1].wg0) ++jn;
#endif
    return jn;
}

// fp32 single-MLP job lists that mix 128-column jobs with narrower ones (A/B builds: 0 = all on the
// generic kernel)
#ifndef MGN_RING_SPLIT
#define MGN_RING_SPLIT 1
#endif

// fp32 ring (wgrad_ring_f32_kernel) for fp32 h=128 MLPs (A/B builds: 0 = the generic weight-gradient
// kernel, 3 launches + 2 reductions per block)
#ifndef MGN_RING_F32
#define MGN_RING_F32 1
#endif

// A-B builds only: cache policy of the ring's LDS-DMA streams (bit 0: X operand nt, bit 1: dZ nt)
#ifndef MGN_RING_NT
#define MGN_RING_NT 0
#endif
template <int AUX = 0>
__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, AUX);
}

__device__ __forceinline__ int rg_swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

// Slab write of a ring workgroup: the waves' 2x4 accumulator tiles (wave (wn, wk): feature blocks
// 2wn + i, column blocks 4wk + j of the job's 128-column block) through a canonical LDS tile (row pitch
// H+4 floats) + the bias row, then coalesced slab stores (as mlp_wgrad_kernel). smem must be free.
__device__ __forceinline__ void ring_epilogue(const RgJob& job, int chunk, const f4 (&acc)[2][4], const float (&bsum)[2],
                                              bool do_bias, int wn, int wk, int lane, char* smem) {
    constexpr int H = 128;
    constexpr int LP = H + 4;
    float* tile = reinterpret_cast<float*>(smem);
    float* btile = tile + H * LP;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                tile[((2 * wn + i) * 16 + (lane >> 4) * 4 + r) * LP + (4 * wk + j) * 16 + (lane & 15)] = acc[i][j][r];
        float t = bsum[i];
        t += __shfl_xor(t, 16);
        t += __shfl_xor(t, 32);
        if (do_bias && lane < 16) btile[(2 * wn + i) * 16 + lane] = t;
    }
    __syncthreads();
    float* part = job.part + (int64_t)chunk * job.G;
    constexpr int C4 = H / 4;
    const int col0 = job.col0;
    const bool vec = ((job.G | job.w_off | (int64_t)job.k) & 3) == 0;
    for (int it = threadIdx.x; it < H * C4; it += 512) {
        const int n = it / C4, k4 = (it % C4) * 4;
        const int kc = col0 + k4;
        if (n >= job.n || kc >= job.k) continue;
        const f4 v = *reinterpret_cast<const f4*>(tile + n * LP + k4);
        float* dst = part + job.w_off + (int64_t)n * job.k + kc;
        if (vec && kc + 4 <= job.k) {
            *reinterpret_cast<f4*>(dst) = v;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (kc + e < job.k) dst[e] = v[e];
        }
    }
    if (job.b_off >= 0 && (int)threadIdx.x < job.n && (int)threadIdx.x < H) part[job.b_off + threadIdx.x] = btile[threadIdx.x];
}

__global__ __launch_bounds__(512) void wgrad_ring_kernel(RgArgs a) {
    constexpr int H = 128;
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wn = w & 3, wk = w >> 2;
    const int jn = rg_job_index(a);
    const RgJob job = a.job[jn];
    const int chunk = (int)blockIdx.x - job.wg0;
    const int64_t r_begin = (int64_t)chunk * job.rows_per_chunk;
    const int64_t r_end = r_begin + job.rows_per_chunk < job.RP ? r_begin + job.rows_per_chunk : job.RP;
    const int nst = r_end > r_begin ? (int)((r_end - r_begin) / RG_RS) : 0;  // 0: zero slab
    const int col0 = job.col0;
    const bool staged = job.ld != 0;
    const __bf16* Z = reinterpret_cast<const __bf16*>(job.z);
    const __bf16* X = reinterpret_cast<const __bf16*>(job.x);
    // this lane's piece of a gathered stage: row 4w + (lane>>4), source chunk for its LDS slot
    const int gr = 4 * w + (lane >> 4), gch = (lane & 15) ^ rg_swz(gr);
    const bool zrm = job.zrm != 0;
    auto issue = [&](int s) {
        const int sc = s < nst ? s : nst - 1;  // past the end: reload the last stage, never consumed
        const int64_t m0 = r_begin + (int64_t)sc * RG_RS;
        char* slot = smem + (s % RG_NS) * RG_SLOT;
        // row-major dZ (rows < RP all written, padding rows zero): the X row image's swizzle
        glds16<(MGN_RING_NT & 2) ? 2 : 0>(zrm ? Z + (m0 + gr) * H + gch * 8 : Z + m0 * H + w * 512 + lane * 8,
                                          slot + w * 1024);
        const __bf16* xs;
        if (!staged) {
            xs = X + (((m0 >> 3) + (w >> 1)) * job.kp + (w & 1) * 64 + lane) * 8;
        } else {
            const int64_t row = m0 + gr < job.M ? m0 + gr : job.M - 1;
            xs = X + row * job.ld + gch * 8;
        }
        glds16<(MGN_RING_NT & 1) ? 2 : 0>(xs, slot + RG_SLOT / 2 + w * 1024);
    };
    f4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    float bsum[2] = {0.f, 0.f};
    const bool do_bias = job.b_off >= 0 && wk == 0;
    if (nst > 0) {
#pragma unroll
        for (int p = 0; p < RG_NS - 1; ++p) issue(p);
    }
    for (int s = 0; s < nst; ++s) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (RG_NS - 2)) : "memory");
        __builtin_amdgcn_s_barrier();
        issue(s + RG_NS - 1);
        const char* zi = smem + (s % RG_NS) * RG_SLOT;
        const char* xi = zi + RG_SLOT / 2;
        bf16x8 fa[2], fb[4];
        if (!zrm) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
                fa[i] = *reinterpret_cast<const bf16x8*>(zi + ((lane >> 4) * H + (2 * wn + i) * 16 + (lane & 15)) * 16);
        }
        if (zrm) {
            // dZ and X both row images: A fragments of feature blocks 2wn+i and B fragments of
            // column blocks 4wk+j by the same transposed reads (A[n][m] = dZ[m][n] has the form
            // of B[m][n'] = X[m][n'])
            const int i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
            const int r0 = 8 * (lane >> 4) + q;
            const unsigned zb = (unsigned)(uintptr_t)(zi), xb = (unsigned)(uintptr_t)(xi);
            u32x2 zl[2], zh[2], lo[4], hi[4];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int ch = (2 * wn + i) * 2 + (p >> 1);
                const unsigned a0 = zb + r0 * (H * 2) + 16 * (ch ^ rg_swz(r0)) + 8 * (p & 1);
                const unsigned a1 = zb + (r0 + 4) * (H * 2) + 16 * (ch ^ rg_swz(r0 + 4)) + 8 * (p & 1);
                asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(zl[i]) : "v"(a0));
                asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(zh[i]) : "v"(a1));
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ch = (4 * wk + j) * 2 + (p >> 1);
                const unsigned a0 = xb + r0 * (H * 2) + 16 * (ch ^ rg_swz(r0)) + 8 * (p & 1);
                const unsigned a1 = xb + (r0 + 4) * (H * 2) + 16 * (ch ^ rg_swz(r0 + 4)) + 8 * (p & 1);
                asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo[j]) : "v"(a0));
                asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi[j]) : "v"(a1));
            }
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(zl[0]), "+v"(zl[1]), "+v"(zh[0]), "+v"(zh[1]), "+v"(lo[0]), "+v"(lo[1]), "+v"(lo[2]),
                           "+v"(lo[3]), "+v"(hi[0]), "+v"(hi[1]), "+v"(hi[2]), "+v"(hi[3]));
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const u32x4 v = {zl[i][0], zl[i][1], zh[i][0], zh[i][1]};
                fa[i] = __builtin_bit_cast(bf16x8, v);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const u32x4 v = {lo[j][0], lo[j][1], hi[j][0], hi[j][1]};
                fb[j] = __builtin_bit_cast(bf16x8, v);
            }
        } else if (!staged) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                fb[j] = *reinterpret_cast<const bf16x8*>(xi + ((lane >> 4) * H + (4 * wk + j) * 16 + (lane & 15)) * 16);
        } else {
            // inline asm: with the builtin, hipcc waits vmcnt(0) (drains the ring) before the
            // transposed reads, assuming they may alias the in-flight LDS-DMA; the trailing wait
            // carries the values so no consumer is scheduled above it
            const int i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
            const int r0 = 8 * (lane >> 4) + q;
            const unsigned base = (unsigned)(uintptr_t)(xi);
            u32x2 lo[4], hi[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ch = (4 * wk + j) * 2 + (p >> 1);
                const unsigned a0 = base + r0 * (H * 2) + 16 * (ch ^ rg_swz(r0)) + 8 * (p & 1);
                const unsigned a1 = base + (r0 + 4) * (H * 2) + 16 * (ch ^ rg_swz(r0 + 4)) + 8 * (p & 1);
                asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo[j]) : "v"(a0));
                asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi[j]) : "v"(a1));
            }
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(lo[0]), "+v"(lo[1]), "+v"(lo[2]), "+v"(lo[3]), "+v"(hi[0]), "+v"(hi[1]), "+v"(hi[2]),
                           "+v"(hi[3]));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const u32x4 v = {lo[j][0], lo[j][1], hi[j][0], hi[j][1]};
                fb[j] = __builtin_bit_cast(bf16x8, v);
            }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        if (do_bias) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int v = 0; v < 8; ++v) bsum[i] += (float)fa[i][v];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing (unconsumed) ring loads
    __syncthreads();
    ring_epilogue(job, chunk, acc, bsum, do_bias, wn, wk, lane, smem);
}

// fp32 form of the ring (the reference's dtype, h = 128): the same self-contained jobs and slabs, on
// v_mfma_f32_16x16x4_f32. A 32-row stage is 16 KiB per operand (R8 dZ: the stage's 4 octets are
// contiguous; X: R8 octets, or 32 plain rows for the re-gathered layer-0 inputs) — 4 ring slots of
// 32 KiB, 3 stages in flight; every wave issues 4 pieces of 1 KiB per stage. The reduction over the
// stage's rows runs in octet order: MFMA j (0..7) takes row 8g + j into k-lane g, so lane (c, g) reads
// its 8 values of one R8 column with two 16-byte LDS loads (dZ, and X when R8).
constexpr int RF_RS = 32;
constexpr int RF_NS = 4;
constexpr int RF_SLOT = 2 * RF_RS * 128 * 4;
constexpr size_t RF_LDS = (size_t)RF_NS * RF_SLOT;
static_assert(RF_LDS >= (size_t)128 * 132 * 4 + 512, "the slab epilogue's tile reuses the ring");

__global__ __launch_bounds__(512) void wgrad_ring_f32_kernel(RgArgs a) {
    constexpr int H = 128;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wn = w & 3, wk = w >> 2;
    const int jn = rg_job_index(a);
    const RgJob job = a.job[jn];
    const int chunk = (int)blockIdx.x - job.wg0;
    const int64_t r_begin = (int64_t)chunk * job.rows_per_chunk;
    const int64_t r_end = r_begin + job.rows_per_chunk < job.RP ? r_begin + job.rows_per_chunk : job.RP;
    const int nst = r_end > r_begin ? (int)((r_end - r_begin) / RF_RS) : 0;  // 0: zero slab
    const bool staged = job.ld != 0;
    const float* Z = reinterpret_cast<const float*>(job.z);
    const float* X = reinterpret_cast<const float*>(job.x);
    auto issue = [&](int s) {
        const int sc = s < nst ? s : nst - 1;  // past the end: reload the last stage, never consumed
        const int64_t m0 = r_begin + (int64_t)sc * RF_RS;
        char* slot = smem + (s % RF_NS) * RF_SLOT;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int pc = 2 * w + p;  // piece 0..15 of each operand
            glds16(Z + m0 * H + pc * 256 + lane * 4, slot + pc * 1024);
            const float* xs;
            if (!staged) {
                xs = X + ((((m0 >> 3) + (pc >> 2)) * job.kp) + (pc & 3) * 32) * 8 + lane * 4;
            } else {
                const int64_t r = m0 + 2 * pc + (lane >> 5);
                xs = X + (r < job.M ? r : job.M - 1) * job.ld + (lane & 31) * 4;
            }
            glds16(xs, slot + RF_SLOT / 2 + pc * 1024);
        }
    };
    f4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    float bsum[2] = {0.f, 0.f};
    const bool do_bias = job.b_off >= 0 && wk == 0;
    const int c16 = lane & 15, g = lane >> 4;
    if (nst > 0) {
#pragma unroll
        for (int p = 0; p < RF_NS - 1; ++p) issue(p);
    }
    for (int s = 0; s < nst; ++s) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (RF_NS - 2)) : "memory");
        __builtin_amdgcn_s_barrier();
        issue(s + RF_NS - 1);
        const float* zi = reinterpret_cast<const float*>(smem + (s % RF_NS) * RF_SLOT);
        const float* xi = zi + RF_SLOT / 8;
        f4 za[2][2], xb[4][2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const float* p = zi + (g * H + (2 * wn + i) * 16 + c16) * 8;
            za[i][0] = *reinterpret_cast<const f4*>(p);
            za[i][1] = *reinterpret_cast<const f4*>(p + 4);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = (4 * wk + j) * 16 + c16;
            if (!staged) {
                const float* p = xi + (g * H + c) * 8;
                xb[j][0] = *reinterpret_cast<const f4*>(p);
                xb[j][1] = *reinterpret_cast<const f4*>(p + 4);
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) xb[j][e >> 2][e & 3] = xi[(8 * g + e) * H + c];
            }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(za[i][e >> 2][e & 3], xb[j][e >> 2][e & 3], acc[i][j],
                                                                     0, 0, 0);
        if (do_bias) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int e = 0; e < 8; ++e) bsum[i] += za[i][e >> 2][e & 3];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing (unconsumed) ring loads
    __syncthreads();
    ring_epilogue(job, chunk, acc, bsum, do_bias, wn, wk, lane, smem);
}

// grads[g] = Σ_c part[c][g] for g < G (blocks [0, ceil(G/64)): 64 outputs x 4 chunk groups each);
// grads[G + s] = Σ_t dscale_part[t][s] (one block per s). Fixed summation order: deterministic.
struct RedDesc {
    const float* part;
    const float* dsp;
    float* grads;
    int64_t G;
    int32_t nchunks, ntiles, NS, blocks;
    // optional column region of W0 ([w0_n][w0_k] at the start of the slab rows): columns >= xcol0
    // sum only their first nchunks_x slabs (w0_k == 0: none)
    int32_t w0_n, w0_k, xcol0, nchunks_x;
    // optional tail [hoff, G) summed over its own first nchunks_h slabs (the recomputed edge
    // weight gradients of layers 1.., chain16_edge_wgrad_recompute; hoff == 0: none)
    int64_t hoff;
    int32_t nchunks_h, pad;
};
// slabs summed for output g
__device__ __forceinline__ int red_nchunks(const RedDesc& d, int64_t g) {
    if (d.hoff > 0 && g >= d.hoff) return d.nchunks_h;
    if (d.w0_k > 0 && g < (int64_t)d.w0_n * d.w0_k && (int)(g % d.w0_k) >= d.xcol0) return d.nchunks_x;
    return d.nchunks;
}

// 16-byte form of the slab sum: a thread sums 4 consecutive outputs (the same per-output order as
// the scalar form: chunk group cg = c mod 4, chunks in increasing order, groups combined 0+1+2+3)
__device__ __forceinline__ bool red_vec(const RedDesc& d) {
    return (d.G & 3) == 0 && ((uintptr_t)d.part & 15) == 0;
}
__device__ __forceinline__ int64_t red_gblocks(const RedDesc& d) {
    return red_vec(d) ? (d.G + 255) / 256 : (d.G + 63) / 64;
}

__device__ __forceinline__ void reduce_block(const RedDesc& d, int64_t b, float* red) {
    const int64_t gblocks = red_gblocks(d);
    const int tid = threadIdx.x;
    const float* part = d.part;
    const int64_t G = d.G;
    if (b < gblocks && red_vec(d)) {
        const int64_t g = b * 256 + 4 * (tid & 63);
        const int cg = tid >> 6;
        f4 sum = f4{0.f, 0.f, 0.f, 0.f};
        const int nch = g < G ? red_nchunks(d, g) : 0;  // one column region per 4 outputs (k0 % 4 == 0)
        if (g < G) {
            int c = cg;
            for (; c + 12 < nch; c += 16) {
                const f4 v0 = *reinterpret_cast<const f4*>(part + (int64_t)c * G + g);
                const f4 v1 = *reinterpret_cast<const f4*>(part + (int64_t)(c + 4) * G + g);
                const f4 v2 = *reinterpret_cast<const f4*>(part + (int64_t)(c + 8) * G + g);
                const f4 v3 = *reinterpret_cast<const f4*>(part + (int64_t)(c + 12) * G + g);
                sum += v0;
                sum += v1;
                sum += v2;
                sum += v3;
            }
            for (; c < nch; c += 4) sum += *reinterpret_cast<const f4*>(part + (int64_t)c * G + g);
        }
        f4* r4 = reinterpret_cast<f4*>(red);
        r4[tid] = sum;
        __syncthreads();
        if (tid < 64 && g < G) {
            const f4 v = ((r4[tid] + r4[tid + 64]) + r4[tid + 128]) + r4[tid + 192];
            if (((uintptr_t)(d.grads + g) & 15) == 0) {
                *reinterpret_cast<f4*>(d.grads + g) = v;
            } else {  // the flat gradient buffer puts a block's slice at any 4-byte offset
#pragma unroll
                for (int q = 0; q < 4; ++q) d.grads[g + q] = v[q];
            }
        }
    } else if (b < gblocks) {
        const int64_t g = b * 64 + (tid & 63);
        const int cg = tid >> 6;
        float s = 0.f;
        if (g < G) {
            const int nch = red_nchunks(d, g);
            int c = cg;
            for (; c + 12 < nch; c += 16) {
                const float v0 = part[(int64_t)c * G + g], v1 = part[(int64_t)(c + 4) * G + g];
                const float v2 = part[(int64_t)(c + 8) * G + g], v3 = part[(int64_t)(c + 12) * G + g];
                s += v0;
                s += v1;
                s += v2;
                s += v3;
            }
            for (; c < nch; c += 4) s += part[(int64_t)c * G + g];
        }
        red[tid] = s;
        __syncthreads();
        if (tid < 64 && g < G) d.grads[g] = ((red[tid] + red[tid + 64]) + red[tid + 128]) + red[tid + 192];
    } else {
        const int sidx = (int)(b - gblocks);
        float s = 0.f;
        for (int t = tid; t < d.ntiles; t += MGN_THREADS) s += d.dsp[(int64_t)t * d.NS + sidx];
        red[tid] = s;
        __syncthreads();
        for (int w = MGN_THREADS / 2; w > 0; w >>= 1) {
            if (tid < w) red[tid] += red[tid + w];
            __syncthreads();
        }
        if (tid == 0) d.grads[G + sidx] = red[0];
    }
}

// one launch reducing up to RED_MAX MLPs (the blocks of desc 0, then desc 1, ...): a block
// backward's two MLPs, or every processor block's at the end of the backward (deferred reduction)
constexpr int RED_MAX = 32;
struct RedArgs {
    RedDesc d[RED_MAX];
    int32_t nd, pad;
};
__global__ __launch_bounds__(MGN_THREADS) void wgrad_reduce_kernel(RedArgs a) {
    __shared__ __attribute__((aligned(16))) float red[4 * MGN_THREADS];
    int64_t b = blockIdx.x;
    int i = 0;
    while (i + 1 < a.nd && b >= a.d[i].blocks) b -= a.d[i++].blocks;
    reduce_block(a.d[i], b, red);
}

// --------------------------------------------------------------------------- weight packing
// element (nn, kk) of a job's (possibly zero-padded) [n][k] matrix
__device__ __forceinline__ float pack_src(const mgn_pack_job& j, int nn, int kk) {
    if (j.kb_pad <= 0) return j.w[(int64_t)nn * j.k + kk];  // unpadded
    if (nn >= j.n_src) return 0.f;
    const int b = kk / j.kb_pad, c = kk - b * j.kb_pad;
    const int sc = b * j.kb_src + c;
    return c < j.kb_src && sc < j.k_src ? j.w[(int64_t)nn * j.k_src + sc] : 0.f;
}

template <class T>
__device__ __forceinline__ void pack_job(const mgn_pack_job& j) {
    constexpr int VEC = Mf<T>::VEC, KSTEP = Mf<T>::KSTEP;
    const int n = j.n, k = j.k;
    const int KS = cdiv(k, KSTEP), NTp = cdiv(n, 16);
    const int NS = cdiv(n, KSTEP), KTp = rup(cdiv(k, 16), 8);
    // one Linear's pack is far below 2^31 elements: 32-bit index math (64-bit divisions by the
    // runtime KS / NS cost tens of instructions each)
    const int tot = (int)linear_pack_elems(n, k, dtype_id<T>());
    const int img0 = tot - chain_images(n, k, dtype_id<T>()) * 128 * 128;  // chain images start
    T* dst = reinterpret_cast<T*>(j.dst);
    T* dstT = reinterpret_cast<T*>(j.dstT);
    for (int e = blockIdx.x * MGN_THREADS + threadIdx.x; e < tot; e += gridDim.x * MGN_THREADS) {
        if (e >= img0) {  // chain images (mgn_common.h): one per 128-column block, permuted k-steps
            const int i = e - img0, r = i & 3, lane = (i >> 2) & 63, t = (i >> 8) & 7, b = (i >> 11) & 7;
            const int cb = 128 * (i >> 14);  // the image's first input column
            const int a16 = b * 16 + (lane & 15), c = t * 16 + 4 * (lane >> 4) + r;
            dst[e] = from_f<T>(pack_src(j, a16, cb + c));   // W[a16][cb + c]
            dstT[e] = from_f<T>(pack_src(j, c, cb + a16));  // W[c][cb + a16]
            continue;
        }
        const int v = e % VEC;
        const int fl = e / VEC;
        const int lane = fl % 64;
        const int tile = fl / 64;
        {  // forward: tile = nt*KS + ks
            float w = 0.f;
            if (tile < NTp * KS) {
                const int nt = tile / KS, ks = tile % KS;
                const int nn = nt * 16 + (lane & 15), kk = ks * KSTEP + VEC * (lane >> 4) + v;
                if (nn < n && kk < k) w = pack_src(j, nn, kk);
            }
            dst[e] = from_f<T>(w);
        }
        {  // transposed: tile = kt*NS + ns
            float w = 0.f;
            if (tile < KTp * NS) {
                const int kt = tile / NS, ns = tile % NS;
                const int kk = kt * 16 + (lane & 15), nn = ns * KSTEP + VEC * (lane >> 4) + v;
                if (nn < n && kk < k) w = pack_src(j, nn, kk);
            }
            dstT[e] = from_f<T>(w);
        }
    }
}

// one launch for every job of either dtype (the job's dtype picks the fragment format)
__global__ __launch_bounds__(MGN_THREADS) void pack_kernel(const mgn_pack_job* jobs) {
    const mgn_pack_job j = jobs[blockIdx.y];
    if (j.dtype == MGN_F32)
        pack_job<float>(j);
    else
        pack_job<__bf16>(j);
}

// --------------------------------------------------------------------------- fp32 edge MLP, register-chained
// The fp32 GraphNetBlock edge MLP at h = 128 (4 Linears + RMSNorm, reference layers.py:652-658,
// 703-719): each wave owns 16 edge rows through all four layers; activations never leave registers.
// Layer l computes D^T[n][row] = Σ_k W[n][k]·X[row][k] with v_mfma_f32_16x16x4_f32; its C layout
// (lane l, reg r: feature 16nt + 4(l>>4) + r of row l&15) is, unchanged, the B operand of layer l+1
// when that layer's k-step (t, r) covers k = 16t + 4(l>>4) + r: a GEMM's k axis may be summed in any
// order, so only the A operand (the weights) follows the permutation. The pack kernel writes each
// 128-wide fp32 Linear's first 128 input columns once more in that order (the "chain image", after the
// fragments: lane l's four k-steps (t, r = 0..3) of n-tile nt as one 16-byte word, forward
// W[16nt + (l&15)][16t + 4(l>>4) + r], transposed W[16t + 4(l>>4) + r][16nt + (l&15)]); a 12-wave
// workgroup streams layer l+1's 64 KiB image into LDS by LDS-DMA while layer l's MFMAs run (double
// buffer, one barrier per layer). Measured on the way (Cfg B, fp32 step): weights streamed from L2 per
// wave (four dword loads per 4 MFMAs) 227–238 µs per edge forward vs 173 µs for the generic kernel;
// register-staged permutation through ds_write, 8 waves: 169.5 / 187 µs (forward / backward vs 173 /
// 186); the same with 4-wave workgroups spilled 200+ bytes per lane.
#ifndef MGN_F32_CHAIN
#define MGN_F32_CHAIN 1  // 0: the fp32 edge MLP on the generic LDS-tiled kernels (A/B builds)
#endif
#ifndef MGN_F32C_SB
#define MGN_F32C_SB 0  // 1: single-buffered images, 6-wave workgroups, two workgroups per CU (A/B builds)
#endif
// MGN_F32C_FLOW (round 6): the forward's per-layer workgroup barrier replaced by LDS counters — a wave
// waits only for the image of the layer it is about to run (ready[l]); the last wave to finish reading an
// image stages layer l+2 into it. Waves drift apart by up to a layer, so one wave's ReLU / mask / store
// phase runs beside another's MFMAs on the same SIMD instead of the whole workgroup idling the MFMA pipe
// in lock-step.
#ifndef MGN_F32C_FLOW
#define MGN_F32C_FLOW 1
#endif
static_assert(!MGN_F32C_FLOW || !MGN_F32C_SB, "the flow-synchronized form needs the double-buffered images");
constexpr int F32C_WAVES = MGN_F32C_SB ? 6 : 12;  // three waves per SIMD (168 VGPRs), 16 rows per wave
constexpr int F32C_NBUF = MGN_F32C_SB ? 1 : 2;    // LDS chain images per workgroup
#define F32C_BOUNDS __launch_bounds__(F32C_WAVES * 64, 3)
constexpr int F32C_LAYER = 128 * 128;  // floats per chain image (64 KiB)

// The chain image of input columns 128b .. 128b + 127 in a pack region (fwd or transposed) of a fp32
// [n][k] Linear: the images follow the fragments (linear_pack_elems counts them: n == 128, k a multiple
// of 128, one per 128-column block).
__host__ __device__ inline int64_t chain_image_off(int n, int k, int b = 0) {
    return linear_pack_elems(n, k, MGN_F32) - (int64_t)(chain_images(n, k, MGN_F32) - b) * F32C_LAYER;
}

// Issue this wave's share of one 64 KiB image copy global -> LDS (1 KiB per LDS-DMA instruction).
__device__ __forceinline__ void f32c_stage(const float* __restrict__ src, float* img) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int c = wave; c < F32C_LAYER / 256; c += F32C_WAVES)
        glds16(src + c * 256 + lane * 4, img + c * 256);
}
__device__ __forceinline__ void f32c_stage_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// 4x4 transpose inside each lane quad (lanes 4k..4k+3): lane i's v[r] <- lane r's v[i] (two DPP
// butterfly stages: swap across lane bit 0, then bit 1). The moves are inline asm: with
// __builtin_amdgcn_mov_dpp / update_dpp this ROCm 7.2 compiler folds the selects below into ONE DPP
// move per stage (wrong values; an isolated 4-DPP kernel shows it); s_nop 1 covers the VALU-write ->
// DPP-read hazard, which the compiler cannot see inside asm.
__device__ __forceinline__ float dpp_xor1(float x) {
    float r;
    asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ float dpp_xor2(float x) {
    float r;
    asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ f4 quad_transpose(f4 v, int lane) {
    f4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float p = dpp_xor1(v[r ^ 1]);
        o[r] = ((r ^ lane) & 1) ? p : v[r];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float p = dpp_xor2(o[r ^ 2]);
        v[r] = ((r ^ lane) & 2) ? p : o[r];
    }
    return v;
}

#ifndef MGN_F32C_DPPRED
#define MGN_F32C_DPPRED 1  // 0: the fp32 backward's RMSNorm-scale row sums on LDS-crossbar shuffles (A/B builds)
#endif
// the 4 components of v summed over the 16 lanes of a DPP row (as mgn_chain16.hip's row16_sum4):
// lane m returns component 2(m&1) + ((m>>1)&1); pairs m^1 trade two components, pairs m^2 one, then
// rotations by 4 and 8 add the four lanes holding the same component
__device__ __forceinline__ float f32c_row16_sum4(const f4& v, int m) {
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

// The lane's address in a fp32 R8 save [rows/8][128][8] for the quad-transposed operand: lane (row, g)
// holds column 16t + 4g + (row & 3) of rows (row & ~3) .. +3 after quad_transpose — 16 contiguous bytes,
// and the 8 lanes of a row octet cover one 128-byte line (columns c..c+3 x 8 rows).
__device__ __forceinline__ int64_t f32c_r8t(int64_t row, int g) {
    return ((row >> 3) * 128 + 4 * g + (row & 3)) * 8 + (row & 4);
}

// acc[nt] += D^T tile nt of X·Wᵀ (16 rows) from the LDS image; x[t][r] = B operand of k-step (t, r).
// save != NULL: also store the operand to its R8 save (save = f32c_r8t of the lane; x[t][r] is column
// 16t + 4(l>>4) + r of the lane's row): one quad-transposed 16-byte store per k-step group (full 128-byte
// lines: 8 store instructions per layer instead of 32 partial-line dword stores), spread over the MFMAs
// (stored at once after each layer, every wave of the chip writes at the same time).
__device__ __forceinline__ void f32c_gemm(f4 (&acc)[8], const f4 (&x)[8], const float* img, int lane,
                                          float* save = nullptr) {
    // LDS reads run one half k-step group ahead (n-tiles 0..3, then 4..7: 16 MFMAs per half)
    f4 w[2][4];
    const f4* ip = reinterpret_cast<const f4*>(img) + lane;
#pragma unroll
    for (int j = 0; j < 4; ++j) w[0][j] = ip[(j * 8 + 0) * 64];
#pragma unroll
    for (int h = 0; h < 16; ++h) {
        const int t = h >> 1, n0 = (h & 1) * 4;
        if (h + 1 < 16) {
            const int t1 = (h + 1) >> 1, n1 = ((h + 1) & 1) * 4;
#pragma unroll
            for (int j = 0; j < 4; ++j) w[(h + 1) & 1][j] = ip[((n1 + j) * 8 + t1) * 64];
        }
        __builtin_amdgcn_sched_barrier(0);  // the next LDS reads stay ahead of these MFMAs
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[n0 + j] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[h & 1][j][r], x[t][r], acc[n0 + j], 0, 0, 0);
        if (save && (h & 1)) *reinterpret_cast<f4*>(save + 128 * t) = quad_transpose(x[t], lane);
    }
}

// LDS counters of the flow-synchronized form: done[l] waves finished reading layer l's image, ready[l]
__device__ __forceinline__ void f32c_wait(const unsigned* f, unsigned target) {
    for (unsigned n = 0; n < (1u << 26); ++n) {  // bounded: a correct schedule never comes near
        if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) break;
        __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

__global__ F32C_BOUNDS void edge_fwd_f32_chain_kernel(FwdArgs a) {
    constexpr int H = 128;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* const img0 = reinterpret_cast<float*>(smem);
    float* const img1 = img0 + (F32C_NBUF - 1) * F32C_LAYER;
    float* const vec = img0 + F32C_NBUF * F32C_LAYER;  // [5][H]: biases b0..b3, RMSNorm scale (LDS: no VMEM loads
                                           // behind the saves' stores, which would wait for them)
    unsigned* const flg = reinterpret_cast<unsigned*>(vec + 5 * 128);  // MGN_F32C_FLOW: done[4], ready[4]
    const int lane = threadIdx.x & 63, g = lane >> 4, ri = lane & 15;
    const int64_t tile = (int64_t)blockIdx.x * F32C_WAVES + (threadIdx.x >> 6);
    const int64_t row0 = tile * 16, row = row0 + ri;
    const bool live = row0 < rows_pad(a.M);  // tiles past the padded rows only join the barriers
    const bool valid = row < a.M;
    F32C_STAMP_DECL;
    const float* pk = reinterpret_cast<const float*>(a.wpack);
    f32c_stage(pk + chain_image_off(H, a.Kpack0), img0);  // layer 0: W0's e-column block
    pk += linear_pack_elems(H, a.Kpack0, MGN_F32);
    // unconditional loads (rows past the end read the last row, then select 0): a conditional load
    // compiles to a branch plus a full wait, eight of them in a row for the gathers
    const int64_t rowc = valid ? row : a.M - 1;
    const int32_t pi = a.proj_i[rowc], pj = a.proj_j[rowc];
    const float* e = reinterpret_cast<const float*>(a.seg[0].p);
    f4 x[8], acc[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) x[t] = *reinterpret_cast<const f4*>(e + rowc * a.seg[0].ld + 16 * t + 4 * g);
    // layer 0's accumulator starts at P_i + P_j + b0: [e ‖ x_i ‖ x_j]·W0ᵀ = e·W0aᵀ + (x·W0bᵀ)[dst] + (x·W0cᵀ)[src]
    {
        const f4* ppi = reinterpret_cast<const f4*>(a.proj + (int64_t)pi * (2 * H)) + g;
        const f4* ppj = reinterpret_cast<const f4*>(a.proj + (int64_t)pj * (2 * H) + H) + g;
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) acc[nt] = ppi[4 * nt];
        __builtin_amdgcn_sched_barrier(0);  // two passes: 32 registers of gathers in flight, not 64
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) acc[nt] += ppj[4 * nt];
    }
    if (!valid) {
#pragma unroll
        for (int t = 0; t < 8; ++t) x[t] = acc[t] = f4{0.f, 0.f, 0.f, 0.f};
    }
    for (int i = threadIdx.x; i < 5 * H; i += F32C_WAVES * 64) {
        const int vl = i >> 7;
        const float* vp = vl == 0 ? a.bias[0] : vl == 1 ? a.bias[1] : vl == 2 ? a.bias[2] : vl == 3 ? a.bias[3] : a.scale;
        vec[i] = vp[i & (H - 1)];
    }
    if (MGN_F32C_FLOW && threadIdx.x < 8) flg[threadIdx.x] = 0u;
    f32c_stage_wait();
    __syncthreads();
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) acc[nt] += *reinterpret_cast<const f4*>(vec + 16 * nt + 4 * g);
    F32C_STAMP(0);
    float* act = reinterpret_cast<float*>(a.act8);
    const int64_t r8 = f32c_r8t(row, g);  // transposed R8 saves
    const float* res = reinterpret_cast<const float*>(a.resid);
    const int wave = threadIdx.x >> 6;
    const float* pk2 = pk;  // MGN_F32C_FLOW: layer l's chain image at pk2 + (l - 1) * step + image offset
    const int64_t pstep = linear_pack_elems(H, H, MGN_F32);
    bool loader = false;    // MGN_F32C_FLOW: this wave staged layer l+2 and signals ready[l+2] after its V_l
#pragma unroll 1
    for (int l = 0; l < 4; ++l) {
        const float* nxt = nullptr;
        if (MGN_F32C_FLOW) {
            if (l == 0) f32c_stage(pk2 + chain_image_off(H, H), img1);  // layer 1, every wave's share
            if (l >= 1) f32c_wait(flg + 4 + l, l == 1 ? F32C_WAVES : 1u);
        } else if (l < 3) {
            // layer l+1's image streams into the other buffer during this layer's MFMAs (its readers,
            // layer l-1, passed the last barrier); single-buffered: after every wave's MFMAs
            nxt = pk + chain_image_off(H, H);
            if (F32C_NBUF == 2) f32c_stage(nxt, (l & 1) ? img0 : img1);
            pk += linear_pack_elems(H, H, MGN_F32);
        }
        // layer l's input (the ReLU output of layer l-1) is saved while it feeds the MFMAs
        // (save pointers by selection: a kernel-argument array indexed at run time is copied to scratch)
        float* sv = l == 1 ? act + a.act_off[1] : l == 2 ? act + a.act_off[2] : act + a.act_off[3];
        f32c_gemm(acc, x, (l & 1) ? img1 : img0, lane, (l > 0 && live) ? sv + r8 : nullptr);
        F32C_STAMP(1);
        if (MGN_F32C_FLOW) {
            // done reading layer l's image (its reads were consumed by the MFMAs): the last wave out
            // stages layer l+2 into it
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            unsigned old = 0;
            if (lane == 0) old = __hip_atomic_fetch_add(flg + l, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            old = __builtin_amdgcn_readfirstlane(old);
            loader = l + 2 <= 3 && old == F32C_WAVES - 1;
            if (loader) {
                const float* src = pk2 + (int64_t)(l + 1) * pstep + chain_image_off(H, H);
                float* img = (l & 1) ? img1 : img0;
                for (int c = 0; c < F32C_LAYER / 256; ++c) glds16(src + c * 256 + lane * 4, img + c * 256);
            }
        }
        if (l < 3) {
            unsigned long long word = 0;
#pragma unroll
            for (int nt = 0; nt < 8; ++nt) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float v = fmaxf(acc[nt][r], 0.f);
                    x[nt][r] = v;
                    const unsigned long long bits = __ballot(v > 0.f);
                    if (lane == nt * 4 + r) word = bits;
                }
                acc[nt] = *reinterpret_cast<const f4*>(vec + (l + 1) * H + 16 * nt + 4 * g);
            }
            // the tile's 32 ballot words of layer l: word nt*4 + r from lane nt*4 + r
            if (live && lane < 32) a.mask[(int64_t)l * a.mask_stride + tile * 32 + lane] = word;
            F32C_STAMP(2);
            if (MGN_F32C_FLOW) {
                f32c_stage_wait();  // this wave's share of layer 1 (l = 0), the image it staged (loader)
                asm volatile("" ::: "memory");
                if (lane == 0) {
                    if (l == 0) __hip_atomic_fetch_add(flg + 5, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (loader) __hip_atomic_store(flg + 4 + l + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                (void)wave;
            } else {
                if (F32C_NBUF == 1) {
                    __syncthreads();
                    f32c_stage(nxt, img0);
                }
                f32c_stage_wait();
                __syncthreads();
            }
            F32C_STAMP(3);
        }
    }
    // the residual rows after the last GEMM (round 6: loaded during it, their 32 registers on top of the
    // GEMM's made the kernel spill ~33 registers per lane at the 168-register cap; now 138, no spills:
    // edge forward 153 -> 144 us at fp32 Cfg B, profiles/r06_fp32_ab.txt)
    f4 rv[8];
#pragma unroll
    for (int nt = 0; nt < 8; ++nt)
        rv[nt] = (res && valid) ? *reinterpret_cast<const f4*>(res + row * H + 16 * nt + 4 * g) : f4{0.f, 0.f, 0.f, 0.f};
    // last Linear (bias in the accumulator): RMSNorm over the row's 128 features (4 lanes of 32), residual
    float ss = 0.f;
#pragma unroll
    for (int nt = 0; nt < 8; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) ss += acc[nt][r] * acc[nt][r];
    ss += __shfl_xor(ss, 16);
    ss += __shfl_xor(ss, 32);
    if (valid) {
        const float q = sqrtf(ss) * a.dinv + RMS_EPS;
        if (g == 0) a.rden_save[row] = q;
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) {
            const int n = 16 * nt + 4 * g;
            const f4 s = *reinterpret_cast<const f4*>(vec + 4 * H + n);
            f4 y;
#pragma unroll
            for (int r = 0; r < 4; ++r) y[r] = s[r] * (acc[nt][r] / q);
            y = rv[nt] + y;
            st4(reinterpret_cast<float*>(a.z_save) + row * H + n, acc[nt]);
            if (a.out_dtype == MGN_BF16)
                st4(reinterpret_cast<__bf16*>(a.out) + row * a.out_ld + n, y);
            else
                st4(reinterpret_cast<float*>(a.out) + row * a.out_ld + n, y);
        }
    }
    F32C_STAMP(4);
    F32C_STAMP_PRINT("f32f");
}

// Backward of the same MLP (data gradients; the weight gradients run on the fp32 ring from the dZ
// saves): the RMSNorm backward gives dZ3 in the C layout, and dH_l^T[k][row] = Σ_n W_l[n][k]·dZ_l[row][n]
// chains exactly like the forward with the transposed chain images. Outputs match mlp_bwd_kernel: dZ_l
// R8 saves, dZ_0 row-major, de_in = dout + dZ_0·W0a, and RMSNorm-scale partials per 32 rows (the
// generic kernel's partial count: two waves combine in LDS).
__global__ F32C_BOUNDS void edge_bwd_f32_chain_kernel(BwdArgs a) {
    constexpr int H = 128;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* const img0 = reinterpret_cast<float*>(smem);
    float* const img1 = img0 + (F32C_NBUF - 1) * F32C_LAYER;
    float* const red = img0 + F32C_NBUF * F32C_LAYER;  // [F32C_WAVES][H] per-wave RMSNorm-scale partials
    unsigned* const flg = reinterpret_cast<unsigned*>(red + F32C_WAVES * 128);  // MGN_F32C_FLOW: done[4], ready[4]
    const int lane = threadIdx.x & 63, g = lane >> 4, ri = lane & 15, wave = threadIdx.x >> 6;
    const int64_t tile = (int64_t)blockIdx.x * F32C_WAVES + wave;
    const int64_t row0 = tile * 16, row = row0 + ri;
    const bool live = row0 < a.RP;
    const bool valid = row < a.M;
    F32C_STAMP_DECL;
    const float* wt = reinterpret_cast<const float*>(a.wtpack);
    int64_t off[4];
    {
        int64_t o = 0;
        for (int l = 0; l < 4; ++l) {
            off[l] = o;
            o += linear_pack_elems(H, l == 0 ? a.Kpack0 : H, MGN_F32);
        }
    }
    f32c_stage(wt + off[3] + chain_image_off(H, H), img0);
    // the tile's ReLU mask words of hidden layers 0..2 (word nt*4 + r in lane nt*4 + r), loaded before
    // any store: a VMEM load issued behind stores waits for them
    unsigned long long mw[3] = {0ull, 0ull, 0ull};
    if (live && lane < 32) {
#pragma unroll
        for (int l = 0; l < 3; ++l) mw[l] = a.mask[(int64_t)l * a.mask_stride + tile * 32 + lane];
    }
    // ---- dY = dout + d_aggr[dst] -> dZ3 (RMSNorm backward)
    f4 dz[8], z[8];
    float q = 1.f;
    {
        // unconditional loads of the last row for rows past the end (then 0): see the forward
        const int64_t rowc = valid ? row : a.M - 1;
        const int64_t gi = a.gath_idx[rowc];
        const float* dout = reinterpret_cast<const float*>(a.dout);
        const float* gath = reinterpret_cast<const float*>(a.gath);
        const float* zs = reinterpret_cast<const float*>(a.z_save);
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) {
            const int n = 16 * nt + 4 * g;
            dz[nt] = *reinterpret_cast<const f4*>(dout + rowc * a.dout_ld + n);
            z[nt] = *reinterpret_cast<const f4*>(zs + rowc * H + n);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) dz[nt] += *reinterpret_cast<const f4*>(gath + gi * H + 16 * nt + 4 * g);
        const float qv = a.rden_save[rowc];
        if (valid) {
            q = qv;
        } else {
#pragma unroll
            for (int nt = 0; nt < 8; ++nt) dz[nt] = z[nt] = f4{0.f, 0.f, 0.f, 0.f};
        }
    }
    float dot = 0.f;
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
        const f4 s = ld4u(a.scale + 16 * nt + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) dot += s[r] * dz[nt][r] * z[nt][r];
    }
    dot += __shfl_xor(dot, 16);
    dot += __shfl_xor(dot, 32);
    const float rms = q - RMS_EPS;
    const float coef = rms > 0.f ? dot / (q * q * rms) * (a.dinv * a.dinv) : 0.f;
    // scale partials: Σ over the wave's 16 rows (the lanes of one g) of dY ⊙ z / q, into LDS; the
    // even wave of each pair adds its odd neighbour's behind the barrier (32 rows per partial)
#if MGN_F32C_DPPRED
    // transposing DPP row sums (6 DPP adds for the 4 components instead of 16 LDS-crossbar shuffles):
    // lane ri < 4 ends with component 2(ri&1) + ((ri>>1)&1) summed over the row
    const int r4 = 2 * (ri & 1) + ((ri >> 1) & 1);
#endif
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
        const f4 s = ld4u(a.scale + 16 * nt + 4 * g);
        f4 dsc;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float dy = dz[nt][r];
            float v = dy * (z[nt][r] / q);
#if !MGN_F32C_DPPRED
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
#endif
            dsc[r] = v;
            dz[nt][r] = s[r] * dy / q - z[nt][r] * coef;
        }
#if MGN_F32C_DPPRED
        const float dsum = f32c_row16_sum4(dsc, ri);
        if (ri < 4) red[wave * H + 16 * nt + 4 * g + r4] = dsum;
#else
        if (ri == 0) *reinterpret_cast<f4*>(red + wave * H + 16 * nt + 4 * g) = dsc;
#endif
    }
    if (MGN_F32C_FLOW && threadIdx.x < 8) flg[threadIdx.x] = 0u;
    f32c_stage_wait();
    __syncthreads();
    F32C_STAMP(0);
    float* dz8 = reinterpret_cast<float*>(a.dz8);
    const int64_t r8 = f32c_r8t(row, g);  // transposed R8 saves
    if (!(wave & 1) && ri == 0) {
        const int64_t p = (int64_t)blockIdx.x * (F32C_WAVES / 2) + (wave >> 1);
        if (p < a.RP / 32) {
#pragma unroll
            for (int nt = 0; nt < 8; ++nt) {
                const int n = 16 * nt + 4 * g;
                *reinterpret_cast<f4*>(a.dscale_part + p * H + n) =
                    *reinterpret_cast<const f4*>(red + wave * H + n) + *reinterpret_cast<const f4*>(red + (wave + 1) * H + n);
            }
        }
    }
    // ---- layers 3..1: dZ_{l-1} = (dZ_l · W_l) ⊙ [A_{l-1} > 0]; then de_in = dout + dZ_0 · W0a
    f4 acc[8], dv[8];
    const float* dout = reinterpret_cast<const float*>(a.dout);
    // MGN_F32C_FLOW: the transposed image of step j (layer 3 - j)
    auto bimg = [&](int j) { return wt + off[3 - j] + chain_image_off(H, j == 3 ? a.Kpack0 : H); };
    bool loader = false;
#pragma unroll 1
    for (int i = 0; i < 4; ++i) {
        const int l = 3 - i;  // layer whose transposed weights this GEMM uses
        const float* nxt = nullptr;
        if (MGN_F32C_FLOW) {
            if (i == 0) f32c_stage(bimg(1), img1);  // every wave's share
            if (i >= 1) f32c_wait(flg + 4 + i, i == 1 ? F32C_WAVES : 1u);
        } else if (i < 3) {
            nxt = wt + off[l - 1] + chain_image_off(H, l == 1 ? a.Kpack0 : H);
            if (F32C_NBUF == 2) f32c_stage(nxt, (i & 1) ? img0 : img1);
        }
        if (i == 3) {
            // de_in = dout + dZ_0·W0a: dout lands during the last GEMM
#pragma unroll
            for (int nt = 0; nt < 8; ++nt)
                dv[nt] = valid ? *reinterpret_cast<const f4*>(dout + row * a.dout_ld + 16 * nt + 4 * g) : f4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) acc[nt] = f4{0.f, 0.f, 0.f, 0.f};
        // dZ_l's R8 save is stored while it feeds the MFMAs
        f32c_gemm(acc, dz, (i & 1) ? img1 : img0, lane, live ? dz8 + (int64_t)l * a.RP * H + r8 : nullptr);
        F32C_STAMP(1);
        if (i == 3) break;
        if (MGN_F32C_FLOW) {  // as the forward: the last wave out of this image stages step i+2's into it
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            unsigned old = 0;
            if (lane == 0) old = __hip_atomic_fetch_add(flg + i, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            old = __builtin_amdgcn_readfirstlane(old);
            loader = i + 2 <= 3 && old == F32C_WAVES - 1;
            if (loader) {
                const float* src = bimg(i + 2);
                float* img = (i & 1) ? img1 : img0;
                for (int c = 0; c < F32C_LAYER / 256; ++c) glds16(src + c * 256 + lane * 4, img + c * 256);
            }
        }
        // ReLU masks of hidden layer l-1: word nt*4 + r of the tile, bit = lane
        const unsigned long long mine = l == 3 ? mw[2] : l == 2 ? mw[1] : mw[0];
#pragma unroll
        for (int nt = 0; nt < 8; ++nt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const unsigned long long wd = ((unsigned long long)__builtin_amdgcn_readlane((int)(mine >> 32), nt * 4 + r) << 32) |
                                              (unsigned)__builtin_amdgcn_readlane((int)mine, nt * 4 + r);
                dz[nt][r] = ((wd >> lane) & 1ull) && valid ? acc[nt][r] : 0.f;
            }
        F32C_STAMP(2);
        if (MGN_F32C_FLOW) {
            f32c_stage_wait();
            asm volatile("" ::: "memory");
            if (lane == 0) {
                if (i == 0) __hip_atomic_fetch_add(flg + 5, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (loader) __hip_atomic_store(flg + 4 + i + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        } else {
            if (F32C_NBUF == 1) {
                __syncthreads();
                f32c_stage(nxt, img0);
            }
            f32c_stage_wait();
            __syncthreads();
        }
        F32C_STAMP(3);
    }
    if (valid) {
        // dZ_0 row-major for the node side (d(x·W0bᵀ)[v] = Σ_{dst(k)=v} dZ_0[k], likewise src), de_in
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) {
            const int n = 16 * nt + 4 * g;
            st4(reinterpret_cast<float*>(a.o2) + row * H + n, dz[nt]);
            st4(reinterpret_cast<float*>(a.o1) + row * H + n, dv[nt] + acc[nt]);
        }
    }
    F32C_STAMP(4);
    F32C_STAMP_PRINT("f32b");
}

// --------------------------------------------------------------------------- fp32 node MLP, register-chained
// The fp32 GraphNetBlock node MLP at h = 128 (round 5; reference layers.py:660-665, 694-699, 733-746:
// [x ‖ Σ_in-edges m] -> 4 Linears -> RMSNorm, + x): the edge MLP's fp32 chain (f32c_gemm: each wave owns
// 16 rows through all layers, activations never leave registers, the C layout of layer l is the B
// operand of layer l+1) with ONE wave per SIMD — N is ≈ E/5.8, so the edge kernels' 12-wave workgroups
// would fill a third of the chip, and a wave alone on its SIMD keeps the MFMA pipe fed from 8
// independent accumulators. The aggregation of the in-edges' messages s_e ⊙ z_k / q_k (target-sorted
// segments, edge order: the reference scatter_add's order, the generic kernel's expression, so the
// aggregates are bit-identical to it) lands straight in the B operand of layer 0's aggregate block.
// Layer 0 is two chain images (x block, aggr block of W0 [H x 2H]) and layers 1..3 one each: five
// images through the two LDS buffers by LDS-DMA, each staged under the previous one's MFMAs. Saves as
// the generic node kernel (the fp32 ring's node jobs read them): aggregate rows, R8 inputs of layers
// 1..3, ReLU ballot words, z and rden. The backward mirrors it: RMSNorm backward, layers 3..1, then
// dx_part = dx' + dZ0·W0[:, :H] and d_aggr = dZ0·W0[:, H:] from the two transposed images of W0.
#ifndef MGN_F32N_CHAIN
#define MGN_F32N_CHAIN 1  // 0: the fp32 node MLP on the generic LDS-tiled kernels (A/B builds)
#endif
#ifndef MGN_F32N_AG
#define MGN_F32N_AG 4  // in-edges gathered per round trip by the fp32 aggregation
#endif
#ifndef MGN_F32N_PROJ
#define MGN_F32N_PROJ 1  // the chained fp32 node MLP computes the next block's projections (A/B builds: 0)
#endif
constexpr int F32N_WAVES = 4;  // one wave per SIMD, 64 rows per workgroup
#define F32N_BOUNDS __launch_bounds__(F32N_WAVES * 64, 1)
constexpr size_t F32N_LDS_FWD = (2 * F32C_LAYER + 5 * 128) * sizeof(float);
constexpr size_t F32N_LDS_BWD = (2 * F32C_LAYER + F32N_WAVES * 128) * sizeof(float);

// this wave's share of one 64 KiB chain image copy global -> LDS (1 KiB per LDS-DMA instruction)
__device__ __forceinline__ void f32n_stage(const float* __restrict__ src, float* img) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int c = wave; c < F32C_LAYER / 256; c += F32N_WAVES)
        glds16(src + c * 256 + lane * 4, img + c * 256);
}

// ReLU of a hidden layer's accumulators into the next B operand + the tile's 32 ballot words (word
// nt*4 + r from lane nt*4 + r: the generic kernels' mask layout at h = 128), as the fp32 edge forward
__device__ __forceinline__ unsigned long long f32c_relu(f4 (&x)[8], const f4 (&acc)[8], int lane) {
    unsigned long long word = 0;
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float v = fmaxf(acc[nt][r], 0.f);
            x[nt][r] = v;
            const unsigned long long bits = __ballot(v > 0.f);
            if (lane == nt * 4 + r) word = bits;
        }
    }
    return word;
}

__global__ F32N_BOUNDS void node_fwd_f32_chain_kernel(FwdArgs a) {
    constexpr int H = 128;
    constexpr int AG = MGN_F32N_AG;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* const img0 = reinterpret_cast<float*>(smem);
    float* const img1 = img0 + F32C_LAYER;
    float* const vec = img1 + F32C_LAYER;  // [5][H]: b0..b3, RMSNorm scale
    const int lane = threadIdx.x & 63, g = lane >> 4, ri = lane & 15;
    const int64_t tile = (int64_t)blockIdx.x * F32N_WAVES + (threadIdx.x >> 6);
    const int64_t row = tile * 16 + ri;
    const bool valid = row < a.M;
    F32C_STAMP_DECL;
    const float* pk = reinterpret_cast<const float*>(a.wpack);
    // layer 0's two images land during phase A
    f32n_stage(pk + chain_image_off(H, 2 * H, 0), img0);
    f32n_stage(pk + chain_image_off(H, 2 * H, 1), img1);
    pk += linear_pack_elems(H, 2 * H, MGN_F32);
    for (int i = threadIdx.x; i < 5 * H; i += F32N_WAVES * 64) {
        const int vl = i >> 7;
        const float* vp = vl == 0 ? a.bias[0] : vl == 1 ? a.bias[1] : vl == 2 ? a.bias[2] : vl == 3 ? a.bias[3] : a.scale;
        vec[i] = vp[i & (H - 1)];
    }
    // phase A: x rows (layer 0's x-block operand and the residual) and the aggregate (its aggr block)
    const int64_t rowc = valid ? row : a.M - 1;
    const float* x = reinterpret_cast<const float*>(a.seg[0].p);
    f4 xr[8], ag[8], sc[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        xr[t] = *reinterpret_cast<const f4*>(x + rowc * a.seg[0].ld + 16 * t + 4 * g);
        sc[t] = ld4u(a.agg_scale + 16 * t + 4 * g);
        ag[t] = f4{0.f, 0.f, 0.f, 0.f};
    }
    {
        const int kb = a.seg_ptr[rowc], ke = valid ? a.seg_ptr[rowc + 1] : kb;
        const float* z = reinterpret_cast<const float*>(a.agg_z);
#pragma unroll 1
        for (int k = kb; k < ke; k += AG) {  // every load of a group before its first add
            f4 zz[AG][8];
            float qq[AG];
#pragma unroll
            for (int u = 0; u < AG; ++u) {
                const int64_t ku = k + u < ke ? k + u : ke - 1;
#pragma unroll
                for (int t = 0; t < 8; ++t) zz[u][t] = *reinterpret_cast<const f4*>(z + ku * H + 16 * t + 4 * g);
                qq[u] = a.agg_rden[ku];
            }
#pragma unroll
            for (int u = 0; u < AG; ++u) {
                if (k + u >= ke) break;
#pragma unroll
                for (int t = 0; t < 8; ++t)
#pragma unroll
                    for (int r = 0; r < 4; ++r) ag[t][r] += sc[t][r] * (zz[u][t][r] / qq[u]);
            }
        }
    }
    if (!valid) {
#pragma unroll
        for (int t = 0; t < 8; ++t) xr[t] = f4{0.f, 0.f, 0.f, 0.f};
    } else {
#pragma unroll
        for (int t = 0; t < 8; ++t) st4(reinterpret_cast<float*>(a.agg_save) + row * H + 16 * t + 4 * g, ag[t]);
    }
    F32C_STAMP(5);  // phase A issued and consumed (x rows, aggregation)
    f32c_stage_wait();
    __syncthreads();
    F32C_STAMP(0);
    f4 acc[8], x1[8];
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) acc[nt] = *reinterpret_cast<const f4*>(vec + 16 * nt + 4 * g);
    f32c_gemm(acc, xr, img0, lane);  // x block
    __syncthreads();                 // every wave is done with img0
    const float* nxt = pk + chain_image_off(H, H);
    f32n_stage(nxt, img0);           // layer 1's image streams in under the aggregate block
    pk += linear_pack_elems(H, H, MGN_F32);
    f32c_gemm(acc, ag, img1, lane);  // aggr block
    F32C_STAMP(1);
    float* act = reinterpret_cast<float*>(a.act8);
    const int64_t r8 = f32c_r8t(row, g);  // transposed R8 saves
    unsigned long long word = f32c_relu(x1, acc, lane);
    if (lane < 32) a.mask[tile * 32 + lane] = word;
    F32C_STAMP(2);
    f32c_stage_wait();
    __syncthreads();
    F32C_STAMP(3);
    // layers 1..3 (layer l on buffer (l + 1) & 1): layer l+1's image streams into the other buffer
#pragma unroll 1
    for (int l = 1; l < 4; ++l) {
        float* cur = (l & 1) ? img0 : img1;
        if (l < 3) {
            f32n_stage(pk + chain_image_off(H, H), (l & 1) ? img1 : img0);
            pk += linear_pack_elems(H, H, MGN_F32);
        }
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) acc[nt] = *reinterpret_cast<const f4*>(vec + l * H + 16 * nt + 4 * g);
        float* sv = l == 1 ? act + a.act_off[1] : l == 2 ? act + a.act_off[2] : act + a.act_off[3];
        if (l == 3 && a.pn_pack)  // the next block's W0b image streams in under the last layer
            f32n_stage(a.pn_pack + chain_image_off(H, 3 * H, 1), img1);
        f32c_gemm(acc, x1, cur, lane, sv + r8);  // its input's R8 save, under the MFMAs
        F32C_STAMP(1);
        if (l < 3) {
            word = f32c_relu(x1, acc, lane);
            if (lane < 32) a.mask[(int64_t)l * a.mask_stride + tile * 32 + lane] = word;
            F32C_STAMP(2);
            f32c_stage_wait();
            __syncthreads();
            F32C_STAMP(3);
        }
    }
    // last Linear (bias in the accumulator): RMSNorm, residual x
    float ss = 0.f;
#pragma unroll
    for (int nt = 0; nt < 8; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) ss += acc[nt][r] * acc[nt][r];
    ss += __shfl_xor(ss, 16);
    ss += __shfl_xor(ss, 32);
    {
        const float q = sqrtf(ss) * a.dinv + RMS_EPS;
        if (valid && g == 0) a.rden_save[row] = q;
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) {
            const int n = 16 * nt + 4 * g;
            const f4 s = *reinterpret_cast<const f4*>(vec + 4 * H + n);
            f4 y;
#pragma unroll
            for (int r = 0; r < 4; ++r) y[r] = s[r] * (acc[nt][r] / q);
            y = xr[nt] + y;
            if (valid) {
                st4(reinterpret_cast<float*>(a.z_save) + row * H + n, acc[nt]);
                st4(reinterpret_cast<float*>(a.out) + row * a.out_ld + n, y);
            }
            x1[nt] = valid ? y : f4{0.f, 0.f, 0.f, 0.f};  // x_out: the projections' B operand
        }
    }
    if (!a.pn_pack) return;
    // the NEXT block's node projections from x_out (reference layers.py:689-690,717 applied per node:
    // [e ‖ x_i ‖ x_j]·W0ᵀ = e·W0aᵀ + (x·W0bᵀ)[dst] + (x·W0cᵀ)[src]), W0b from img1, W0c from img0
    f32c_stage_wait();
    __syncthreads();  // W0b landed; every wave is done with img0 (layer 3)
    f32n_stage(a.pn_pack + chain_image_off(H, 3 * H, 2), img0);
#pragma unroll 1
    for (int half = 0; half < 2; ++half) {
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) acc[nt] = f4{0.f, 0.f, 0.f, 0.f};
        f32c_gemm(acc, x1, half ? img0 : img1, lane);
        if (valid) {
#pragma unroll
            for (int nt = 0; nt < 8; ++nt) st4(a.pn_out + row * (2 * H) + half * H + 16 * nt + 4 * g, acc[nt]);
        }
        if (half == 0) {
            f32c_stage_wait();
            __syncthreads();
        }
    }
    F32C_STAMP(4);
    F32C_STAMP_PRINT("f32nf");
}

// Split form (round 6, MGN_F32N_SPLIT): the same node MLP with TWO waves per 16-row tile — wave 2p + h owns
// output features 64h .. 64h + 63 (n-tiles 4h .. 4h + 3) of every layer — so a workgroup runs 8 waves
// (two per SIMD) on the same 64 rows, and one wave's aggregation gathers, LDS waits and barrier slack
// overlap the other's MFMAs (the one-wave-per-SIMD form above ran its MFMA pipe 31 % busy). The halves
// meet in LDS: each layer's ReLU output (the next layer's B operand) and the last layer's accumulators
// are exchanged between the two waves of a tile. Per accumulator the same MFMAs in the same k order, the
// aggregate's terms per feature in the same edge order, the RMSNorm sum in the same order: the results
// are bit-identical to the one-wave form. LDS: the two 64 KiB images + 4 KiB of exchange per wave (the
// biases and scales come from L2, a layer ahead).
#ifndef MGN_F32N_SPLIT
#define MGN_F32N_SPLIT 1
#endif
constexpr int F32S_WAVES = 8;
#define F32S_BOUNDS __launch_bounds__(F32S_WAVES * 64, 2)
constexpr size_t F32S_LDS_FWD = 2 * F32C_LAYER * sizeof(float) + (size_t)F32S_WAVES * 4 * 64 * sizeof(f4);
static_assert(F32S_LDS_FWD <= 160 * 1024, "split fp32 node forward: LDS");

__device__ __forceinline__ void f32s_stage(const float* __restrict__ src, float* img) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int c = wave; c < F32C_LAYER / 256; c += F32S_WAVES) glds16(src + c * 256 + lane * 4, img + c * 256);
}

// acc[j] += n-tile 4nh + j of X·Wᵀ (all 32 k-steps, f32c_gemm's k order); save: the k-groups t of this
// wave's half of the input's R8 save (the partner stores the other half)
template <int nh>
__device__ __forceinline__ void f32s_gemm(f4 (&acc)[4], const f4 (&x)[8], const float* img, int lane,
                                          float* save = nullptr) {
    f4 w[2][4];
    const f4* ip = reinterpret_cast<const f4*>(img) + lane;
#pragma unroll
    for (int j = 0; j < 4; ++j) w[0][j] = ip[((4 * nh + j) * 8 + 0) * 64];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        if (t + 1 < 8) {
#pragma unroll
            for (int j = 0; j < 4; ++j) w[(t + 1) & 1][j] = ip[((4 * nh + j) * 8 + t + 1) * 64];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[t & 1][j][r], x[t][r], acc[j], 0, 0, 0);
        if (save && (t >> 2) == nh) *reinterpret_cast<f4*>(save + 128 * t) = quad_transpose(x[t], lane);
    }
}

// the half is a template parameter: register arrays indexed by it stay statically indexed (a run-time
// half made the compiler move them with indexed register moves: 4x slower)
template <int nh>
__device__ __forceinline__ void node_fwd_f32_split_body(const FwdArgs& a) {
    constexpr int H = 128;
    constexpr int AG = MGN_F32N_AG;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* const img0 = reinterpret_cast<float*>(smem);
    float* const img1 = img0 + F32C_LAYER;
    f4* const xch = reinterpret_cast<f4*>(img1 + F32C_LAYER);  // [wave][4][64]
    const int lane = threadIdx.x & 63, g = lane >> 4, ri = lane & 15, wave = threadIdx.x >> 6;
    f4* const mine = xch + (size_t)wave * 256 + lane;
    const f4* const theirs = xch + (size_t)(wave ^ 1) * 256 + lane;
    const int64_t tile = (int64_t)blockIdx.x * (F32S_WAVES / 2) + (wave >> 1);
    const int64_t row = tile * 16 + ri;
    const bool valid = row < a.M;
    const float* pk = reinterpret_cast<const float*>(a.wpack);
    f32s_stage(pk + chain_image_off(H, 2 * H, 0), img0);
    f32s_stage(pk + chain_image_off(H, 2 * H, 1), img1);
    pk += linear_pack_elems(H, 2 * H, MGN_F32);
    // layer 0's bias half, then each next layer's one layer ahead
    f4 bias[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bias[j] = ld4u(a.bias[0] + 16 * (4 * nh + j) + 4 * g);
    // phase A: x rows (whole: layer 0's x-block operand and the residual), this wave's half of the aggregate
    const int64_t rowc = valid ? row : a.M - 1;
    const float* x = reinterpret_cast<const float*>(a.seg[0].p);
    f4 xr[8], ag[8], sc[4];
#pragma unroll
    for (int t = 0; t < 8; ++t) xr[t] = *reinterpret_cast<const f4*>(x + rowc * a.seg[0].ld + 16 * t + 4 * g);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        sc[j] = ld4u(a.agg_scale + 16 * (4 * nh + j) + 4 * g);
        ag[4 * nh + j] = f4{0.f, 0.f, 0.f, 0.f};
    }
    {
        const int kb = a.seg_ptr[rowc], ke = valid ? a.seg_ptr[rowc + 1] : kb;
        const float* z = reinterpret_cast<const float*>(a.agg_z);
#pragma unroll 1
        for (int k = kb; k < ke; k += AG) {
            f4 zz[AG][4];
            float qq[AG];
#pragma unroll
            for (int u = 0; u < AG; ++u) {
                const int64_t ku = k + u < ke ? k + u : ke - 1;
#pragma unroll
                for (int j = 0; j < 4; ++j) zz[u][j] = *reinterpret_cast<const f4*>(z + ku * H + 16 * (4 * nh + j) + 4 * g);
                qq[u] = a.agg_rden[ku];
            }
#pragma unroll
            for (int u = 0; u < AG; ++u) {
                if (k + u >= ke) break;
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) ag[4 * nh + j][r] += sc[j][r] * (zz[u][j][r] / qq[u]);
            }
        }
    }
    if (!valid) {
#pragma unroll
        for (int t = 0; t < 8; ++t) xr[t] = f4{0.f, 0.f, 0.f, 0.f};
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            st4(reinterpret_cast<float*>(a.agg_save) + row * H + 16 * (4 * nh + j) + 4 * g, ag[4 * nh + j]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) mine[64 * j] = ag[4 * nh + j];
    f32c_stage_wait();
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) ag[4 * (1 - nh) + j] = theirs[64 * j];
    f4 acc[4], x1[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = bias[j];
#pragma unroll
    for (int j = 0; j < 4; ++j) bias[j] = ld4u(a.bias[1] + 16 * (4 * nh + j) + 4 * g);
    f32s_gemm<nh>(acc, xr, img0, lane);  // x block
    __syncthreads();                     // every wave is done with img0 (and has read its partner's aggregate)
    f32s_stage(pk + chain_image_off(H, H), img0);
    pk += linear_pack_elems(H, H, MGN_F32);
    f32s_gemm<nh>(acc, ag, img1, lane);  // aggr block
    float* act = reinterpret_cast<float*>(a.act8);
    const int64_t r8 = f32c_r8t(row, g);
    // ReLU of this wave's half -> the exchange; ballot words nt*4 + r (nt = 4nh + j) from lane nt*4 + r
    auto relu_half = [&](int l) {
        unsigned long long word = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float v = fmaxf(acc[j][r], 0.f);
                x1[4 * nh + j][r] = v;
                const unsigned long long bits = __ballot(v > 0.f);
                if (lane == (4 * nh + j) * 4 + r) word = bits;
            }
            mine[64 * j] = x1[4 * nh + j];
        }
        if ((lane >> 4) == nh && lane < 32) a.mask[(int64_t)l * a.mask_stride + tile * 32 + lane] = word;
    };
    relu_half(0);
    f32c_stage_wait();
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) x1[4 * (1 - nh) + j] = theirs[64 * j];
    __syncthreads();  // the partner's half is read before either wave writes the exchange again
#pragma unroll 1
    for (int l = 1; l < 4; ++l) {
        float* cur = (l & 1) ? img0 : img1;
        if (l < 3) {
            f32s_stage(pk + chain_image_off(H, H), (l & 1) ? img1 : img0);
            pk += linear_pack_elems(H, H, MGN_F32);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = bias[j];
        const float* bn = l == 1 ? a.bias[2] : a.bias[3];
        if (l < 3) {
#pragma unroll
            for (int j = 0; j < 4; ++j) bias[j] = ld4u(bn + 16 * (4 * nh + j) + 4 * g);
        }
        float* sv = l == 1 ? act + a.act_off[1] : l == 2 ? act + a.act_off[2] : act + a.act_off[3];
        if (l == 3 && a.pn_pack) f32s_stage(a.pn_pack + chain_image_off(H, 3 * H, 1), img1);
        f32s_gemm<nh>(acc, x1, cur, lane, sv + r8);
        if (l < 3) {
            relu_half(l);
            f32c_stage_wait();
            __syncthreads();
#pragma unroll
            for (int j = 0; j < 4; ++j) x1[4 * (1 - nh) + j] = theirs[64 * j];
            __syncthreads();
        }
    }
    // last Linear: the two halves of the accumulators meet, RMSNorm in the one-wave form's order
#pragma unroll
    for (int j = 0; j < 4; ++j) mine[64 * j] = acc[j];
    __syncthreads();
    f4 full[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        full[4 * nh + j] = acc[j];
        full[4 * (1 - nh) + j] = theirs[64 * j];
    }
    float ss = 0.f;
#pragma unroll
    for (int nt = 0; nt < 8; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) ss += full[nt][r] * full[nt][r];
    ss += __shfl_xor(ss, 16);
    ss += __shfl_xor(ss, 32);
    {
        const float q = sqrtf(ss) * a.dinv + RMS_EPS;
        if (valid && g == 0 && nh == 0) a.rden_save[row] = q;
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) {
            const int n = 16 * nt + 4 * g;
            const f4 s = ld4u(a.scale + n);
            f4 y;
#pragma unroll
            for (int r = 0; r < 4; ++r) y[r] = s[r] * (full[nt][r] / q);
            y = xr[nt] + y;
            if (valid && (nt >> 2) == nh) {
                st4(reinterpret_cast<float*>(a.z_save) + row * H + n, full[nt]);
                st4(reinterpret_cast<float*>(a.out) + row * a.out_ld + n, y);
            }
            x1[nt] = valid ? y : f4{0.f, 0.f, 0.f, 0.f};  // x_out: the projections' B operand
        }
    }
    if (!a.pn_pack) return;
    // the NEXT block's node projections from x_out, this wave's half of each ([x·W0bᵀ ‖ x·W0cᵀ])
    f32c_stage_wait();
    __syncthreads();  // W0b landed; every wave is done with img0 (layer 3)
    f32s_stage(a.pn_pack + chain_image_off(H, 3 * H, 2), img0);
#pragma unroll 1
    for (int half = 0; half < 2; ++half) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = f4{0.f, 0.f, 0.f, 0.f};
        f32s_gemm<nh>(acc, x1, half ? img0 : img1, lane);
        if (valid) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                st4(a.pn_out + row * (2 * H) + half * H + 16 * (4 * nh + j) + 4 * g, acc[j]);
        }
        if (half == 0) {
            f32c_stage_wait();
            __syncthreads();
        }
    }
}

__global__ F32S_BOUNDS void node_fwd_f32_split_kernel(FwdArgs a) {
    if ((threadIdx.x >> 6) & 1)  // wave-uniform: both bodies pass the same barriers
        node_fwd_f32_split_body<1>(a);
    else
        node_fwd_f32_split_body<0>(a);
}

__global__ F32N_BOUNDS void node_bwd_f32_chain_kernel(BwdArgs a) {
    constexpr int H = 128;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* const img0 = reinterpret_cast<float*>(smem);
    float* const img1 = img0 + F32C_LAYER;
    float* const red = img1 + F32C_LAYER;  // [F32N_WAVES][H] per-wave RMSNorm-scale partials
    const int lane = threadIdx.x & 63, g = lane >> 4, ri = lane & 15, wave = threadIdx.x >> 6;
    const int64_t tile = (int64_t)blockIdx.x * F32N_WAVES + wave;
    const int64_t row = tile * 16 + ri;
    const bool valid = row < a.M;
    F32C_STAMP_DECL;
    const float* wt = reinterpret_cast<const float*>(a.wtpack);
    const int64_t off1 = linear_pack_elems(H, 2 * H, MGN_F32);       // transposed pack offsets
    const int64_t off2 = off1 + linear_pack_elems(H, H, MGN_F32), off3 = off2 + linear_pack_elems(H, H, MGN_F32);
    f32n_stage(wt + off3 + chain_image_off(H, H), img0);  // W3ᵀ, then W2ᵀ: both buffers
    f32n_stage(wt + off2 + chain_image_off(H, H), img1);
    unsigned long long mw[3] = {0ull, 0ull, 0ull};
    if (lane < 32) {
#pragma unroll
        for (int l = 0; l < 3; ++l) mw[l] = a.mask[(int64_t)l * a.mask_stride + tile * 32 + lane];
    }
    // ---- dY = dx_out -> dZ3 (RMSNorm backward), as the fp32 edge backward
    f4 dz[8], z[8], dv[8];
    float q = 1.f;
    {
        const int64_t rowc = valid ? row : a.M - 1;
        const float* dout = reinterpret_cast<const float*>(a.dout);
        const float* zs = reinterpret_cast<const float*>(a.z_save);
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) {
            const int n = 16 * nt + 4 * g;
            dz[nt] = *reinterpret_cast<const f4*>(dout + rowc * a.dout_ld + n);
            z[nt] = *reinterpret_cast<const f4*>(zs + rowc * H + n);
        }
        const float qv = a.rden_save[rowc];
        if (valid) {
            q = qv;
        } else {
#pragma unroll
            for (int nt = 0; nt < 8; ++nt) dz[nt] = z[nt] = f4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) dv[nt] = dz[nt];  // dx_part = dx_out + dA0[:, :H]
    }
    float dot = 0.f;
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
        const f4 s = ld4u(a.scale + 16 * nt + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) dot += s[r] * dz[nt][r] * z[nt][r];
    }
    dot += __shfl_xor(dot, 16);
    dot += __shfl_xor(dot, 32);
    const float rms = q - RMS_EPS;
    const float coef = rms > 0.f ? dot / (q * q * rms) * (a.dinv * a.dinv) : 0.f;
    const int r4 = 2 * (ri & 1) + ((ri >> 1) & 1);
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
        const f4 s = ld4u(a.scale + 16 * nt + 4 * g);
        f4 dsc;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float dy = dz[nt][r];
            dsc[r] = dy * (z[nt][r] / q);
            dz[nt][r] = s[r] * dy / q - z[nt][r] * coef;
        }
        const float dsum = f32c_row16_sum4(dsc, ri);
        if (ri < 4) red[wave * H + 16 * nt + 4 * g + r4] = dsum;
    }
    F32C_STAMP(5);
    f32c_stage_wait();
    __syncthreads();
    F32C_STAMP(0);
    float* dz8 = reinterpret_cast<float*>(a.dz8);
    const int64_t r8 = f32c_r8t(row, g);
    if (!(wave & 1) && ri == 0) {  // partials per 32 rows (the generic node kernel's count)
        const int64_t p = (int64_t)blockIdx.x * (F32N_WAVES / 2) + (wave >> 1);
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) {
            const int n = 16 * nt + 4 * g;
            *reinterpret_cast<f4*>(a.dscale_part + p * H + n) =
                *reinterpret_cast<const f4*>(red + wave * H + n) + *reinterpret_cast<const f4*>(red + (wave + 1) * H + n);
        }
    }
    // ---- layers 3..1 (images W3ᵀ img0, W2ᵀ img1, W1ᵀ img0), then W0ᵀ's x block (img1), aggr block (img0)
    f4 acc[8];
#pragma unroll 1
    for (int i = 0; i < 5; ++i) {
        float* cur = (i & 1) ? img1 : img0;
        // the image after next streams into the buffer the previous step freed (barrier below)
        if (i >= 1 && i <= 3) {
            const float* src = i == 1 ? wt + off1 + chain_image_off(H, H)                  // W1ᵀ
                             : i == 2 ? wt + chain_image_off(H, 2 * H, 0)                  // W0ᵀ, x block
                                      : wt + chain_image_off(H, 2 * H, 1);                 // W0ᵀ, aggr block
            f32n_stage(src, (i & 1) ? img0 : img1);
        }
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) acc[nt] = f4{0.f, 0.f, 0.f, 0.f};
        const int l = 3 - i;  // dZ_l feeds this GEMM (i = 4: dZ0 again, the aggr block)
        float* sv = i < 4 ? dz8 + (int64_t)l * a.RP * H + r8 : nullptr;
        f32c_gemm(acc, dz, cur, lane, sv);
        F32C_STAMP(1);
        if (i < 3) {
            const unsigned long long mine = l == 3 ? mw[2] : l == 2 ? mw[1] : mw[0];
#pragma unroll
            for (int nt = 0; nt < 8; ++nt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const unsigned long long wd =
                        ((unsigned long long)__builtin_amdgcn_readlane((int)(mine >> 32), nt * 4 + r) << 32) |
                        (unsigned)__builtin_amdgcn_readlane((int)mine, nt * 4 + r);
                    dz[nt][r] = ((wd >> lane) & 1ull) && valid ? acc[nt][r] : 0.f;
                }
        } else if (i == 3 && valid) {
#pragma unroll
            for (int nt = 0; nt < 8; ++nt)
                st4(reinterpret_cast<float*>(a.o1) + row * H + 16 * nt + 4 * g, dv[nt] + acc[nt]);
        } else if (i == 4 && valid) {
#pragma unroll
            for (int nt = 0; nt < 8; ++nt) st4(reinterpret_cast<float*>(a.o2) + row * H + 16 * nt + 4 * g, acc[nt]);
        }
        F32C_STAMP(2);
        if (i < 4) {
            f32c_stage_wait();
            __syncthreads();
        }
        F32C_STAMP(3);
    }
    F32C_STAMP_PRINT("f32nb");
}

// --------------------------------------------------------------------------- host side
// Round 5 (small graphs): the generic bf16 kernels on 32-row edge / dense and 16-row
// node workgroups — twice / four times the workgroups of a small graph's launch, each a shorter chain
// (Cfg C at plate.json's sizes 1,032 -> 1,166 steps/s same box, `profiles/r05_ab.txt`; Cfg B's bf16
// generic launch, the decoder, measured neutral at 32 rows in round 2). fp32 keeps 32 / 32: the fp32
// node MLP's chained backward writes its RMSNorm-scale partials per 32 rows, and 16 rows bought Cfg A
// (fp32 h=32) only +0.9 %.
#ifndef MGN_BF16_BM
#define MGN_BF16_BM 32  // rows per workgroup of the generic bf16 dense / edge kernels (A/B builds: 64)
#endif
#ifndef MGN_F32_BM
#define MGN_F32_BM 32  // rows per workgroup of the generic fp32 dense / edge kernels (A/B builds: 64)
#endif
#ifndef MGN_NODE_BM16
#define MGN_NODE_BM16 16  // rows per workgroup of the generic bf16 node-MLP kernels (A/B builds: 32)
#endif
template <class T>
constexpr int bm_of() { return sizeof(T) == 4 ? MGN_F32_BM : MGN_BF16_BM; }
// rows per workgroup tile: node MLPs use 32 rows in fp32 and MGN_NODE_BM16 in bf16 (N is ~6x smaller than
// E: more, shorter workgroups)
template <class T, int MODE>
constexpr int bm_for() { return MODE == MODE_NODE ? (sizeof(T) == 4 ? 32 : MGN_NODE_BM16) : bm_of<T>(); }
int bm_host(int dtype, int mode) {
    return mode == MODE_NODE ? (dtype == MGN_F32 ? 32 : MGN_NODE_BM16) : dtype == MGN_F32 ? MGN_F32_BM : MGN_BF16_BM;
}

// Raise a kernel's dynamic-LDS limit once (not per launch: launches may be inside a graph capture).
int set_lds(const void* fn, size_t bytes) {
    if (bytes <= 65536) return 0;
    static std::mutex mu;
    static std::unordered_map<const void*, size_t> done;
    std::lock_guard<std::mutex> lk(mu);
    auto it = done.find(fn);
    if (it != done.end() && it->second >= bytes) return 0;
    MGN_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    done[fn] = bytes;
    return 0;
}

template <class T>
int pad_ld(int cols) {
    return cols + (int)(16 / sizeof(T));
}

int check_mlp(const mgn_mlp* m) {
    MGN_REQUIRE(m != nullptr, "mlp descriptor is NULL");
    MGN_REQUIRE(m->n_layers >= 2 && m->n_layers <= MGN_MAX_LAYERS,
                "The MLP must have at least 2 layers (input and output) and at most 8");
    MGN_REQUIRE(m->hidden == 16 || m->hidden == 32 || m->hidden == 64 || m->hidden == 128 || m->hidden == 256,
                "kernel width (mgn_mlp.hidden) must be 16, 32, 64, 128 or 256; a model of another hidden size "
                "<= 256 runs zero-padded to the next width with norm_dim = its true size");
    MGN_REQUIRE(m->norm_dim >= 0 && m->norm_dim <= m->out_dim, "norm_dim must be in [0, out_dim]");
    MGN_REQUIRE(m->in_dim >= 1, "in_dim must be >= 1");
    MGN_REQUIRE(m->out_dim == m->hidden || (m->out_dim >= 1 && m->out_dim <= 16),
                "out_dim must equal hidden or be in [1, 16]");
    MGN_REQUIRE(!m->has_norm || m->out_dim == m->hidden, "RMSNorm requires out_dim == hidden");
    MGN_REQUIRE(m->dtype == MGN_F32 || m->dtype == MGN_BF16, "dtype must be MGN_F32 or MGN_BF16");
    MGN_REQUIRE(m->wpack && m->wtpack, "packed weights missing");
    for (int l = 0; l < m->n_layers; ++l) MGN_REQUIRE(m->bias[l], "bias pointer missing");
    MGN_REQUIRE(!m->has_norm || m->scale, "RMSNorm scale pointer missing");
    return 0;
}

struct MlpIn {
    SrcSeg seg[3];
    int nseg;
    int K0;               // staged layer-0 columns (0: m->in_dim)
    const float* proj;    // EDGE: node projections (see FwdArgs)
    const int32_t* proj_i;
    const int32_t* proj_j;
    const float* pn_pack; // NODE, fp32 h=128: the next block's projections (FwdArgs), if the chained kernel runs
    float* pn_out;
    int* pn_done;         // set to 1 when they were computed
};

template <class T, int H, int MODE>
int launch_fwd(const mgn_mlp* m, const MlpIn& in, int64_t M, void* out, int out_dtype, int64_t out_ld,
               const void* resid, mgn_mlp_saved* sv, const mgn_topology* topo, const mgn_mlp* agg_mlp,
               const mgn_mlp_saved* agg_sv, void* agg_save, hipStream_t st) {
    constexpr int BM = bm_for<T, MODE>();
    FwdArgs a;
    memset(&a, 0, sizeof(a));
    for (int s = 0; s < in.nseg; ++s) a.seg[s] = in.seg[s];
    a.nseg = in.nseg;
    a.L = m->n_layers;
    a.K0 = in.K0 ? in.K0 : m->in_dim;
    a.Kpack0 = m->in_dim;
    a.kstride0 = cdiv(m->in_dim, Mf<T>::KSTEP);
    a.proj = in.proj;
    a.proj_i = in.proj_i;
    a.proj_j = in.proj_j;
    a.H = H;
    a.NOUT = m->out_dim;
    a.has_norm = m->has_norm;
    a.ldi = pad_ld<T>(rup(a.K0, Mf<T>::KSTEP));
    a.ldh = pad_ld<T>(rup(H, Mf<T>::KSTEP));
    a.M = M;
    a.wpack = m->wpack;
    for (int l = 0; l < m->n_layers; ++l) a.bias[l] = m->bias[l];
    a.scale = m->scale;
    a.dinv = norm_dinv(m);
    if (MODE == MODE_NODE) {
        a.seg_ptr = topo->col_ptr;
        a.agg_z = agg_sv->z;
        a.agg_rden = agg_sv->rden;
        a.agg_scale = agg_mlp->scale;
        a.agg_save = agg_save;
    }
    a.out = out;
    a.out_dtype = out_dtype;
    a.out_ld = out_ld;
    a.resid = resid;
    a.act8 = sv->act;
    for (int l = 0; l < m->n_layers; ++l) a.act_off[l] = act_off(*m, M, l, MODE != MODE_DENSE);
    a.mask = reinterpret_cast<unsigned long long*>(sv->mask);
    a.mask_stride = mask_words_per_layer(*m, M);
    a.z_save = sv->z;
    a.rden_save = sv->rden;
    a.ablate = ablate_mask();
    if constexpr (sizeof(T) == 4 && H == 128 && MODE == MODE_EDGE) {
        auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
        const SrcSeg& s0 = a.seg[0];
        if (MGN_F32_CHAIN && a.L == 4 && a.has_norm && a.NOUT == H && a.nseg == 1 && !s0.idx &&
            s0.dtype == MGN_F32 && s0.ncols == H && s0.coff == 0 && s0.ld % 4 == 0 && al16(s0.p) && a.K0 == H &&
            a.Kpack0 == 3 * H && a.proj && al16(a.proj) && (!a.resid || al16(a.resid)) && al16(a.z_save) &&
            al16(a.act8) && a.out_ld % 4 == 0 && ((uintptr_t)a.out & (out_dtype == MGN_F32 ? 15 : 7)) == 0 &&
            !a.ablate) {
            const int grid = (int)cdiv64(rows_pad(M), 16 * F32C_WAVES);
            if (grid == 0) return 0;
            const size_t lds = (F32C_NBUF * F32C_LAYER + 5 * H) * sizeof(float) + (MGN_F32C_FLOW ? 32 : 0);
            if (int e = set_lds((const void*)edge_fwd_f32_chain_kernel, lds)) return e;
            ProfScope ps(PROF_FWD_EDGE, st);
            hipLaunchKernelGGL(edge_fwd_f32_chain_kernel, dim3(grid), dim3(F32C_WAVES * 64), lds, st, a);
            MGN_LAUNCH_CHECK();
            return 0;
        }
    }
    if constexpr (sizeof(T) == 4 && H == 128 && MODE == MODE_NODE) {
        auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
        const SrcSeg& s0 = a.seg[0];
        if (MGN_F32N_CHAIN && a.L == 4 && a.has_norm && a.NOUT == H && a.nseg == 1 && !s0.idx && s0.dtype == MGN_F32 &&
            s0.ncols == H && s0.coff == 0 && s0.ld % 4 == 0 && al16(s0.p) && a.K0 == 2 * H && a.Kpack0 == 2 * H &&
            a.resid == s0.p && a.seg_ptr && a.agg_z && al16(a.agg_z) && a.agg_rden && a.agg_scale && a.agg_save &&
            al16(a.agg_save) && al16(a.z_save) && al16(a.act8) && out_dtype == MGN_F32 && a.out_ld % 4 == 0 &&
            al16(a.out) && !a.ablate) {
            const int grid = (int)(rows_pad(M) / (16 * F32N_WAVES));
            if (grid == 0) return 0;
            if (in.pn_pack && in.pn_out) {
                a.pn_pack = in.pn_pack;
                a.pn_out = in.pn_out;
                if (in.pn_done) *in.pn_done = 1;
            }
            if (MGN_F32N_SPLIT) {
                if (int e = set_lds((const void*)node_fwd_f32_split_kernel, F32S_LDS_FWD)) return e;
                ProfScope ps(PROF_FWD_NODE, st);
                hipLaunchKernelGGL(node_fwd_f32_split_kernel, dim3(grid), dim3(F32S_WAVES * 64), F32S_LDS_FWD, st, a);
                MGN_LAUNCH_CHECK();
                return 0;
            }
            if (int e = set_lds((const void*)node_fwd_f32_chain_kernel, F32N_LDS_FWD)) return e;
            ProfScope ps(PROF_FWD_NODE, st);
            hipLaunchKernelGGL(node_fwd_f32_chain_kernel, dim3(grid), dim3(F32N_WAVES * 64), F32N_LDS_FWD, st, a);
            MGN_LAUNCH_CHECK();
            return 0;
        }
    }
    size_t r0 = (size_t)BM * (a.ldi > a.ldh ? a.ldi : a.ldh) * sizeof(T);
    const size_t zb = m->has_norm ? (size_t)BM * (H + 4) * sizeof(float) : 0;
    if (zb > r0) r0 = zb;
    r0 = (r0 + 15) / 16 * 16;
    a.r0_elems = (int)(r0 / sizeof(T));
    size_t lds = r0 + (size_t)BM * a.ldh * sizeof(T) + 4 * BM * sizeof(float);
    // weights in LDS: the fragment prefix each layer's GEMM reads (layer 0 only when its k-steps are
    // contiguous: no split layer 0 reading the e block of a wider pack)
    bool wl = false;
    if (H <= 64 && a.kstride0 == rup(a.K0, Mf<T>::KSTEP) / Mf<T>::KSTEP && !a.ablate) {
        constexpr int FE = 64 * Mf<T>::VEC;  // elements per fragment
        int64_t src = 0, lo = 0;
        for (int l = 0; l < a.L; ++l) {
            int n, k;
            mlp_layer_shape(*m, l, &n, &k);
            const int ks = l == 0 ? a.kstride0 : cdiv(H, Mf<T>::KSTEP);
            const int nt = (l == a.L - 1 && a.NOUT != H) ? 1 : H / 16;
            a.wl.src[l] = src;
            a.wl.cnt[l] = nt * ks * FE;
            a.wl.lo[l] = (int32_t)lo;
            lo += a.wl.cnt[l];
            src += linear_pack_elems(n, k, dtype_id<T>());
        }
        a.wl.n = a.L;
        const size_t wb = (size_t)lo * sizeof(T);
        if (wb <= 48 * 1024) {
            lds = (lds + 15) / 16 * 16;
            a.wl_elems = (int32_t)(lds / sizeof(T));
            lds += wb;
            wl = true;
        } else {
            a.wl.n = 0;
        }
    }
    auto fn = wl ? mlp_fwd_kernel<T, H, BM, MODE, true> : mlp_fwd_kernel<T, H, BM, MODE, false>;
    if (int e = set_lds((const void*)fn, lds)) return e;
    const int grid = (int)(rows_pad(M) / BM);
    if (grid == 0) return 0;
    ProfScope ps(MODE == MODE_EDGE ? PROF_FWD_EDGE : MODE == MODE_NODE ? PROF_FWD_NODE : PROF_FWD_DENSE, st);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(MGN_THREADS), lds, st, a);
    MGN_LAUNCH_CHECK();
    return 0;
}

struct BwdOut {
    int mode;
    const void* gath;
    const int32_t* gath_idx;
    void* din;
    int din_dtype;
    int64_t din_ld;
    void* o1;
    void* o2;
};

template <class T, int H, int MODE>
int launch_bwd(const mgn_mlp* m, int64_t M, const mgn_mlp_saved* sv, const void* dout, int dout_dtype,
               int64_t dout_ld, const BwdOut& o, void* dz_save, float* dscale_part, hipStream_t st) {
    constexpr int BM = bm_for<T, MODE>();
    BwdArgs a;
    memset(&a, 0, sizeof(a));
    a.M = M;
    a.L = m->n_layers;
    a.K0 = MODE == MODE_EDGE ? H : m->in_dim;
    a.Kpack0 = m->in_dim;
    a.H = H;
    a.NOUT = m->out_dim;
    a.has_norm = m->has_norm;
    a.ldh = pad_ld<T>(rup(H, Mf<T>::KSTEP));
    a.mode = MODE;
    a.dinv = norm_dinv(m);
    a.wtpack = m->wtpack;
    a.scale = m->scale;
    a.mask = reinterpret_cast<const unsigned long long*>(sv->mask);
    a.mask_stride = mask_words_per_layer(*m, M);
    a.z_save = sv->z;
    a.rden_save = sv->rden;
    a.dout = dout;
    a.dout_dtype = dout_dtype;
    a.dout_ld = dout_ld;
    a.gath = o.gath;
    a.gath_idx = o.gath_idx;
    a.dz8 = dz_save;
    a.RP = rows_pad(M);
    a.dscale_part = dscale_part;
    a.din = o.din;
    a.din_dtype = o.din_dtype;
    a.din_ld = o.din_ld;
    a.o1 = o.o1;
    a.o2 = o.o2;
    if constexpr (sizeof(T) == 4 && H == 128 && MODE == MODE_EDGE) {
        auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
        if (MGN_F32_CHAIN && a.L == 4 && a.has_norm && a.NOUT == H && a.Kpack0 == 3 * H && a.dout_dtype == MGN_F32 &&
            a.dout_ld % 4 == 0 && al16(a.dout) && al16(a.gath) && a.gath_idx && al16(a.z_save) && al16(a.dz8) &&
            al16(a.o1) && al16(a.o2) && al16(a.dscale_part) && BM == 32) {
            const int grid = (int)cdiv64(a.RP, 16 * F32C_WAVES);
            if (grid == 0) return 0;
            const size_t lds = (F32C_NBUF * F32C_LAYER + F32C_WAVES * H) * sizeof(float) + (MGN_F32C_FLOW ? 32 : 0);
            if (int e = set_lds((const void*)edge_bwd_f32_chain_kernel, lds)) return e;
            ProfScope ps(PROF_BWD_EDGE, st);
            hipLaunchKernelGGL(edge_bwd_f32_chain_kernel, dim3(grid), dim3(F32C_WAVES * 64), lds, st, a);
            MGN_LAUNCH_CHECK();
            return 0;
        }
    }
    if constexpr (sizeof(T) == 4 && H == 128 && MODE == MODE_NODE) {
        auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
        if (MGN_F32N_CHAIN && a.L == 4 && a.has_norm && a.NOUT == H && a.Kpack0 == 2 * H && a.dout_dtype == MGN_F32 &&
            a.dout_ld % 4 == 0 && al16(a.dout) && al16(a.z_save) && al16(a.dz8) && al16(a.o1) && al16(a.o2) &&
            al16(a.dscale_part) && BM == 32 && !a.din) {
            const int grid = (int)(a.RP / (16 * F32N_WAVES));
            if (grid == 0) return 0;
            if (int e = set_lds((const void*)node_bwd_f32_chain_kernel, F32N_LDS_BWD)) return e;
            ProfScope ps(PROF_BWD_NODE, st);
            hipLaunchKernelGGL(node_bwd_f32_chain_kernel, dim3(grid), dim3(F32N_WAVES * 64), F32N_LDS_BWD, st, a);
            MGN_LAUNCH_CHECK();
            return 0;
        }
    }
    size_t lds = 2 * (size_t)BM * a.ldh * sizeof(T) + MGN_THREADS * 4 * sizeof(float);
    // weights in LDS (as launch_fwd): the transposed-fragment prefix each layer's GEMM reads
    bool wl = false;
    if (H <= 64) {
        constexpr int FE = 64 * Mf<T>::VEC;
        const int NO = a.NOUT;
        int64_t src = 0, lo = 0;
        const int nchunk = (MODE == MODE_DENSE && o.din == nullptr) ? 0 : cdiv(cdiv(a.K0, 16), H / 16);
        for (int l = 0; l < a.L; ++l) {
            int n, k;
            mlp_layer_shape(*m, l, &n, &k);
            const int Nl = l == a.L - 1 ? NO : H;
            a.wl.src[l] = src;
            a.wl.cnt[l] = l == 0 ? nchunk * (H / 16) * cdiv(a.L == 1 ? NO : H, Mf<T>::KSTEP) * FE
                                 : (H / 16) * cdiv(Nl, Mf<T>::KSTEP) * FE;
            a.wl.lo[l] = (int32_t)lo;
            lo += a.wl.cnt[l];
            src += linear_pack_elems(n, k, dtype_id<T>());
        }
        a.wl.n = a.L;
        const size_t wb = (size_t)lo * sizeof(T);
        if (wb <= 48 * 1024) {
            lds = (lds + 15) / 16 * 16;
            a.wl_elems = (int32_t)(lds / sizeof(T));
            lds += wb;
            wl = true;
        } else {
            a.wl.n = 0;
        }
    }
    auto fn = wl ? mlp_bwd_kernel<T, H, BM, MODE, true> : mlp_bwd_kernel<T, H, BM, MODE, false>;
    if (int e = set_lds((const void*)fn, lds)) return e;
    const int grid = (int)(rows_pad(M) / BM);
    if (grid == 0) return 0;
    ProfScope ps(MODE == MODE_EDGE ? PROF_BWD_EDGE : MODE == MODE_NODE ? PROF_BWD_NODE : PROF_BWD_DENSE, st);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(MGN_THREADS), lds, st, a);
    MGN_LAUNCH_CHECK();
    return 0;
}

// flat grad vector size (excluding RMSNorm scale)
int64_t grad_G(const mgn_mlp* m) {
    int64_t g = 0;
    for (int l = 0; l < m->n_layers; ++l) {
        int n, k;
        mlp_layer_shape(*m, l, &n, &k);
        g += (int64_t)n * k + n;
    }
    return g;
}

// rows per chunk: enough workgroups to fill the chip (~512), at most 64 partial slabs
// one 512-thread workgroup per CU fits (VGPRs + LDS), so chunks x jobs stays within one wave of
// workgroups over the CUs (a second, partial round doubles a short launch)
// Small hidden sizes (H <= 32: cylinder.json's h = 32): a chunk's slab is tiny (H x 3H floats) and
// one workgroup per CU leaves the kernel latency-bound (its fp32 path loads fragments straight from
// global memory), so those launches cut the rows into up to 4 x CUs chunks (several workgroups per
// CU) and up to 256 slabs per job.
int64_t wgrad_max_chunks(int64_t RP, int H = 128) {
    const int64_t cap = H <= 32 ? 256 : 64;
    int64_t c = RP / 64;
    if (c > cap) c = cap;
    return c < 1 ? 1 : c;
}
int wgrad_wgs_per_cu(int H) { return H <= 32 ? MGN_WG_PER_CU32 : 1; }
// Slabs of the recomputed edge weight gradients (chain16_edge_wgrad_recompute: one 8-wave workgroup
// per CU, layers 1..3 regions only): up to MGN_REW_CHUNKS (env, default MGN_REW_MAXCH) chunks of at
// least 256 rows. The bf16 h=128 slab buffers (keep_layout, mlp_bwd_ws) hold max(this, wgrad_max_chunks).
#ifndef MGN_REW_MAXCH
#define MGN_REW_MAXCH 256
#endif
int64_t rew_max_chunks(int64_t RP) {
    static const int64_t cap = [] {
        const char* v = getenv("MGN_REW_CHUNKS");
        const long c = v ? atol(v) : MGN_REW_MAXCH;
        return (int64_t)(c < 1 ? 1 : c > 1024 ? 1024 : c);
    }();
    int64_t c = RP / 256;
    if (c > cap) c = cap;
    return c < 1 ? 1 : c;
}
// Only an edge MLP of a chained bf16 h=128 block (layer-0 input [e ‖ x_i ‖ x_j] = 3h columns) can run
// the recompute, so only its slab capacity is raised (node MLPs never need it), and never
// beyond one slab per CU (the recompute launch runs at most wgrad_cus() chunks)
int64_t slab_chunks(int64_t RP, const mgn_mlp* m) {
    const int64_t c = wgrad_max_chunks(RP, m->hidden);
    if (m->hidden != 128 || m->dtype != MGN_BF16 || m->in_dim != 3 * m->hidden) return c;
    int64_t r = rew_max_chunks(RP);
    if (r > hw_cus()) r = hw_cus();
    return r > c ? r : c;
}
int wgrad_rows_per_chunk(int64_t RP, int njobs, int H = 128) {
    int64_t chunks = (int64_t)wgrad_wgs_per_cu(H) * wgrad_cus() / njobs;
    const int64_t cap = wgrad_max_chunks(RP, H);
    if (chunks > cap) chunks = cap;
    if (chunks < 1) chunks = 1;
    int64_t r = cdiv64(RP, chunks);
    r = cdiv64(r, 64) * 64;
    if (r < 64) r = 64;
    return (int)r;
}

RedDesc red_desc(const mgn_mlp* m, const float* part, int nchunks, const float* dscale_part, int ntiles,
                 float* grads) {
    RedDesc d;
    d.part = part;
    d.dsp = dscale_part;
    d.grads = grads;
    d.G = grad_G(m);
    d.nchunks = nchunks;
    d.ntiles = ntiles;
    d.NS = m->has_norm ? m->out_dim : 0;
    d.w0_n = d.w0_k = d.xcol0 = 0;
    d.nchunks_x = nchunks;
    d.hoff = 0;
    d.nchunks_h = nchunks;
    d.pad = 0;
    const bool vec = (d.G & 3) == 0 && ((uintptr_t)part & 15) == 0;
    d.blocks = (int32_t)(cdiv64(d.G, vec ? 256 : 64) + d.NS);  // = red_gblocks + NS
    return d;
}

int launch_reduce2(const RedDesc* d, int nd, hipStream_t st) {
    for (int i0 = 0; i0 < nd; i0 += RED_MAX) {
        RedArgs a;
        memset(&a, 0, sizeof(a));
        a.nd = nd - i0 < RED_MAX ? nd - i0 : RED_MAX;
        unsigned blocks = 0;
        for (int i = 0; i < a.nd; ++i) {
            a.d[i] = d[i0 + i];
            blocks += (unsigned)a.d[i].blocks;
        }
        if (blocks == 0) continue;
        ProfScope ps(PROF_WGRAD_REDUCE, st);
        hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(MGN_THREADS), 0, st, a);
        MGN_LAUNCH_CHECK();
    }
    return 0;
}

int launch_reduce(const mgn_mlp* m, const float* part, int nchunks, const float* dscale_part, int ntiles,
                  float* grads, hipStream_t st) {
    const RedDesc d = red_desc(m, part, nchunks, dscale_part, ntiles, grads);
    return launch_reduce2(&d, 1, st);
}

// ring-kernel form of a single-MLP job list (h=128, bf16 or fp32): every R8 job spans a full
// 128-column block, re-gathered inputs are plain rows (no index). false: not eligible (generic kernel).
// job j of a: its X operand as the ring reads it (a full 128-column block), or false
template <class T>
bool ring_job_x(const WgArgs& a, const WgJob& jb, const void** x, int64_t* ld) {
    constexpr int H = 128;
    const int col0 = jb.kb * H;
    if (jb.staged) {
        int s = 0;
        while (s + 1 < a.nseg && col0 >= a.seg[s + 1].coff) ++s;
        const SrcSeg& g = a.seg[s];
        if (g.idx != nullptr || g.ld % 8 != 0 || g.ld == 0 || g.dtype != dtype_id<T>() || col0 - g.coff + H > g.ncols)
            return false;
        *x = reinterpret_cast<const T*>(g.p) + (col0 - g.coff);
        *ld = g.ld;
    } else {
        if (col0 + H > jb.kp) return false;
        *x = reinterpret_cast<const T*>(a.act8) + jb.act_off + (int64_t)col0 * 8;
        *ld = 0;
    }
    return true;
}

template <class T>
bool ring_jobs_from(const WgArgs& a, int nj, int nchunks, RgArgs& r) {
    constexpr int H = 128;
    if (a.H != H || a.M <= 0 || a.rows_per_chunk % RG_RS != 0 || nj > 12) return false;
    memset(&r, 0, sizeof(r));
    r.njobs = nj;
    for (int j = 0; j < nj; ++j) {
        const WgJob& jb = a.job[j];
        RgJob& q = r.job[j];
        const int col0 = jb.kb * H;
        if (!ring_job_x<T>(a, jb, &q.x, &q.ld)) return false;
        q.z = reinterpret_cast<const T*>(a.dz8) + (int64_t)jb.zl * a.RP * H;
        q.RP = a.RP;
        q.M = a.M;
        q.part = a.part;
        q.G = a.G;
        q.w_off = jb.w_off;
        q.b_off = jb.b_off;
        q.n = jb.n;
        q.k = jb.k;
        q.kp = jb.kp;
        q.col0 = col0;
        q.rows_per_chunk = a.rows_per_chunk;
        q.nchunks = nchunks;
        q.wg0 = j * nchunks;
    }
    return true;
}

// prof_kind: PROF_WGRAD for the processor blocks' launch, PROF_WGRAD_DENSE for encoders / decoder;
// f32: the fp32 ring (wgrad_ring_f32_kernel)
int launch_ring(const RgArgs& r, hipStream_t st, int prof_kind = PROF_WGRAD_DENSE, bool f32 = false) {
    const void* fn = f32 ? (const void*)wgrad_ring_f32_kernel : (const void*)wgrad_ring_kernel;
    const size_t lds = f32 ? RF_LDS : RG_LDS;
    if (int e = set_lds(fn, lds)) return e;
    int wgs = 0;
    for (int j = 0; j < r.njobs; ++j) wgs = r.job[j].wg0 + r.job[j].nchunks > wgs ? r.job[j].wg0 + r.job[j].nchunks : wgs;
    if (wgs == 0) return 0;
    ProfScope ps(prof_kind, st);
    if (f32)
        hipLaunchKernelGGL(wgrad_ring_f32_kernel, dim3(wgs), dim3(512), lds, st, r);
    else
        hipLaunchKernelGGL(wgrad_ring_kernel, dim3(wgs), dim3(512), lds, st, r);
    MGN_LAUNCH_CHECK();
    return 0;
}

// jobs: the launch's job list (a.job is filled from it; more than fit one WgArgs — hidden > 128, whose
// 128 x 128 tiles multiply the jobs — run as several launches over the same chunks and slabs)
template <class T, int H>
int launch_wgrad_kernel(WgArgs& a, const WgJob* jobs, int nj, int nchunks, hipStream_t st) {
    constexpr int JMAX = (int)(sizeof(a.job) / sizeof(a.job[0]));
    if constexpr (H <= 128) {
        MGN_REQUIRE(nj <= JMAX, "too many weight-gradient jobs");
        for (int j = 0; j < nj; ++j) a.job[j] = jobs[j];
    }
    a.njobs = nj;
    if constexpr (H == 128) {
        RgArgs r;
        if ((sizeof(T) == 2 || MGN_RING_F32) && ring_jobs_from<T>(a, nj, nchunks, r)) {
            if (nchunks > 0 && nj > 0) return launch_ring(r, st, PROF_WGRAD_DENSE, sizeof(T) == 4);
            return 0;
        }
        // mixed fp32 job lists (the encoders: a layer-0 input narrower than 128 columns): the
        // 128-column jobs on the fp32 ring, the rest on the generic kernel, into the same slabs
        // (disjoint columns): fp32 encoders 163 -> 74 us per launch. bf16: no faster (the generic
        // bf16 kernel is 22 us), so the bf16 encoders keep one launch.
        if (MGN_RING_SPLIT && sizeof(T) == 4 && MGN_RING_F32 && nchunks > 0 && nj > 1) {
            WgArgs ra = a, ga = a;
            int nr = 0, ng = 0;
            for (int j = 0; j < nj; ++j) {
                const void* x;
                int64_t ld;
                if (ring_job_x<T>(a, a.job[j], &x, &ld))
                    ra.job[nr++] = a.job[j];
                else
                    ga.job[ng++] = a.job[j];
            }
            if (nr > 0 && ng > 0 && ring_jobs_from<T>(ra, nr, nchunks, r)) {
                if (int e = launch_ring(r, st, PROF_WGRAD_DENSE, sizeof(T) == 4)) return e;
                a = ga;
                nj = ng;
                a.njobs = nj;
            }
        }
    }
    auto fn = mlp_wgrad_kernel<T, H>;
    const size_t lds = wgrad_lds_bytes<T, H>(a.gathered != 0);
    if (int e = set_lds((const void*)fn, wgrad_lds_bytes<T, H>(true))) return e;
    if (nchunks <= 0 || nj <= 0) return 0;
    if constexpr (H <= 128) {
        ProfScope ps(PROF_WGRAD_DENSE, st);
        hipLaunchKernelGGL(fn, dim3(nchunks, nj), dim3(MGN_THREADS * WG_GROUPS), lds, st, a);
        MGN_LAUNCH_CHECK();
    } else {
        for (int j0 = 0; j0 < nj; j0 += JMAX) {
            const int n = nj - j0 < JMAX ? nj - j0 : JMAX;
            for (int j = 0; j < n; ++j) a.job[j] = jobs[j0 + j];
            a.njobs = n;
            ProfScope ps(PROF_WGRAD_DENSE, st);
            hipLaunchKernelGGL(fn, dim3(nchunks, n), dim3(MGN_THREADS * WG_GROUPS), lds, st, a);
            MGN_LAUNCH_CHECK();
        }
    }
    return 0;
}

// Weight gradients of one MLP over M rows, then the slab reduction into grads. l0_jobs limits the
// layer-0 column blocks (a block edge MLP covers only its e block here; see launch_wgrad_proj).
// nchunks_out: the slab count used (the projection launch must write the same slabs).
template <class T, int H>
int launch_wgrad(const mgn_mlp* m, int64_t M, const void* act8, const void* dz8, const float* dscale_part,
                 int ntiles, float* part, float* grads, const MlpIn* gin, int l0_jobs, int* nchunks_out,
                 bool reduce, hipStream_t st) {
    WgArgs a;
    memset(&a, 0, sizeof(a));
    a.RP = rows_pad(M);
    a.M = M;
    a.gathered = gin != nullptr;
    if (gin) {
        for (int s2 = 0; s2 < gin->nseg; ++s2) a.seg[s2] = gin->seg[s2];
        a.nseg = gin->nseg;
    }
    a.H = H;
    a.dz8 = dz8;
    a.act8 = act8;
    a.part = part;
    a.G = grad_G(m);
    constexpr int TW = wg_tile<H>(), SUB = H / TW;  // 128 x 128 tiles per H x H block (hidden > 128)
    WgJob jobs[MGN_MAX_LAYERS * 3 * SUB * SUB];
    int nj = 0;
    int64_t off = 0;
    for (int l = 0; l < m->n_layers; ++l) {
        int n, k;
        mlp_layer_shape(*m, l, &n, &k);
        int nkb = cdiv(k, H);  // H-wide input blocks (l0_jobs counts these)
        if (l == 0 && l0_jobs > 0 && l0_jobs < nkb) nkb = l0_jobs;
        const int ntb = cdiv(nkb * H < k ? nkb * H : k, TW), nnb = cdiv(n, TW);
        for (int kb = 0; kb < ntb; ++kb)
            for (int nb = 0; nb < nnb; ++nb) {
                MGN_REQUIRE(nj < (int)(sizeof(jobs) / sizeof(jobs[0])), "too many weight-gradient jobs");
                WgJob& j = jobs[nj++];
                memset(&j, 0, sizeof(j));
                j.layer = l;
                j.kb = kb;
                j.nb = nb;
                j.n = n;
                j.k = k;
                j.kp = act_cols(*m, l);
                j.staged = gin != nullptr && l == 0;
                j.zl = l;
                j.w_off = off;
                j.b_off = kb == 0 ? off + (int64_t)n * k : -1;
                j.act_off = act_off(*m, M, l, gin != nullptr);
            }
        off += (int64_t)n * k + n;
    }
    a.rows_per_chunk = wgrad_rows_per_chunk(a.RP, nj, H);
    const int nchunks = (int)cdiv64(a.RP, a.rows_per_chunk);
    if (nchunks_out) *nchunks_out = nchunks;
    if (int e = launch_wgrad_kernel<T, H>(a, jobs, nj, nchunks, st)) return e;
    return reduce ? launch_reduce(m, part, nchunks, dscale_part, ntiles, grads, st) : 0;
}

// dW0[:, H:2H] = Σ_v dP_i[v]ᵀ x[v] and dW0[:, 2H:3H] = Σ_v dP_j[v]ᵀ x[v] of a block edge MLP (the
// node-side form of Σ_k dZ0[k]ᵀ x[dst(k)] / x[src(k)]), into the same nchunks slabs as the edge
// rows (chunks past the node rows write zeros), so one reduction sums both.
template <class T, int H>
int launch_wgrad_proj(const mgn_mlp* m, int64_t N, const void* dP8, const void* x, float* part, int nchunks,
                      hipStream_t st) {
    WgArgs a;
    memset(&a, 0, sizeof(a));
    a.RP = rows_pad(N);
    a.M = N;
    a.gathered = 1;
    a.seg[0] = SrcSeg{x, nullptr, H, H, dtype_id<T>(), H, 0};
    a.seg[1] = SrcSeg{x, nullptr, H, H, dtype_id<T>(), 2 * H, 0};
    a.nseg = 2;
    a.H = H;
    a.dz8 = dP8;
    a.part = part;
    a.G = grad_G(m);
    constexpr int TW = wg_tile<H>(), SUB = H / TW;
    WgJob jobs[2 * SUB * SUB];
    int nj = 0;
    for (int s2 = 0; s2 < 2; ++s2)
        for (int kt = 0; kt < SUB; ++kt)
            for (int nb = 0; nb < SUB; ++nb) {
                WgJob& j = jobs[nj++];
                memset(&j, 0, sizeof(j));
                j.layer = 0;
                j.kb = (1 + s2) * SUB + kt;  // W0 columns [(1 + s2) H + kt TW, + TW)
                j.nb = nb;
                j.n = H;
                j.k = m->in_dim;
                j.kp = m->in_dim;
                j.staged = 1;
                j.zl = s2;
                j.w_off = 0;
                j.b_off = -1;
            }
    if (nchunks <= 0) return 0;
    a.rows_per_chunk = (int)(cdiv64(cdiv64(a.RP, nchunks), 64) * 64);
    return launch_wgrad_kernel<T, H>(a, jobs, nj, nchunks, st);
}

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

// All weight gradients of a GraphNetBlock (bf16, h=128, chained path) in ONE ring launch — the
// edge MLP over edge rows (e block of W0 + layers 1-3), the node MLP over node rows ([x ‖ aggr]
// blocks of W0 + layers 1-3), and the x blocks of the edge W0 over node rows (dP_i/dP_j, into the
// edge MLP's slabs) — then ONE reduction of both MLPs' slabs. Rows per workgroup are balanced over
// all 11 jobs so the grid is about one workgroup per CU.
struct BlockWgradIn {
    int64_t E, N;
    const void *e, *x, *aggr;
    const void *eact, *edz8, *dz0, *dP8;  // dz0: row-major [RP][H] dZ of the edge layer 0
    const float* edsp;
    int entiles;
    float *epart, *egrads;
    const void *nact, *ndz8;
    const float* ndsp;
    int nntiles;
    float *npart, *ngrads;
    // chained bf16, non-NULL: the edge layers 1..3 weight gradients from inputs recomputed out of e
    // and the forward's node projections (mgn_block_saved.proj; pi / pj the P_i / P_j gather indices)
    const void* proj;
    const int32_t *pi, *pj;
};

// T = __bf16: the chained bf16 blocks (dZ0 row-major, the bf16 ring); T = float: fp32 h=128 blocks on
// the generic MLP kernels (every dZ in R8, incl. layer 0; the fp32 ring)
template <class T>
int block_wgrad_ring(const mgn_mlp* edge, const mgn_mlp* node, const BlockWgradIn& in, hipStream_t st,
                     RedDesc* defer = nullptr) {
    constexpr int H = 128;
    constexpr bool F32 = sizeof(T) == 4;
    const int64_t RPE = rows_pad(in.E), RPN = rows_pad(in.N);
    auto rows_for = [](int64_t RP, int64_t target, int* nch, int64_t cmax) {
        int64_t c = cdiv64(RP, target);
        if (c > cmax) c = cmax;
        if (c < 1) c = 1;
        int64_t r = cdiv64(cdiv64(RP, c), 64) * 64;
        *nch = (int)cdiv64(RP, r);
        return (int)r;
    };
    // one round of workgroups, every one over about the same number of rows: 4 edge jobs on ce
    // chunks, 5 node jobs on cn chunks, the 2 W0-projection jobs (node rows, into the edge slabs'
    // x-block columns) on cp ≈ cn chunks — the reduction sums only the first cp slabs of those
    // columns (RedDesc x-columns), so the projections need not be cut into ce short chunks. The
    // edge slab buffer holds slab_chunks(RPE) slabs (keep_layout, mlp_bwd_ws): cp is capped
    // there (graphs with more nodes than edges).
    const int cus = wgrad_cus();
    // recomputed edge layers 1..3 (chain16_edge_wgrad_recompute): their own launch ahead of the ring,
    // cr chunks of 32-row steps over the first cr edge slabs; the ring keeps one edge job (W0's e block)
    const bool rew = !F32 && in.proj != nullptr;
    const int ejobs = rew ? 1 : 4;
    int cr = 0;
    if (rew) {
        int64_t c = rew_max_chunks(RPE);
        if (c > cus) c = cus;
        const int64_t rr = cdiv64(cdiv64(RPE, c), 32) * 32;
        cr = (int)cdiv64(RPE, rr);
        if (int e2 = chain16_edge_wgrad_recompute(edge, in.e, in.proj, in.pi, in.pj, in.E, in.edz8, in.epart,
                                                  grad_G(edge), (int)rr, cr, st))
            return e2;
    }
    int ce = 1, cn = 1, cp = 1;
    int re = 0, rn = 0, rp = 0;
    // chunks per job up to the slab buffers' capacity (keep_layout / mlp_bwd_ws: slab_chunks) — with the
    // recomputed layers the edge MLP keeps ONE ring job, which needs more than 64 chunks to fill the
    // chip on large graphs (Cfg E: 64 chunks of 21.8k rows ran 326 µs on 64 CUs)
    const int64_t cemax = slab_chunks(RPE, edge), cnmax = slab_chunks(RPN, node);
    {
        const int64_t total = ejobs * RPE + 7 * RPN;
        for (int64_t target = cdiv64(cdiv64(total, cus), 64) * 64;; target += 64) {
            re = rows_for(RPE, target, &ce, cemax);
            rn = rows_for(RPN, target, &cn, cnmax);
            if (ejobs * ce + 7 * cn <= cus || (ce == 1 && cn == 1)) break;
        }
        const int64_t cpmax = cemax;
        const int64_t c = cn < cpmax ? cn : cpmax;
        rp = (int)(cdiv64(cdiv64(RPN, c), 64) * 64);
        cp = (int)cdiv64(RPN, rp);
    }
    RgArgs r;
    memset(&r, 0, sizeof(r));
    int nj = 0, wg = 0;
    auto add = [&](const void* z, const void* xs, int64_t ld, int64_t RP, int64_t M, float* part, int64_t G,
                   int64_t w_off, int64_t b_off, int n, int k, int kp, int col0, int rows, int nch) {
        RgJob& q = r.job[nj++];
        q.z = z;
        q.x = xs;
        q.ld = ld;
        q.RP = RP;
        q.M = M;
        q.part = part;
        q.G = G;
        q.w_off = w_off;
        q.b_off = b_off;
        q.n = n;
        q.k = k;
        q.kp = kp;
        q.col0 = col0;
        q.rows_per_chunk = rows;
        q.nchunks = nch;
        q.wg0 = wg;
        wg += nch;
    };
    const T* edz = reinterpret_cast<const T*>(in.edz8);
    const T* ndz = reinterpret_cast<const T*>(in.ndz8);
    const T* dP = reinterpret_cast<const T*>(in.dP8);
    const int64_t Ge = grad_G(edge), Gn = grad_G(node);
    // edge MLP over edge rows (heaviest first: dispatch order)
    int64_t off = 0;
    int64_t hoff = 0;
    for (int l = 0; l < edge->n_layers; ++l) {
        int n, k;
        mlp_layer_shape(*edge, l, &n, &k);
        const T* z = edz + (int64_t)l * RPE * H;
        if (l == 0) {
            add(F32 ? (const void*)z : in.dz0, in.e, H, RPE, in.E, in.epart, Ge, off, off + (int64_t)n * k, n, k, k, 0,
                re, ce);
            r.job[nj - 1].zrm = F32 ? 0 : 1;
            hoff = off + (int64_t)n * k + n;
        } else if (!rew)
            add(z, reinterpret_cast<const T*>(in.eact) + act_off(*edge, in.E, l, 1), 0, RPE, in.E, in.epart, Ge,
                off, off + (int64_t)n * k, n, k, act_cols(*edge, l), 0, re, ce);
        off += (int64_t)n * k + n;
    }
    // node MLP over node rows
    off = 0;
    for (int l = 0; l < node->n_layers; ++l) {
        int n, k;
        mlp_layer_shape(*node, l, &n, &k);
        const T* z = ndz + (int64_t)l * RPN * H;
        if (l == 0) {
            add(z, in.x, H, RPN, in.N, in.npart, Gn, off, off + (int64_t)n * k, n, k, k, 0, rn, cn);
            add(z, in.aggr, H, RPN, in.N, in.npart, Gn, off, -1, n, k, k, H, rn, cn);
        } else {
            add(z, reinterpret_cast<const T*>(in.nact) + act_off(*node, in.N, l, 1), 0, RPN, in.N, in.npart, Gn,
                off, off + (int64_t)n * k, n, k, act_cols(*node, l), 0, rn, cn);
        }
        off += (int64_t)n * k + n;
    }
    // x blocks of the edge W0 over node rows, into the edge slabs (chunks past N write zeros)
    for (int s2 = 0; s2 < 2; ++s2)
        add(dP + (int64_t)s2 * RPN * H, in.x, H, RPN, in.N, in.epart, Ge, 0, -1, H, edge->in_dim, edge->in_dim,
            (1 + s2) * H, rp, cp);
    r.njobs = nj;
    if (int e2 = launch_ring(r, st, PROF_WGRAD, F32)) return e2;
    RedDesc d[2] = {red_desc(edge, in.epart, ce, in.edsp, in.entiles, in.egrads),
                    red_desc(node, in.npart, cn, in.ndsp, in.nntiles, in.ngrads)};
    // W0 [H][3H] of the edge MLP: its x-block columns [H, 3H) hold cp slabs (the projection jobs)
    d[0].w0_n = H;
    d[0].w0_k = edge->in_dim;
    d[0].xcol0 = H;
    d[0].nchunks_x = cp;
    if (rew) {  // layers 1..3 of the edge slabs: the recomputed launch's cr chunks
        d[0].hoff = hoff;
        d[0].nchunks_h = cr;
    }
    (void)re;
    if (defer) {  // the caller reduces later (mgn_wgrad_reduce_many): slabs + partials must persist
        defer[0] = d[0];
        defer[1] = d[1];
        return 0;
    }
    return launch_reduce2(d, 2, st);
}



// Every weight gradient of a GraphNetBlock on the GENERIC kernels (hidden 16/32/64, fp32 or bf16: the
// small configurations — training_config/cylinder.json h=32 fp32, plate.json h=64) in ONE
// mlp_wgrad_kernel launch of per-job operands (WgArgs.multi), jobs and chunking as block_wgrad_ring:
// the edge MLP over edge rows (e block of W0, layers 1-3), the node MLP over node rows ([x ‖ aggr]
// blocks of W0, layers 1-3), the edge W0's x blocks over node rows (dP_i / dP_j, into the edge
// slabs' x-block columns). Replaces 3 weight-gradient launches + 2 reductions per block (the
// reduction joins the deferred one, mgn_wgrad_reduce_many). Every dZ (layer 0 included) is R8.
template <class T, int H>
int block_wgrad_generic(const mgn_mlp* edge, const mgn_mlp* node, const BlockWgradIn& in, hipStream_t st,
                        RedDesc* defer = nullptr) {
    const int64_t RPE = rows_pad(in.E), RPN = rows_pad(in.N);
    auto rows_for = [](int64_t RP, int64_t target, int* nch) {
        int64_t c = cdiv64(RP, target);
        const int64_t cmax = wgrad_max_chunks(RP, H);
        if (c > cmax) c = cmax;
        if (c < 1) c = 1;
        int64_t r = cdiv64(cdiv64(RP, c), 64) * 64;
        *nch = (int)cdiv64(RP, r);
        return (int)r;
    };
    const int cus = wgrad_wgs_per_cu(H) * wgrad_cus();
    int ce = 1, cn = 1, cp = 1, re = 0, rn = 0, rp = 0;
    {
        const int64_t total = 4 * RPE + 7 * RPN;
        for (int64_t target = cdiv64(cdiv64(total, cus), 64) * 64;; target += 64) {
            re = rows_for(RPE, target, &ce);
            rn = rows_for(RPN, target, &cn);
            if (4 * ce + 7 * cn <= cus || (ce == 1 && cn == 1)) break;
        }
        const int64_t cpmax = wgrad_max_chunks(RPE, H);
        const int64_t c = cn < cpmax ? cn : cpmax;
        rp = (int)(cdiv64(cdiv64(RPN, c), 64) * 64);
        cp = (int)cdiv64(RPN, rp);
    }
    WgArgs a;
    memset(&a, 0, sizeof(a));
    a.H = H;
    a.multi = 1;
    a.gathered = 1;
    int nj = 0, maxch = 0;
    const int dt = dtype_id<T>();
    auto add = [&](int layer, int kb, int n, int k, int kp, const void* dz, const void* act, int64_t act_offv,
                   const void* seg_p, int64_t RP, int64_t M, float* part, int64_t Gm, int64_t w_off, int64_t b_off,
                   int rows, int nch) {
        WgJob& j = a.job[nj++];
        j.layer = layer;
        j.kb = kb;
        j.n = n;
        j.k = k;
        j.kp = kp;
        j.staged = seg_p != nullptr;
        j.w_off = w_off;
        j.b_off = b_off;
        j.act_off = act_offv;
        j.zl = 0;
        j.RP = RP;
        j.M = M;
        j.rows_per_chunk = rows;
        j.nchunks = nch;
        j.dz8 = dz;
        j.act8 = act;
        j.part = part;
        j.G = Gm;
        j.seg = SrcSeg{seg_p, nullptr, H, H, dt, kb * H, 0};
        if (nch > maxch) maxch = nch;
    };
    const T* edz = reinterpret_cast<const T*>(in.edz8);
    const T* ndz = reinterpret_cast<const T*>(in.ndz8);
    const T* dP = reinterpret_cast<const T*>(in.dP8);
    const int64_t Ge = grad_G(edge), Gn = grad_G(node);
    int64_t off = 0;
    for (int l = 0; l < edge->n_layers; ++l) {
        int n, k;
        mlp_layer_shape(*edge, l, &n, &k);
        const T* z = edz + (int64_t)l * RPE * H;
        if (l == 0)
            add(0, 0, n, k, k, z, nullptr, 0, in.e, RPE, in.E, in.epart, Ge, off, off + (int64_t)n * k, re, ce);
        else
            add(l, 0, n, k, act_cols(*edge, l), z, in.eact, act_off(*edge, in.E, l, 1), nullptr, RPE, in.E, in.epart,
                Ge, off, off + (int64_t)n * k, re, ce);
        off += (int64_t)n * k + n;
    }
    off = 0;
    for (int l = 0; l < node->n_layers; ++l) {
        int n, k;
        mlp_layer_shape(*node, l, &n, &k);
        const T* z = ndz + (int64_t)l * RPN * H;
        if (l == 0) {
            add(0, 0, n, k, k, z, nullptr, 0, in.x, RPN, in.N, in.npart, Gn, off, off + (int64_t)n * k, rn, cn);
            add(0, 1, n, k, k, z, nullptr, 0, in.aggr, RPN, in.N, in.npart, Gn, off, -1, rn, cn);
        } else {
            add(l, 0, n, k, act_cols(*node, l), z, in.nact, act_off(*node, in.N, l, 1), nullptr, RPN, in.N, in.npart,
                Gn, off, off + (int64_t)n * k, rn, cn);
        }
        off += (int64_t)n * k + n;
    }
    for (int s2 = 0; s2 < 2; ++s2)
        add(0, 1 + s2, H, edge->in_dim, edge->in_dim, dP + (int64_t)s2 * RPN * H, nullptr, 0, in.x, RPN, in.N,
            in.epart, Ge, 0, -1, rp, cp);
    a.njobs = nj;
    auto fn = mlp_wgrad_kernel<T, H>;
    size_t lds = wgrad_lds_bytes<T, H>(true);
    if (wgrad_lds_bytes<T, H>(false) > lds) lds = wgrad_lds_bytes<T, H>(false);
    if (int e = set_lds((const void*)fn, lds)) return e;
    {
        ProfScope ps(PROF_WGRAD, st);
        hipLaunchKernelGGL(fn, dim3(maxch, nj), dim3(MGN_THREADS * WG_GROUPS), lds, st, a);
        MGN_LAUNCH_CHECK();
    }
    RedDesc d[2] = {red_desc(edge, in.epart, ce, in.edsp, in.entiles, in.egrads),
                    red_desc(node, in.npart, cn, in.ndsp, in.nntiles, in.ngrads)};
    d[0].w0_n = H;
    d[0].w0_k = edge->in_dim;
    d[0].xcol0 = H;
    d[0].nchunks_x = cp;
    if (defer) {
        defer[0] = d[0];
        defer[1] = d[1];
        return 0;
    }
    return launch_reduce2(d, 2, st);
}

size_t mlp_bwd_ws(const mgn_mlp* m, int64_t M) {
    const size_t es = m->dtype == MGN_F32 ? 4 : 2;
    // dscale partial rows: the most any backward kernel writes (generic: one per 32-row tile;
    // chained node kernel: one per workgroup, at most one per 16-row tile)
    const int64_t ntiles = rows_pad(M) / 16;
    const int64_t nchunks = slab_chunks(rows_pad(M), m);
    size_t b = align_up((size_t)m->n_layers * rows_pad(M) * m->hidden * es);  // dz8
    b += align_up((size_t)ntiles * m->out_dim * sizeof(float));              // dscale partials
    b += align_up((size_t)nchunks * grad_G(m) * sizeof(float));              // wgrad partial slabs
    return b;
}

}  // namespace

// =========================================================================== dispatch helpers
#define MGN_DISPATCH_H(H_, ...)                                                          \
    switch (H_) {                                                                        \
        case 16: { constexpr int HH = 16; __VA_ARGS__; } break;                          \
        case 32: { constexpr int HH = 32; __VA_ARGS__; } break;                          \
        case 64: { constexpr int HH = 64; __VA_ARGS__; } break;                          \
        case 128: { constexpr int HH = 128; __VA_ARGS__; } break;                        \
        case 256: { constexpr int HH = 256; __VA_ARGS__; } break;                        \
        default: MGN_REQUIRE(false, "unsupported hidden size");                          \
    }

static int mlp_fwd_any(const mgn_mlp* m, int mode, const MlpIn& in, int64_t M, void* out, int out_dtype,
                       int64_t out_ld, const void* resid, mgn_mlp_saved* sv, const mgn_topology* topo,
                       const mgn_mlp* agg_mlp, const mgn_mlp_saved* agg_sv, void* agg_save, hipStream_t st) {
    int rc = 0;
#define MGN_F_CALL(T_, MODE_) rc = launch_fwd<T_, HH, MODE_>(m, in, M, out, out_dtype, out_ld, resid, sv, topo, agg_mlp, agg_sv, agg_save, st)
    if (m->dtype == MGN_F32) {
        if (mode == MODE_DENSE) { MGN_DISPATCH_H(m->hidden, MGN_F_CALL(float, MODE_DENSE)) }
        else if (mode == MODE_EDGE) { MGN_DISPATCH_H(m->hidden, MGN_F_CALL(float, MODE_EDGE)) }
        else { MGN_DISPATCH_H(m->hidden, MGN_F_CALL(float, MODE_NODE)) }
    } else {
        if (mode == MODE_DENSE) { MGN_DISPATCH_H(m->hidden, MGN_F_CALL(__bf16, MODE_DENSE)) }
        else if (mode == MODE_EDGE) { MGN_DISPATCH_H(m->hidden, MGN_F_CALL(__bf16, MODE_EDGE)) }
        else { MGN_DISPATCH_H(m->hidden, MGN_F_CALL(__bf16, MODE_NODE)) }
    }
#undef MGN_F_CALL
    return rc;
}

static int mlp_bwd_any(const mgn_mlp* m, int mode, int64_t M, const mgn_mlp_saved* sv, const void* dout,
                       int dout_dtype, int64_t dout_ld, const BwdOut& o, void* dz, float* dsp, hipStream_t st) {
    int rc = 0;
#define MGN_B_CALL(T_, MODE_) rc = launch_bwd<T_, HH, MODE_>(m, M, sv, dout, dout_dtype, dout_ld, o, dz, dsp, st)
    if (m->dtype == MGN_F32) {
        if (mode == MODE_DENSE) { MGN_DISPATCH_H(m->hidden, MGN_B_CALL(float, MODE_DENSE)) }
        else if (mode == MODE_EDGE) { MGN_DISPATCH_H(m->hidden, MGN_B_CALL(float, MODE_EDGE)) }
        else { MGN_DISPATCH_H(m->hidden, MGN_B_CALL(float, MODE_NODE)) }
    } else {
        if (mode == MODE_DENSE) { MGN_DISPATCH_H(m->hidden, MGN_B_CALL(__bf16, MODE_DENSE)) }
        else if (mode == MODE_EDGE) { MGN_DISPATCH_H(m->hidden, MGN_B_CALL(__bf16, MODE_EDGE)) }
        else { MGN_DISPATCH_H(m->hidden, MGN_B_CALL(__bf16, MODE_NODE)) }
    }
#undef MGN_B_CALL
    return rc;
}

static int mlp_wgrad_any(const mgn_mlp* m, int64_t M, const void* act, const void* dz, const float* dsp,
                         int ntiles, float* part, float* grads, const MlpIn* gin, int l0_jobs, int* nchunks,
                         bool reduce, hipStream_t st) {
    int rc = 0;
#define MGN_W_CALL(T_) rc = launch_wgrad<T_, HH>(m, M, act, dz, dsp, ntiles, part, grads, gin, l0_jobs, nchunks, reduce, st)
    if (m->dtype == MGN_F32) {
        MGN_DISPATCH_H(m->hidden, MGN_W_CALL(float))
    } else {
        MGN_DISPATCH_H(m->hidden, MGN_W_CALL(__bf16))
    }
#undef MGN_W_CALL
    return rc;
}

// Full backward of one MLP: data chain + weight grads. Workspace carve: dz | dscale | part.
static int mlp_backward_impl(const mgn_mlp* m, int mode, int64_t M, const MlpIn& in, const mgn_mlp_saved* sv,
                             const void* dout, int dout_dtype, int64_t dout_ld, const BwdOut& o, float* grads,
                             void* ws, size_t ws_bytes, hipStream_t st) {
    MGN_REQUIRE(ws_bytes >= mlp_bwd_ws(m, M), "backward workspace too small");
    const size_t es = m->dtype == MGN_F32 ? 4 : 2;
    const int ntiles = (int)(rows_pad(M) / bm_host(m->dtype, mode));
    char* p = reinterpret_cast<char*>(ws);
    void* dz = p;
    p += align_up((size_t)m->n_layers * rows_pad(M) * m->hidden * es);
    float* dsp = reinterpret_cast<float*>(p);
    p += align_up((size_t)ntiles * m->out_dim * sizeof(float));
    float* part = reinterpret_cast<float*>(p);
    if (M == 0) {
        MGN_TRY(hipMemsetAsync(grads, 0, (grad_G(m) + (m->has_norm ? m->out_dim : 0)) * sizeof(float), st));
        return 0;
    }
    if (int e = mlp_bwd_any(m, mode, M, sv, dout, dout_dtype, dout_ld, o, dz, dsp, st)) return e;
    return mlp_wgrad_any(m, M, sv->act, dz, dsp, ntiles, part, grads, mode == MODE_DENSE ? nullptr : &in, 0,
                         nullptr, true, st);
}

// =========================================================================== node side of the edge MLP's layer 0
// The edge MLP's first Linear acts on [e ‖ x_i ‖ x_j] (layers.py:689-690,717). Its x blocks are
// applied per NODE instead of per edge: P = [x·W0bᵀ ‖ x·W0cᵀ] (N rows, not E), gathered by the edge
// kernel's layer-0 epilogue. Backward: dP_i[v] = Σ_{dst(k)=v} dZ0[k], dP_j[v] = Σ_{src(k)=v} dZ0[k],
// dx += dP_i·W0b + dP_j·W0c, dW0b = dP_iᵀx, dW0c = dP_jᵀx.
struct ProjArgs {
    const void* x;      // [N][H] (T)
    const void* w0;     // forward fragments of the edge layer 0 ([H x 3H])
    float* proj;        // [N][2H] fp32, or bf16 when out_bf16 (the chained bf16 edge kernels)
    const float* bias0; // optional: b0 folded into the x_i block (the chained edge kernel's layer 0)
    int64_t N;
    int32_t out_bf16;
    int32_t ldi, kstride;
    int32_t wb[2], off[2], ks0[2], nks[2];  // LDS window / leading zero cols / first k-step / k-steps
};

template <class T, int H, int BM>
__global__ __launch_bounds__(MGN_THREADS) void node_proj_kernel(ProjArgs a) {
    constexpr int NTH = H / 16, MT = BM / 16, VEC = Mf<T>::VEC, KSTEP = Mf<T>::KSTEP;
    using G = Gemm<T, NTH, MT>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* In = reinterpret_cast<T*>(smem);
    const int64_t row0 = (int64_t)blockIdx.x * BM;
    const int nw = a.wb[1] == a.wb[0] ? 1 : 2;
    for (int s = 0; s < nw; ++s) {
        const int lead = a.off[s];
        for (int it = threadIdx.x; it < BM * lead; it += MGN_THREADS)
            In[(size_t)(it / lead) * a.ldi + a.wb[s] + it % lead] = from_f<T>(0.f);
        const SrcSeg g{a.x, nullptr, H, H, dtype_id<T>(), a.wb[s] + lead, 0};
        load_tile<T, BM>(In, a.ldi, a.wb[s] + lead + H, a.wb[s] + a.nks[s] * KSTEP, &g, 1, row0, a.N);
    }
    __syncthreads();
    const T* w0 = reinterpret_cast<const T*>(a.w0);
    for (int s = 0; s < 2; ++s) {
        G g;
        g.run(w0 + (size_t)a.ks0[s] * 64 * VEC, a.nks[s], In + a.wb[s], a.ldi, false, a.kstride);
        if (!g.active) continue;
#pragma unroll
        for (int j = 0; j < G::C::MTW; ++j) {
            const int64_t row = row0 + g.m_of(j);
            if (row >= a.N) continue;
#pragma unroll
            for (int i = 0; i < G::C::NTW; ++i) {
                f4 v = g.acc[i][j];
                if (s == 0 && a.bias0) v += ld4u(a.bias0 + g.n_of(i));
                const int n = g.n_of(i);  // 16t + 4g: bf16 P in the chained kernels' pair layout
                const int64_t o = row * (2 * H) + s * H +
                                  (a.out_bf16 ? 32 * (n >> 5) + 8 * ((n >> 2) & 3) + 4 * ((n >> 4) & 1) : n);
                if (a.out_bf16) {
                    const bf16x4 b = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
                    *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(a.proj) + o) = b;
                } else {
                    *reinterpret_cast<f4*>(a.proj + o) = v;
                }
            }
        }
    }
}

#ifndef MGN_COMB_IDXPF
#define MGN_COMB_IDXPF 1  // node_grad: source-direction edge ids prefetched one group ahead (A/B builds: 0)
#endif
#ifndef MGN_COMB_PAIR
#define MGN_COMB_PAIR 0  // 1: node_grad's segment-sum items two at a time (A/B builds)
#endif
struct CombArgs {
    const void* dz0;      // [E][H] (T) dZ of the edge layer 0, target-sorted edges
    const int32_t* col_ptr;
    const int32_t* row_ptr;
    const int32_t* row_perm;
    const void* dx_part;  // [N][H] (T) node-MLP part of dx
    const void* wt0;      // transposed fragments of the edge layer 0 ([3H x H])
    void* dP8;            // R8 [2][RP][H] (T): dP_i, dP_j (weight-gradient operands)
    void* dx;             // [N][H] (T)
    int64_t N, RP;
    int32_t ldb, HP, NS;
    int32_t dx_pair;      // dx in the chained kernels' pair layout (bf16 h=128)
    // round 6, edge-side aggregation: dP_i from the chained edge backward's per-tile run sums of dZ0
    // (chain16_edge_backward agg_scratch): agg_full[v], or agg_tail[tb] + agg_head[tb + 1] + ... + agg_head[te]
    const float* agg_full;
    const float* agg_head;
    const float* agg_tail;
};

template <class T, int H, int BM>
__global__ __launch_bounds__(MGN_THREADS) void node_grad_kernel(CombArgs a) {
    constexpr int NTH = H / 16, MT = BM / 16, VEC = Mf<T>::VEC;
    constexpr int CH = 16 / sizeof(T), CPR = H / CH;
    using G = Gemm<T, NTH, MT>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* B = reinterpret_cast<T*>(smem);  // [BM][ldb]: dP_i at column 0, dP_j at column HP
    const int64_t row0 = (int64_t)blockIdx.x * BM;
    const T* dz = reinterpret_cast<const T*>(a.dz0);
    // segment sums, one (direction, row, 16-byte column chunk) item at a time: every item's segment
    // bounds are loaded up front, then each item gathers its edges in groups of SG with ONE round
    // trip per group (indices past the segment end re-read its last edge and are not added), in
    // edge order — the same fp32 sums as an edge-by-edge loop
    constexpr int NIT = (2 * BM * CPR + MGN_THREADS - 1) / MGN_THREADS, SG = 8;
    int kbs[NIT], kes[NIT];
#pragma unroll
    for (int j = 0; j < NIT; ++j) {
        const int it = threadIdx.x + j * MGN_THREADS;
        const int s = it / (BM * CPR), r = (it - s * (BM * CPR)) / CPR;
        const int64_t v = row0 + r;
        kbs[j] = kes[j] = 0;
        if (it < 2 * BM * CPR && v < a.N) {
            const int32_t* ptr = s == 0 ? a.col_ptr : a.row_ptr;
            kbs[j] = ptr[v];
            kes[j] = ptr[v + 1];
        }
    }
#if MGN_COMB_PAIR
    // two items at a time: the first edge group of BOTH items is in flight together (one round trip
    // for the common in-degree <= SG), longer segments finish item by item; same sums in edge order
    auto item = [&](int j, int& s, int& r, int& c) {
        const int it = threadIdx.x + j * MGN_THREADS;
        s = it / (BM * CPR);
        const int rem = it - s * (BM * CPR);
        r = rem / CPR;
        c = (rem - r * CPR) * CH;
        return it < 2 * BM * CPR;
    };
    auto group = [&](int s, int c, int k, int ke, float (&acc)[CH]) {
        int64_t src[SG];
#pragma unroll
        for (int u = 0; u < SG; ++u) {
            const int ku = k + u < ke ? k + u : ke - 1;
            src[u] = s == 0 ? (int64_t)ku : (int64_t)a.row_perm[ku];
        }
        float t[SG][CH];
#pragma unroll
        for (int u = 0; u < SG; ++u) Chunk<T>::load(dz + src[u] * H + c, t[u]);
#pragma unroll
        for (int u = 0; u < SG; ++u)
            if (k + u < ke) {
#pragma unroll
                for (int e = 0; e < CH; ++e) acc[e] += t[u][e];
            }
    };
#pragma unroll 1
    for (int j = 0; j < NIT; j += 2) {
        int s0, r0, c0, s1 = 0, r1 = 0, c1 = 0;
        if (!item(j, s0, r0, c0)) break;
        const bool two = j + 1 < NIT && item(j + 1, s1, r1, c1);
        const int kb0 = kbs[j], ke0 = kes[j];
        const int kb1 = two ? kbs[j + 1] : 0, ke1 = two ? kes[j + 1] : 0;
        float acc0[CH], acc1[CH];
#pragma unroll
        for (int e = 0; e < CH; ++e) acc0[e] = acc1[e] = 0.f;
        if (kb0 < ke0 && kb1 < ke1) {
            // both first groups' loads issued before either's adds
            int64_t sa[SG], sb[SG];
#pragma unroll
            for (int u = 0; u < SG; ++u) {
                const int ka = kb0 + u < ke0 ? kb0 + u : ke0 - 1, kq = kb1 + u < ke1 ? kb1 + u : ke1 - 1;
                sa[u] = s0 == 0 ? (int64_t)ka : (int64_t)a.row_perm[ka];
                sb[u] = s1 == 0 ? (int64_t)kq : (int64_t)a.row_perm[kq];
            }
            float ta[SG][CH], tb[SG][CH];
#pragma unroll
            for (int u = 0; u < SG; ++u) Chunk<T>::load(dz + sa[u] * H + c0, ta[u]);
#pragma unroll
            for (int u = 0; u < SG; ++u) Chunk<T>::load(dz + sb[u] * H + c1, tb[u]);
#pragma unroll
            for (int u = 0; u < SG; ++u) {
                if (kb0 + u < ke0) {
#pragma unroll
                    for (int e = 0; e < CH; ++e) acc0[e] += ta[u][e];
                }
                if (kb1 + u < ke1) {
#pragma unroll
                    for (int e = 0; e < CH; ++e) acc1[e] += tb[u][e];
                }
            }
#pragma unroll 1
            for (int k = kb0 + SG; k < ke0; k += SG) group(s0, c0, k, ke0, acc0);
#pragma unroll 1
            for (int k = kb1 + SG; k < ke1; k += SG) group(s1, c1, k, ke1, acc1);
        } else {
#pragma unroll 1
            for (int k = kb0; k < ke0; k += SG) group(s0, c0, k, ke0, acc0);
#pragma unroll 1
            for (int k = kb1; k < ke1; k += SG) group(s1, c1, k, ke1, acc1);
        }
        Chunk<T>::store(B + (size_t)r0 * a.ldb + s0 * a.HP + c0, acc0);
        if (two) Chunk<T>::store(B + (size_t)r1 * a.ldb + s1 * a.HP + c1, acc1);
    }
#else
#pragma unroll 1
    for (int j = 0; j < NIT; ++j) {
        const int it = threadIdx.x + j * MGN_THREADS;
        if (it >= 2 * BM * CPR) break;
        const int s = it / (BM * CPR), rem = it - s * (BM * CPR);
        const int r = rem / CPR, c = (rem - r * CPR) * CH;
        const int kb = kbs[j], ke = kes[j];
        float acc[CH];
#pragma unroll
        for (int e = 0; e < CH; ++e) acc[e] = 0.f;
        if (s == 0 && a.agg_full != nullptr) {
            // target direction from the edge backward's partial rows (fp32), in tile order
            if (kb < ke) {
                const int tb = kb >> 4, te = (ke - 1) >> 4;
                const float* p0 = tb == te ? a.agg_full + (row0 + r) * H + c : a.agg_tail + (int64_t)tb * H + c;
#pragma unroll
                for (int e = 0; e < CH; e += 4) {
                    const f4 v = ld4(p0 + e);
                    acc[e] = v[0], acc[e + 1] = v[1], acc[e + 2] = v[2], acc[e + 3] = v[3];
                }
#pragma unroll 1
                for (int tt = tb + 1; tt <= te; ++tt) {
#pragma unroll
                    for (int e = 0; e < CH; e += 4) {
                        const f4 v = ld4(a.agg_head + (int64_t)tt * H + c + e);
                        acc[e] += v[0], acc[e + 1] += v[1], acc[e + 2] += v[2], acc[e + 3] += v[3];
                    }
                }
            }
        } else if (s == 0 || !MGN_COMB_IDXPF) {
#pragma unroll 1
            for (int k = kb; k < ke; k += SG) {
                int64_t src[SG];
#pragma unroll
                for (int u = 0; u < SG; ++u) {
                    const int ku = k + u < ke ? k + u : ke - 1;
                    src[u] = s == 0 ? (int64_t)ku : (int64_t)a.row_perm[ku];
                }
                float t[SG][CH];
#pragma unroll
                for (int u = 0; u < SG; ++u) Chunk<T>::load(dz + src[u] * H + c, t[u]);
#pragma unroll
                for (int u = 0; u < SG; ++u)
                    if (k + u < ke) {
#pragma unroll
                        for (int e = 0; e < CH; ++e) acc[e] += t[u][e];
                    }
            }
        } else if (kb < ke) {
            // source direction: the next group's edge ids (row_perm) load under this group's row
            // loads, so a group costs one round trip instead of two (ids past the segment end clamp
            // to its last edge; same sums in edge order)
            int32_t id[SG];
#pragma unroll
            for (int u = 0; u < SG; ++u) id[u] = a.row_perm[kb + u < ke ? kb + u : ke - 1];
#pragma unroll 1
            for (int k = kb; k < ke; k += SG) {
                float t[SG][CH];
#pragma unroll
                for (int u = 0; u < SG; ++u) Chunk<T>::load(dz + (int64_t)id[u] * H + c, t[u]);
#pragma unroll
                for (int u = 0; u < SG; ++u) id[u] = a.row_perm[k + SG + u < ke ? k + SG + u : ke - 1];
#pragma unroll
                for (int u = 0; u < SG; ++u)
                    if (k + u < ke) {
#pragma unroll
                        for (int e = 0; e < CH; ++e) acc[e] += t[u][e];
                    }
            }
        }
        Chunk<T>::store(B + (size_t)r * a.ldb + s * a.HP + c, acc);
    }
#endif
    const int padc = a.HP - H;
    if (padc > 0)
        for (int it = threadIdx.x; it < 2 * BM * padc; it += MGN_THREADS) {
            const int s = it / (BM * padc), rem = it - s * (BM * padc);
            B[(size_t)(rem / padc) * a.ldb + s * a.HP + H + rem % padc] = from_f<T>(0.f);
        }
    __syncthreads();
    for (int s = 0; s < 2; ++s)
        copy_out_r8<T, BM>(B + s * a.HP, a.ldb, H, reinterpret_cast<T*>(a.dP8) + (int64_t)s * a.RP * H, row0);
    const T* wt = reinterpret_cast<const T*>(a.wt0);
    const size_t tile = (size_t)NTH * a.NS * 64 * VEC;  // one H-wide block of transposed tiles
    G g;
    g.run(wt + tile, a.NS, B, a.ldb);
    g.run(wt + 2 * tile, a.NS, B + a.HP, a.ldb, false, 0, true);
    if (!g.active) return;
    const T* dxp = reinterpret_cast<const T*>(a.dx_part);
    T* dx = reinterpret_cast<T*>(a.dx);
#pragma unroll
    for (int j = 0; j < G::C::MTW; ++j) {
        const int64_t row = row0 + g.m_of(j);
        if (row >= a.N) continue;
#pragma unroll
        for (int i = 0; i < G::C::NTW; ++i) {
            const int n = g.n_of(i);  // 16t + 4g (pair layout: 32(t>>1) + 8g + 4(t&1))
            const int nd = a.dx_pair ? 32 * (n >> 5) + 8 * ((n >> 2) & 3) + 4 * ((n >> 4) & 1) : n;
            st4(dx + row * H + nd, ld4(dxp + row * H + n) + g.acc[i][j]);
        }
    }
}

// layer-0 column window s (1: x_i block, 2: x_j block) of the packed [H x 3H] weight
template <class T>
void proj_window(int H, int s, int* ks0, int* nks, int* off) {
    constexpr int KSTEP = Mf<T>::KSTEP;
    *ks0 = s * H / KSTEP;
    *nks = cdiv((s + 1) * H, KSTEP) - *ks0;
    *off = s * H - *ks0 * KSTEP;
}

#ifndef MGN_PROJ_BM
#define MGN_PROJ_BM 32  // rows per node_proj workgroup (A/B builds: 16)
#endif
template <class T, int H>
int launch_proj(const mgn_mlp* edge, const void* x, int64_t N, float* proj, const float* bias0, hipStream_t st,
                bool out_bf16 = false) {
    constexpr int BM = MGN_PROJ_BM, KSTEP = Mf<T>::KSTEP;
    ProjArgs a;
    memset(&a, 0, sizeof(a));
    a.x = x;
    a.w0 = edge->wpack;
    a.proj = proj;
    a.bias0 = bias0;
    a.out_bf16 = out_bf16;
    a.N = N;
    a.kstride = cdiv(3 * H, KSTEP);
    for (int s = 0; s < 2; ++s) proj_window<T>(H, s + 1, &a.ks0[s], &a.nks[s], &a.off[s]);
    a.wb[0] = 0;
    const bool shared = a.off[0] == 0 && a.off[1] == 0 && a.nks[0] == a.nks[1];
    a.wb[1] = shared ? 0 : a.nks[0] * KSTEP;
    a.ldi = pad_ld<T>(a.wb[1] + a.nks[1] * KSTEP);
    const size_t lds = (size_t)BM * a.ldi * sizeof(T);
    auto fn = node_proj_kernel<T, H, BM>;
    if (int e = set_lds((const void*)fn, lds)) return e;
    const int grid = (int)(rows_pad(N) / BM);
    if (grid == 0) return 0;
    ProfScope ps(PROF_PROJ, st);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(MGN_THREADS), lds, st, a);
    MGN_LAUNCH_CHECK();
    return 0;
}

#ifndef MGN_COMB_BM
#define MGN_COMB_BM 16  // rows per node_grad workgroup: 16 (2 segment-sum items per thread) 20.3 -> 18.1 us vs 32
#endif
template <class T, int H>
int launch_node_grad(const mgn_mlp* edge, const mgn_topology* t, const void* dz0, const void* dx_part, void* dP8,
                     void* dx, hipStream_t st, bool dx_pair = false, void* agg_scratch = nullptr) {
    constexpr int BM = MGN_COMB_BM, KSTEP = Mf<T>::KSTEP;
    CombArgs a;
    memset(&a, 0, sizeof(a));
    if (agg_scratch) {
        MGN_REQUIRE(!MGN_COMB_PAIR && H == 128 && sizeof(T) == 2, "edge-side aggregation: the chained bf16 blocks");
        float *full, *head, *tail;
        chain16_edge_agg_parts(agg_scratch, t->num_nodes, t->num_edges, &full, &head, &tail);
        a.agg_full = full;
        a.agg_head = head;
        a.agg_tail = tail;
    }
    a.dz0 = dz0;
    a.col_ptr = t->col_ptr;
    a.row_ptr = t->row_ptr;
    a.row_perm = t->row_perm;
    a.dx_part = dx_part;
    a.wt0 = edge->wtpack;
    a.dP8 = dP8;
    a.dx = dx;
    a.dx_pair = dx_pair && H == 128 && sizeof(T) == 2;
    a.N = t->num_nodes;
    a.RP = rows_pad(a.N);
    a.HP = rup(H, KSTEP);
    a.NS = cdiv(H, KSTEP);
    a.ldb = pad_ld<T>(2 * a.HP);
    const size_t lds = (size_t)BM * a.ldb * sizeof(T);
    auto fn = node_grad_kernel<T, H, BM>;
    if (int e = set_lds((const void*)fn, lds)) return e;
    const int grid = (int)(a.RP / BM);
    if (grid == 0) return 0;
    ProfScope ps(PROF_COMBINE, st);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(MGN_THREADS), lds, st, a);
    MGN_LAUNCH_CHECK();
    return 0;
}

// =========================================================================== C ABI
extern "C" {

int64_t mgn_linear_pack_elems(int32_t n, int32_t k, int32_t dtype) { return linear_pack_elems(n, k, dtype); }

int64_t mgn_mlp_pack_elems(const mgn_mlp* m) {
    int64_t t = 0;
    for (int l = 0; l < m->n_layers; ++l) {
        int n, k;
        mlp_layer_shape(*m, l, &n, &k);
        t += linear_pack_elems(n, k, m->dtype);
    }
    return t;
}

int mgn_pack_weights(const mgn_pack_job* jobs, int32_t njobs, int64_t max_elems, mgn_stream_t stream) {
    if (njobs <= 0) return 0;
    MGN_REQUIRE(jobs != nullptr, "pack jobs NULL");
    // grid-stride over each job (packed size can exceed n*k: padding); ~4 elements per thread for the
    // largest job keeps the (blocks x jobs) grid small: most workgroups of a wider grid find no work
    int64_t blocks = cdiv64(max_elems, 4 * MGN_THREADS);
    if (blocks > 1024) blocks = 1024;
    if (blocks < 1) blocks = 1;
    ProfScope ps(PROF_PACK, (hipStream_t)stream);
    hipLaunchKernelGGL(pack_kernel, dim3((unsigned)blocks, njobs), dim3(MGN_THREADS), 0, (hipStream_t)stream, jobs);
    MGN_LAUNCH_CHECK();
    return 0;
}

int mgn_mlp_forward(const mgn_mlp* m, const void* in, int32_t in_dtype, int64_t in_ld, const int32_t* in_rows,
                    int64_t rows, void* out, int32_t out_dtype, mgn_mlp_saved* saved, mgn_stream_t stream) {
    if (int e = check_mlp(m)) return e;
    MGN_REQUIRE(saved && saved->act && (m->n_layers < 2 || saved->mask) && (!m->has_norm || (saved->z && saved->rden)),
                "saved buffers missing");
    MGN_REQUIRE(in_dtype == MGN_F32 || in_dtype == m->dtype, "input dtype must be fp32 or the MLP dtype");
    if (chain_dense_eligible(m))
        return chain16_dense_forward(m, in, in_dtype, in_ld, in_rows, rows, out, out_dtype, saved, (hipStream_t)stream);
    MlpIn mi;
    memset(&mi, 0, sizeof(mi));
    mi.seg[0] = SrcSeg{in, in_rows, in_ld, m->in_dim, in_dtype, 0, 0};
    mi.nseg = 1;
    return mlp_fwd_any(m, MODE_DENSE, mi, rows, out, out_dtype, m->out_dim, nullptr, saved, nullptr, nullptr,
                       nullptr, nullptr, (hipStream_t)stream);
}

size_t mgn_mlp_backward_workspace_bytes(const mgn_mlp* m, int64_t rows) { return mlp_bwd_ws(m, rows); }

int mgn_mlp_saved_elems(const mgn_mlp* m, int64_t rows, int32_t block_mlp, int64_t* act_elems,
                        int64_t* mask_words) {
    *act_elems = act_off(*m, rows, m->n_layers, block_mlp != 0);
    *mask_words = (int64_t)(m->n_layers - 1) * mask_words_per_layer(*m, rows);
    return 0;
}

// keep != NULL: the dscale partials and weight-gradient slabs go to `keep` (mlp_keep_bytes) and the
// reduction is left to the caller (*defer); else they are carved from ws and reduced here.
static size_t mlp_keep_bytes(const mgn_mlp* m, int64_t rows) {
    const int64_t ntiles = rows_pad(rows) / 16;  // the most any backward kernel writes (as mlp_bwd_ws)
    return align_up((size_t)ntiles * m->out_dim * sizeof(float)) +
           align_up((size_t)wgrad_max_chunks(rows_pad(rows), m->hidden) * grad_G(m) * sizeof(float));
}

// part: 0 = data + weight gradients; MGN_BWD_DATA_ONLY = the data gradients (and the saves the weight
// gradients read; defer->ntiles = the dscale partial rows written); MGN_BWD_WGRAD_ONLY = the weight
// gradients of an earlier DATA_ONLY call over the same buffers (defer->ntiles as it left it)
static int mlp_backward_entry(const mgn_mlp* m, const void* in, int32_t in_dtype, int64_t in_ld, const int32_t* in_rows,
                              int64_t rows, const mgn_mlp_saved* saved, const void* dout, int32_t dout_dtype, void* din,
                              int32_t din_dtype, float* grads, void* ws, size_t ws_bytes, void* keep, RedDesc* defer,
                              hipStream_t st, int32_t part = 0) {
    if (int e = check_mlp(m)) return e;
    MGN_REQUIRE(ws_bytes >= mlp_bwd_ws(m, rows), "backward workspace too small");
    const bool chained = chain_dense_eligible(m) && rows > 0;
    const size_t es = m->dtype == MGN_F32 ? 4 : 2;
    int ntiles = (int)(rows_pad(rows) / bm_host(m->dtype, MODE_DENSE));
    char* p = reinterpret_cast<char*>(ws);
    void* dz = p;
    p += align_up((size_t)m->n_layers * rows_pad(rows) * m->hidden * (chained ? 2 : es));
    char* q = keep ? reinterpret_cast<char*>(keep) : p;
    float* dsp = reinterpret_cast<float*>(q);
    q += align_up((size_t)(keep ? rows_pad(rows) / 16 : ntiles) * m->out_dim * sizeof(float));
    float* part_buf = reinterpret_cast<float*>(q);
    if (rows == 0) {
        if (part != MGN_BWD_DATA_ONLY)
            MGN_TRY(hipMemsetAsync(grads, 0, (grad_G(m) + (m->has_norm ? m->out_dim : 0)) * sizeof(float), st));
        return 0;
    }
    if (part == MGN_BWD_WGRAD_ONLY) {
        MGN_REQUIRE(defer && defer->ntiles > 0, "MGN_BWD_WGRAD_ONLY needs the reduce descriptor of the DATA_ONLY call");
        ntiles = defer->ntiles;
    } else if (chained) {
        // chained data gradients (dZ of every layer, din) + the generic weight gradients over the
        // same R8 operands
        MGN_REQUIRE(dout_dtype == MGN_F32 || dout_dtype == MGN_BF16, "dout dtype must be MGN_F32 or MGN_BF16");
        if (int e = chain16_dense_backward(m, rows, saved, dout, dout_dtype, din, din_dtype, m->in_dim, dz, dsp,
                                           &ntiles, st))
            return e;
    } else {
        BwdOut o;
        memset(&o, 0, sizeof(o));
        o.mode = MODE_DENSE;
        o.din = din;
        o.din_dtype = din_dtype;
        o.din_ld = m->in_dim;
        if (int e = mlp_bwd_any(m, MODE_DENSE, rows, saved, dout, dout_dtype, m->out_dim, o, dz, dsp, st)) return e;
    }
    if (part == MGN_BWD_DATA_ONLY) {
        memset(defer, 0, sizeof(*defer));
        defer->ntiles = ntiles;  // blocks = 0: nothing to reduce yet
        return 0;
    }
    int nchunks = 0;
    if (int e = mlp_wgrad_any(m, rows, saved->act, dz, dsp, ntiles, part_buf, grads, nullptr, 0, &nchunks,
                              defer == nullptr, st))
        return e;
    if (defer) *defer = red_desc(m, part_buf, nchunks, dsp, ntiles, grads);
    return 0;
}

int mgn_mlp_backward(const mgn_mlp* m, const void* in, int32_t in_dtype, int64_t in_ld, const int32_t* in_rows,
                     int64_t rows, const mgn_mlp_saved* saved, const void* dout, int32_t dout_dtype, void* din,
                     int32_t din_dtype, float* grads, void* ws, size_t ws_bytes, mgn_stream_t stream) {
    (void)in;
    (void)in_dtype;
    (void)in_ld;
    (void)in_rows;  // a dense MLP's layer-0 input is in its R8 saves
    return mlp_backward_entry(m, in, in_dtype, in_ld, in_rows, rows, saved, dout, dout_dtype, din, din_dtype, grads, ws,
                              ws_bytes, nullptr, nullptr, (hipStream_t)stream);
}

size_t mgn_mlp_backward_keep_bytes(const mgn_mlp* m, int64_t rows) { return mlp_keep_bytes(m, rows); }

int mgn_mlp_backward_deferred(const mgn_mlp* m, const void* in, int32_t in_dtype, int64_t in_ld,
                              const int32_t* in_rows, int64_t rows, const mgn_mlp_saved* saved, const void* dout,
                              int32_t dout_dtype, void* din, int32_t din_dtype, float* grads, void* ws,
                              size_t ws_bytes, void* keep, size_t keep_bytes, mgn_wgrad_reduce* reduce1,
                              mgn_stream_t stream) {
    return mgn_mlp_backward_deferred2(m, in, in_dtype, in_ld, in_rows, rows, saved, dout, dout_dtype, din, din_dtype,
                                      grads, ws, ws_bytes, keep, keep_bytes, reduce1, 0, stream);
}

int mgn_mlp_backward_deferred2(const mgn_mlp* m, const void* in, int32_t in_dtype, int64_t in_ld,
                               const int32_t* in_rows, int64_t rows, const mgn_mlp_saved* saved, const void* dout,
                               int32_t dout_dtype, void* din, int32_t din_dtype, float* grads, void* ws,
                               size_t ws_bytes, void* keep, size_t keep_bytes, mgn_wgrad_reduce* reduce1,
                               int32_t flags, mgn_stream_t stream) {
    MGN_REQUIRE(reduce1 && keep, "keep buffer and reduce1 required");
    const int32_t part = flags & (MGN_BWD_DATA_ONLY | MGN_BWD_WGRAD_ONLY);
    MGN_REQUIRE(!(flags & ~(MGN_BWD_DATA_ONLY | MGN_BWD_WGRAD_ONLY)) && part != (MGN_BWD_DATA_ONLY | MGN_BWD_WGRAD_ONLY),
                "flags: 0, MGN_BWD_DATA_ONLY or MGN_BWD_WGRAD_ONLY");
    if (int e = check_mlp(m)) return e;
    MGN_REQUIRE(keep_bytes >= mlp_keep_bytes(m, rows), "mlp backward keep buffer too small");
    RedDesc d;
    if (part == MGN_BWD_WGRAD_ONLY)
        memcpy(&d, reduce1, sizeof(d));  // the DATA_ONLY call's partial-row count
    else
        memset(&d, 0, sizeof(d));
    memset(reduce1, 0, sizeof(mgn_wgrad_reduce));
    if (int e = mlp_backward_entry(m, in, in_dtype, in_ld, in_rows, rows, saved, dout, dout_dtype, din, din_dtype, grads,
                                   ws, ws_bytes, keep, &d, (hipStream_t)stream, part))
        return e;
    memcpy(reduce1, &d, sizeof(d));
    return 0;
}

int mgn_mlp_backward_deferred3(const mgn_mlp* m, const void* in, int32_t in_dtype, int64_t in_ld,
                               const int32_t* in_rows, int64_t rows, const mgn_mlp_saved* saved, const void* dout,
                               int32_t dout_dtype, void* din, int32_t din_dtype, float* grads, void* ws,
                               size_t ws_bytes, void* keep, size_t keep_bytes, mgn_wgrad_reduce* reduce1,
                               int32_t flags, const mgn_call_opts* opts, mgn_stream_t stream) {
    MGN_REQUIRE(!opts || (opts->data_cus >= 0 && opts->wgrad_cus >= 0), "CU caps must be >= 0 (0 = no cap)");
    CallScope cs(opts);
    return mgn_mlp_backward_deferred2(m, in, in_dtype, in_ld, in_rows, rows, saved, dout, dout_dtype, din, din_dtype,
                                      grads, ws, ws_bytes, keep, keep_bytes, reduce1, flags, stream);
}

static size_t block_fwd_ws(const mgn_topology* t, const mgn_mlp* edge) {
    return align_up((size_t)t->num_nodes * 2 * edge->hidden * sizeof(float));
}

int mgn_block_forward_inference_supported(const mgn_mlp* edge, const mgn_mlp* node) {
    return chain_eligible(edge) && chain_node_eligible(node) ? 1 : 0;
}

size_t mgn_block_forward_workspace_bytes(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node) {
    (void)node;
    return block_fwd_ws(t, edge);
}

// Edge-side aggregation (round 6, chain16_fwd_kernel EAGG): for graphs of high in-degree the edge
// forward sums each 16-edge tile's messages per run of equal dst and the node forward adds those partial
// rows (about deg/16 + 1 per node) instead of gathering every in-edge's z row — at Cfg E (in-degree 62)
// the node forward's 0.36 GB of z gathers per block. MGN_EDGE_AGG: "auto" (default: E >= 16 N), "1"
// (every chained training block), "0" (never). The partial sums re-associate the fp32 aggregation (fixed
// order, deterministic); the per-edge messages are the same bf16-z terms.
// bwd: the backward's use (the edge backward's dZ0 sums for node_grad's dP_i) — measured at Cfg E
// (profiles/r06_eagg_ab.txt): node_grad 145.5 -> 127.5 us but the edge backward 510 -> 533 us, so "auto"
// keeps it off (the target-direction half of node_grad streams contiguous rows and was already cheap);
// MGN_EDGE_AGG "1" turns both on, "fwd" / "bwd" one direction alone (tests, A/B)
static bool edge_agg_mode(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node, bool bwd = false) {
    if (!(chain_eligible(edge) && chain_node_eligible(node) && t->num_nodes > 0 && t->num_edges > 0)) return false;
    const char* v = getenv("MGN_EDGE_AGG");
    if (v && v[0] == '0') return false;
    if (v && v[0] == '1') return true;
    if (v && !strcmp(v, "fwd")) return !bwd;
    if (v && !strcmp(v, "bwd")) return bwd;
    return !bwd && t->num_edges >= 16 * t->num_nodes;
}

static int block_forward_impl(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node, const void* x,
                              const void* e, void* x_out, void* e_out, mgn_block_saved* saved, void* ws,
                              size_t ws_bytes, int proj_ready, const mgn_mlp* next_edge, void* next_ws,
                              size_t next_ws_bytes, int* next_proj_ready, mgn_stream_t stream,
                              void* scratch = nullptr, size_t scratch_bytes = 0) {
    if (next_proj_ready) *next_proj_ready = 0;
    if (int r = check_mlp(edge)) return r;
    if (int r = check_mlp(node)) return r;
    const int H = edge->hidden;
    MGN_REQUIRE(edge->in_dim == 3 * H && edge->out_dim == H, "edge MLP must be 3h -> h");
    MGN_REQUIRE(node->in_dim == 2 * H && node->out_dim == H && node->hidden == H, "node MLP must be 2h -> h");
    MGN_REQUIRE(saved->edge.z && saved->edge.rden, "block saved buffers missing");
    MGN_REQUIRE(edge->dtype == node->dtype, "edge/node MLP dtype mismatch");
    // inference (saved->edge.act == NULL): the chained bf16 h=128 kernels skip every backward save
    const bool infer = saved->edge.act == nullptr;
    MGN_REQUIRE(infer || saved->aggr, "block saved buffers missing");
    MGN_REQUIRE(!infer || (chain_eligible(edge) && chain_node_eligible(node) &&
                           saved->node.act == nullptr),
                "inference block forward (saved act = NULL) needs the chained bf16 h=128 path "
                "(mgn_block_forward_inference_supported)");
    MGN_REQUIRE(ws_bytes >= block_fwd_ws(t, edge) && (ws || t->num_nodes == 0), "block forward workspace too small");
    // saved->proj (ABI v16): no R8 saves of the edge MLP's hidden-layer inputs, the backward recomputes
    // them from e and the projections this call leaves in ws
    const bool rew = saved->proj != nullptr;
    MGN_REQUIRE(!rew || (!infer && chain_eligible(edge) && chain_node_eligible(node) && saved->proj == ws &&
                         t->num_nodes > 0 && t->num_edges > 0),
                "saved->proj: a training forward of chained bf16 h=128 edge and node MLPs, proj == ws");
    hipStream_t st = (hipStream_t)stream;
    const int dt = edge->dtype;
    float* proj = reinterpret_cast<float*>(ws);
    const bool chain = chain_eligible(edge);
    const float* b0 = chain ? edge->bias[0] : nullptr;  // the chained kernel takes b0 from P_i
    MGN_REQUIRE(!proj_ready || chain || dt == MGN_F32,
                "proj_ready: the workspace holds the projections of the chained bf16 path or of the fp32 node MLP");
    // Small graphs on the generic kernels (hidden <= 64): layer 0 as the reference's single K = 3h
    // product over the gathered [e ‖ x_i ‖ x_j] rows (layers.py:689-690) — the node-projection launch
    // would cost more than the 4h² FLOPs per edge it saves (cylinder.json / plate.json sizes)
    const bool unsplit = !chain && H <= 64 && t->num_edges > 0 && t->num_edges <= (1 << 18);
    int rc = 0;
    if (proj_ready || unsplit) {
        // P already in ws: the previous block's node-MLP forward wrote it from its x_out
    } else if (dt == MGN_F32) {
        MGN_DISPATCH_H(H, rc = (launch_proj<float, HH>(edge, x, t->num_nodes, proj, b0, st)))
    } else {
        // the chained edge kernels gather P as bf16 (half the bytes; P rounded once, like the bf16
        // layer output the reference's autocast produces)
        MGN_DISPATCH_H(H, rc = (launch_proj<__bf16, HH>(edge, x, t->num_nodes, proj, b0, st, chain)))
    }
    if (rc) return rc;
    MlpIn ein;
    memset(&ein, 0, sizeof(ein));
    ein.seg[0] = SrcSeg{e, nullptr, H, H, dt, 0, 0};
    ein.nseg = 1;
    ein.K0 = H;
    ein.proj = proj;
    ein.proj_i = t->csc_dst;
    ein.proj_j = t->csc_src;
    if (unsplit) {
        ein.seg[1] = SrcSeg{x, t->csc_dst, H, H, dt, H, 0};      // x_i = x[edge_index[1]]
        ein.seg[2] = SrcSeg{x, t->csc_src, H, H, dt, 2 * H, 0};  // x_j = x[edge_index[0]]
        ein.nseg = 3;
        ein.K0 = 3 * H;
        ein.proj = nullptr;
    }
    // edge-side aggregation: a training forward given the scratch (mgn_block_forward_scratch_bytes)
    void* agg = nullptr;
    if (chain && !infer && scratch && edge_agg_mode(t, edge, node)) {
        MGN_REQUIRE(scratch_bytes >= chain16_edge_agg_bytes(t->num_nodes, t->num_edges),
                    "block forward scratch too small (mgn_block_forward_scratch_bytes)");
        agg = scratch;
    }
    if (chain) {
        if (int r = chain16_edge_forward(edge, e, proj, t->csc_dst, t->csc_src, t->num_edges, e_out, &saved->edge, st,
                                         chain_node_eligible(node), !rew, t->num_nodes, agg))
            return r;
    } else if (int r = mlp_fwd_any(edge, MODE_EDGE, ein, t->num_edges, e_out, dt, H, e, &saved->edge, t, nullptr,
                                   nullptr, nullptr, st)) {
        return r;
    }
    if (chain && chain_node_eligible(node)) {
        const bool fuse = next_edge && next_ws && chain_eligible(next_edge) && next_edge->hidden == H &&
                          next_ws_bytes >= block_fwd_ws(t, next_edge) && t->num_nodes > 0;
        if (int r = chain16_node_forward(node, x, t, edge, &saved->edge, t->num_nodes, x_out, saved->aggr,
                                         &saved->node, st, fuse ? next_edge : nullptr, fuse ? next_ws : nullptr, agg))
            return r;
        if (fuse && next_proj_ready) *next_proj_ready = 1;
        return 0;
    }
    MlpIn nin;
    memset(&nin, 0, sizeof(nin));
    nin.seg[0] = SrcSeg{x, nullptr, H, H, dt, 0, 0};
    nin.nseg = 1;
    // fp32 h=128: the chained node kernel also computes the next block's node projections (the next
    // call skips its projection launch)
    int pn_done = 0;
    if (MGN_F32N_PROJ && dt == MGN_F32 && H == 128 && next_edge && next_ws && next_edge->dtype == MGN_F32 &&
        next_edge->hidden == H &&
        next_edge->in_dim == 3 * H && next_ws_bytes >= block_fwd_ws(t, next_edge) && t->num_nodes > 0 &&
        t->num_edges > 0) {
        nin.pn_pack = reinterpret_cast<const float*>(next_edge->wpack);
        nin.pn_out = reinterpret_cast<float*>(next_ws);
        nin.pn_done = &pn_done;
    }
    // K0 = 2H: the aggregation fills columns [H, 2H) inside the kernel
    if (int r = mlp_fwd_any(node, MODE_NODE, nin, t->num_nodes, x_out, dt, H, x, &saved->node, t, edge, &saved->edge,
                            saved->aggr, st))
        return r;
    if (pn_done && next_proj_ready) *next_proj_ready = 1;
    return 0;
}

int mgn_block_forward(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node, const void* x, const void* e,
                      void* x_out, void* e_out, mgn_block_saved* saved, void* ws, size_t ws_bytes,
                      mgn_stream_t stream) {
    return block_forward_impl(t, edge, node, x, e, x_out, e_out, saved, ws, ws_bytes, 0, nullptr, nullptr, 0, nullptr,
                              stream);
}

size_t mgn_block_forward_scratch_bytes(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node) {
    return edge_agg_mode(t, edge, node) ? chain16_edge_agg_bytes(t->num_nodes, t->num_edges) : 0;
}

int mgn_block_forward_chain2(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node, const void* x,
                             const void* e, void* x_out, void* e_out, mgn_block_saved* saved, void* ws,
                             size_t ws_bytes, int proj_ready, const mgn_mlp* next_edge, void* next_ws,
                             size_t next_ws_bytes, int* next_proj_ready, void* scratch, size_t scratch_bytes,
                             mgn_stream_t stream) {
    return block_forward_impl(t, edge, node, x, e, x_out, e_out, saved, ws, ws_bytes, proj_ready, next_edge, next_ws,
                              next_ws_bytes, next_proj_ready, stream, scratch, scratch_bytes);
}

int mgn_block_forward_chain(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node, const void* x,
                            const void* e, void* x_out, void* e_out, mgn_block_saved* saved, void* ws,
                            size_t ws_bytes, int proj_ready, const mgn_mlp* next_edge, void* next_ws,
                            size_t next_ws_bytes, int* next_proj_ready, mgn_stream_t stream) {
    return block_forward_impl(t, edge, node, x, e, x_out, e_out, saved, ws, ws_bytes, proj_ready, next_edge, next_ws,
                              next_ws_bytes, next_proj_ready, stream);
}

// mlp: edge MLP backward workspace (generic path: shared with the node MLP's, used in sequence);
// nmlp: the node MLP's own (chained path: its dZ saves and slabs live until the block's single
// weight-gradient launch at the end)
struct BlockWs {
    size_t mlp, nmlp, dxpart, daggr, dz0, dP8, agg, total;
};

static BlockWs block_ws_parts(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node) {
    const size_t es = edge->dtype == MGN_F32 ? 4 : 2;
    const int H = edge->hidden;
    size_t mlp_ws = mlp_bwd_ws(edge, t->num_edges);
    const size_t nws = mlp_bwd_ws(node, t->num_nodes);
    if (nws > mlp_ws) mlp_ws = nws;
    BlockWs w;
    size_t o = 0;
    w.mlp = o;
    o += align_up(mlp_ws);
    w.nmlp = o;
    o += align_up(nws);
    w.dxpart = o;
    o += align_up((size_t)t->num_nodes * H * es);
    w.daggr = o;
    o += align_up((size_t)t->num_nodes * H * es);
    w.dz0 = o;
    o += align_up((size_t)rows_pad(t->num_edges) * H * es);  // chained path: padded rows written (zero)
    w.dP8 = o;
    o += align_up((size_t)2 * rows_pad(t->num_nodes) * H * es);
    // edge-side aggregation of dZ0 (round 6, edge_agg_mode): the edge backward's per-tile run sums
    w.agg = 0;
    if (edge_agg_mode(t, edge, node, true)) {
        w.agg = o;
        o += align_up(chain16_edge_agg_bytes(t->num_nodes, t->num_edges));
    }
    w.total = o;
    return w;
}

size_t mgn_block_backward_workspace_bytes(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node) {
    return block_ws_parts(t, edge, node).total;
}

// The block backward in two halves over one workspace: _data (node-MLP backward, edge-MLP backward,
// node gradients: dx, de) and _wgrad (weight gradients + fixed-order reduction into the gradient
// buffers). _wgrad reads only what _data left in `ws` and the forward saves, so the caller may run it
// on another stream, overlapped with the next block's _data on a second workspace (the hot path:
// the bandwidth-bound weight-gradient launch fills the CUs the latency-bound node kernels leave idle).
struct BlockBwdCarve {
    bool gen1;       // generic MLPs of hidden < 128: one multi-job weight-gradient launch (block_wgrad_generic)
    void *mlp_ws, *dx_part, *d_aggr, *dz0, *dP8;
    void* ndz;       // chained / ring32: node dZ saves (R8)
    float* ndsp;     // chained / ring32: node dscale partials
    float* npart;    // chained / ring32: node slabs
    void* dz8;       // edge dZ saves (R8)
    float* dsp;      // edge dscale partials
    float* part;     // edge slabs
    bool chained;    // bf16 h=128 register-chained MLPs (+ the bf16 ring)
    bool ring32;     // fp32 h=128 generic MLPs + the fp32 ring
    void* agg;       // edge-side aggregation scratch (BlockWs.agg; nullptr: off)
};

// fp32 h=128 processor blocks (the reference's dtype): the node MLP's weight gradients join ONE fp32
// ring launch per block with the edge MLP's and the W0 projections', as in the chained bf16 blocks
static bool ring_f32_eligible(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node) {
    return MGN_RING_F32 && edge->dtype == MGN_F32 && node->dtype == MGN_F32 && edge->hidden == 128 &&
           node->hidden == 128 && edge->n_layers == 4 && node->n_layers == 4 && edge->in_dim == 3 * 128 &&
           node->in_dim == 2 * 128 && edge->out_dim == 128 && node->out_dim == 128 && t->num_nodes > 0 &&
           t->num_edges > 0;
}

// generic blocks of hidden < 128 (cylinder.json h=32 fp32, plate.json h=64 bf16): the node MLP keeps its
// dZ saves for ONE multi-job weight-gradient launch per block (block_wgrad_generic)
static bool gen1_eligible(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node) {
    const int H = edge->hidden;
    return (H == 16 || H == 32 || H == 64) && node->hidden == H && edge->dtype == node->dtype &&
           edge->n_layers == 4 && node->n_layers == 4 && edge->in_dim == 3 * H && node->in_dim == 2 * H &&
           edge->out_dim == H && node->out_dim == H && t->num_nodes > 0 && t->num_edges > 0;
}

// Deferred-reduction "keep" buffer of one block: the RMSNorm-scale partial rows and the weight-
// gradient slabs of both MLPs, which then outlive the block's call (the caller reduces every block's
// in one launch, mgn_wgrad_reduce_many). Sizes: the most any launch writes (as mlp_bwd_ws).
struct KeepLayout {
    size_t edsp, epart, ndsp, npart, total;
};
static KeepLayout keep_layout(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node) {
    KeepLayout k;
    size_t o = 0;
    const int64_t RPE = rows_pad(t->num_edges), RPN = rows_pad(t->num_nodes);
    k.edsp = o;
    o += align_up((size_t)(RPE / 16) * edge->out_dim * sizeof(float));
    k.epart = o;
    o += align_up((size_t)slab_chunks(RPE, edge) * grad_G(edge) * sizeof(float));
    k.ndsp = o;
    o += align_up((size_t)(RPN / 16) * node->out_dim * sizeof(float));
    k.npart = o;
    o += align_up((size_t)slab_chunks(RPN, node) * grad_G(node) * sizeof(float));
    k.total = o;
    return k;
}

static BlockBwdCarve block_bwd_carve(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node, void* ws,
                                     const BlockWs& wl, void* keep = nullptr) {
    BlockBwdCarve c;
    memset(&c, 0, sizeof(c));
    const int H = edge->hidden, dt = edge->dtype;
    char* w = reinterpret_cast<char*>(ws);
    c.mlp_ws = w + wl.mlp;
    c.dx_part = w + wl.dxpart;
    c.d_aggr = w + wl.daggr;
    c.dz0 = w + wl.dz0;
    c.dP8 = w + wl.dP8;
    c.chained = chain_eligible(edge) && chain_node_eligible(node) && t->num_nodes > 0 && t->num_edges > 0;
    c.agg = wl.agg && c.chained ? w + wl.agg : nullptr;
    c.ring32 = !c.chained && ring_f32_eligible(t, edge, node);
    c.gen1 = !c.chained && !c.ring32 && gen1_eligible(t, edge, node);
    if (c.chained || c.ring32 || c.gen1) {
        const int64_t Nn = t->num_nodes;
        char* q = w + wl.nmlp;
        c.ndz = q;
        q += align_up((size_t)node->n_layers * rows_pad(Nn) * H * (node->dtype == MGN_F32 ? 4 : 2));
        c.ndsp = reinterpret_cast<float*>(q);
        q += align_up((size_t)(rows_pad(Nn) / 16) * node->out_dim * sizeof(float));  // = mlp_bwd_ws carve
        c.npart = reinterpret_cast<float*>(q);
    }
    const int64_t E = t->num_edges;
    const size_t es = dt == MGN_F32 ? 4 : 2;
    const int ntiles = (int)(rows_pad(E) / bm_host(dt, MODE_EDGE));
    char* p = reinterpret_cast<char*>(c.mlp_ws);
    c.dz8 = p;
    p += align_up((size_t)edge->n_layers * rows_pad(E) * H * es);
    c.dsp = reinterpret_cast<float*>(p);
    p += align_up((size_t)ntiles * edge->out_dim * sizeof(float));
    c.part = reinterpret_cast<float*>(p);
    if (keep && (c.chained || c.ring32 || c.gen1)) {
        const KeepLayout k = keep_layout(t, edge, node);
        char* q = reinterpret_cast<char*>(keep);
        c.dsp = reinterpret_cast<float*>(q + k.edsp);
        c.part = reinterpret_cast<float*>(q + k.epart);
        c.ndsp = reinterpret_cast<float*>(q + k.ndsp);
        c.npart = reinterpret_cast<float*>(q + k.npart);
    }
    return c;
}

static int block_bwd_check(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node, const void* de_out,
                           size_t ws_bytes, BlockWs* wl) {
    if (int r = check_mlp(edge)) return r;
    if (int r = check_mlp(node)) return r;
    *wl = block_ws_parts(t, edge, node);
    MGN_REQUIRE(ws_bytes >= wl->total, "block backward workspace too small");
    MGN_REQUIRE(de_out || t->num_edges == 0 || chain_eligible(edge),
                "de_out = NULL (zero edge-output gradient) needs the chained bf16 h=128 edge MLP");
    MGN_REQUIRE(wl->nmlp - wl->mlp >= mlp_bwd_ws(edge, t->num_edges), "backward workspace too small");
    return 0;
}

static int block_backward_data_impl(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node, const void* x,
                                    const mgn_block_saved* saved, const void* dx_out, const void* de_out, void* dx,
                                    void* de, float* node_grads, void* ws, size_t ws_bytes, void* keep,
                                    mgn_stream_t stream, int32_t flags = 0) {
    BlockWs wl;
    if (int r = block_bwd_check(t, edge, node, de_out, ws_bytes, &wl)) return r;
    hipStream_t st = (hipStream_t)stream;
    const int H = edge->hidden, dt = edge->dtype;
    const BlockBwdCarve c = block_bwd_carve(t, edge, node, ws, wl, keep);
    flags &= ~(MGN_BWD_DATA_ONLY | MGN_BWD_WGRAD_ONLY);
    MGN_REQUIRE(!(flags & ~(MGN_BWD_DE_OUT_PAIR | MGN_BWD_DE_PAIR | MGN_BWD_DX_OUT_PAIR | MGN_BWD_DX_PAIR)),
                "unknown backward layout flags");
    MGN_REQUIRE(!flags || (chain_eligible(edge) && chain_node_eligible(node)),
                "pair-layout de (MGN_BWD_DE_*_PAIR) needs the chained bf16 h=128 edge and node MLPs");

    // node MLP: dY = dx_out -> dx_part = dx_out + dA0[:, :H], d_aggr = dA0[:, H:]
    if (c.chained) {
        // chained data gradients; the node MLP's weight gradients join the block's single ring launch
        MGN_REQUIRE(wl.dxpart - wl.nmlp >= mlp_bwd_ws(node, t->num_nodes), "backward workspace too small");
        int nparts = 0;
        if (int r = chain16_node_backward(node, t->num_nodes, &saved->node, dx_out, c.ndz, c.ndsp, &nparts, c.dx_part,
                                          c.d_aggr, st, flags & MGN_BWD_DX_OUT_PAIR))
            return r;
    } else if (c.ring32 || c.gen1) {
        // generic data gradients, dZ saves and dscale partials kept for the block's single
        // weight-gradient launch (the fp32 ring, or block_wgrad_generic)
        MGN_REQUIRE(wl.dxpart - wl.nmlp >= mlp_bwd_ws(node, t->num_nodes), "backward workspace too small");
        BwdOut on;
        memset(&on, 0, sizeof(on));
        on.mode = MODE_NODE;
        on.o1 = c.dx_part;
        on.o2 = c.d_aggr;
        if (int r = mlp_bwd_any(node, MODE_NODE, t->num_nodes, &saved->node, dx_out, dt, H, on, c.ndz, c.ndsp, st))
            return r;
    } else {
        MlpIn nin;
        memset(&nin, 0, sizeof(nin));
        nin.seg[0] = SrcSeg{x, nullptr, H, H, dt, 0, 0};
        nin.seg[1] = SrcSeg{saved->aggr, nullptr, H, H, dt, H, 0};
        nin.nseg = 2;
        BwdOut on;
        memset(&on, 0, sizeof(on));
        on.mode = MODE_NODE;
        on.o1 = c.dx_part;
        on.o2 = c.d_aggr;
        if (int r = mlp_backward_impl(node, MODE_NODE, t->num_nodes, nin, &saved->node, dx_out, dt, H, on, node_grads,
                                      c.mlp_ws, wl.nmlp - wl.mlp, st))
            return r;
    }
    // edge MLP data gradients: dY = de_out + d_aggr[dst] -> de = de_out + dZ0·W0a, dZ0 (row-major)
    const int64_t E = t->num_edges;
    BwdOut oe;
    memset(&oe, 0, sizeof(oe));
    oe.mode = MODE_EDGE;
    oe.gath = c.d_aggr;
    oe.gath_idx = t->csc_dst;
    oe.o1 = de;
    oe.o2 = c.dz0;
    if (chain_eligible(edge)) {
        int ntiles = 0;
        // pair-layout z and d_aggr iff the node MLP is chained too (as in the forward)
        if (int r = chain16_edge_backward(edge, E, &saved->edge, de_out, c.d_aggr, t->csc_dst, c.dz8, c.dsp, &ntiles,
                                          de, c.dz0, st, chain_node_eligible(node), flags & MGN_BWD_DE_OUT_PAIR,
                                          flags & MGN_BWD_DE_PAIR, t->num_nodes, c.agg))
            return r;
    } else if (E > 0) {
        if (int r = mlp_bwd_any(edge, MODE_EDGE, E, &saved->edge, de_out, dt, H, oe, c.dz8, c.dsp, st)) return r;
    }
    // node side: dP = segment sums of dZ0, dx = dx_part + dP_i·W0b + dP_j·W0c
    int rc = 0;
    if (dt == MGN_F32) {
        MGN_DISPATCH_H(H, rc = (launch_node_grad<float, HH>(edge, t, c.dz0, c.dx_part, c.dP8, dx, st)))
    } else {
        MGN_DISPATCH_H(H, rc = (launch_node_grad<__bf16, HH>(edge, t, c.dz0, c.dx_part, c.dP8, dx, st,
                                                              flags & MGN_BWD_DX_PAIR, c.agg)))
    }
    return rc;
}

int mgn_block_backward_data(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node, const void* x,
                            const void* e, const mgn_block_saved* saved, const void* dx_out, const void* de_out,
                            void* dx, void* de, float* edge_grads, float* node_grads, void* ws, size_t ws_bytes,
                            mgn_stream_t stream) {
    (void)e;
    (void)edge_grads;
    return block_backward_data_impl(t, edge, node, x, saved, dx_out, de_out, dx, de, node_grads, ws, ws_bytes,
                                    nullptr, stream);
}

static int block_backward_wgrad_impl(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node, const void* x,
                                     const void* e, const mgn_block_saved* saved, const void* de_out,
                                     float* edge_grads, float* node_grads, void* ws, size_t ws_bytes, void* keep,
                                     RedDesc* defer, mgn_stream_t stream) {
    BlockWs wl;
    if (int r = block_bwd_check(t, edge, node, de_out, ws_bytes, &wl)) return r;
    hipStream_t st = (hipStream_t)stream;
    const int H = edge->hidden, dt = edge->dtype;
    const BlockBwdCarve c = block_bwd_carve(t, edge, node, ws, wl, keep);
    const int64_t E = t->num_edges, N = t->num_nodes;
    if (c.chained) {
        BlockWgradIn in;
        in.E = E;
        in.N = N;
        in.e = e;
        in.x = x;
        in.aggr = saved->aggr;
        in.eact = saved->edge.act;
        in.edz8 = c.dz8;
        in.dz0 = c.dz0;
        in.dP8 = c.dP8;
        in.edsp = c.dsp;
        in.entiles = chain16_edge_backward_parts(E);
        in.epart = c.part;
        in.egrads = edge_grads;
        in.nact = saved->node.act;
        in.ndz8 = c.ndz;
        in.ndsp = c.ndsp;
        in.nntiles = chain16_node_backward_parts(N);
        in.npart = c.npart;
        in.ngrads = node_grads;
        in.proj = saved->proj;
        in.pi = t->csc_dst;
        in.pj = t->csc_src;
        return block_wgrad_ring<__bf16>(edge, node, in, st, keep ? defer : nullptr);
    }
    if (c.ring32 || c.gen1) {
        BlockWgradIn in;
        in.E = E;
        in.N = N;
        in.e = e;
        in.x = x;
        in.aggr = saved->aggr;
        in.eact = saved->edge.act;
        in.edz8 = c.dz8;
        in.dz0 = c.dz0;
        in.dP8 = c.dP8;
        in.edsp = c.dsp;
        in.entiles = (int)(rows_pad(E) / bm_host(dt, MODE_EDGE));
        in.epart = c.part;
        in.egrads = edge_grads;
        in.nact = saved->node.act;
        in.ndz8 = c.ndz;
        in.ndsp = c.ndsp;
        in.nntiles = (int)(rows_pad(N) / bm_host(dt, MODE_NODE));
        in.npart = c.npart;
        in.ngrads = node_grads;
        in.proj = nullptr;
        in.pi = in.pj = nullptr;
        if (c.ring32) return block_wgrad_ring<float>(edge, node, in, st, keep ? defer : nullptr);
        int rc = 0;
        if (dt == MGN_F32) {
            MGN_DISPATCH_H(H, rc = (block_wgrad_generic<float, HH>(edge, node, in, st, keep ? defer : nullptr)))
        } else {
            MGN_DISPATCH_H(H, rc = (block_wgrad_generic<__bf16, HH>(edge, node, in, st, keep ? defer : nullptr)))
        }
        return rc;
    }
    // weight gradients: edge rows (e block of W0 + layers 1..), node rows (x blocks of W0), one reduce
    const int ntiles = chain_eligible(edge) ? chain16_edge_backward_parts(E) : (int)(rows_pad(E) / bm_host(dt, MODE_EDGE));
    MlpIn ein;
    memset(&ein, 0, sizeof(ein));
    ein.seg[0] = SrcSeg{e, nullptr, H, H, dt, 0, 0};
    ein.nseg = 1;
    int nchunks = 0;
    if (int r = mlp_wgrad_any(edge, E, saved->edge.act, c.dz8, c.dsp, ntiles, c.part, edge_grads, &ein, 1, &nchunks,
                              false, st))
        return r;
    int rc = 0;
    if (dt == MGN_F32) {
        MGN_DISPATCH_H(H, rc = (launch_wgrad_proj<float, HH>(edge, N, c.dP8, x, c.part, nchunks, st)))
    } else {
        MGN_DISPATCH_H(H, rc = (launch_wgrad_proj<__bf16, HH>(edge, N, c.dP8, x, c.part, nchunks, st)))
    }
    if (rc) return rc;
    return launch_reduce(edge, c.part, nchunks, c.dsp, ntiles, edge_grads, st);
}

int mgn_block_backward_wgrad(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node, const void* x,
                             const void* e, const mgn_block_saved* saved, const void* dx_out, const void* de_out,
                             void* dx, void* de, float* edge_grads, float* node_grads, void* ws, size_t ws_bytes,
                             mgn_stream_t stream) {
    (void)dx_out;
    (void)dx;
    (void)de;
    return block_backward_wgrad_impl(t, edge, node, x, e, saved, de_out, edge_grads, node_grads, ws, ws_bytes,
                                     nullptr, nullptr, stream);
}

static_assert(sizeof(mgn_wgrad_reduce) == sizeof(RedDesc) && offsetof(mgn_wgrad_reduce, G) == offsetof(RedDesc, G) &&
                  offsetof(mgn_wgrad_reduce, blocks) == offsetof(RedDesc, blocks),
              "mgn_wgrad_reduce must mirror RedDesc");

size_t mgn_block_backward_keep_bytes(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node) {
    return keep_layout(t, edge, node).total;
}

int mgn_block_backward_deferred(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node, const void* x,
                                const void* e, const mgn_block_saved* saved, const void* dx_out, const void* de_out,
                                void* dx, void* de, float* edge_grads, float* node_grads, void* ws, size_t ws_bytes,
                                void* keep, size_t keep_bytes, mgn_wgrad_reduce* reduce2, mgn_stream_t stream) {
    return mgn_block_backward_deferred2(t, edge, node, x, e, saved, dx_out, de_out, dx, de, edge_grads, node_grads, ws,
                                        ws_bytes, keep, keep_bytes, reduce2, 0, stream);
}

int mgn_block_backward_deferred2(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node, const void* x,
                                 const void* e, const mgn_block_saved* saved, const void* dx_out, const void* de_out,
                                 void* dx, void* de, float* edge_grads, float* node_grads, void* ws,
                                 size_t ws_bytes, void* keep, size_t keep_bytes, mgn_wgrad_reduce* reduce2,
                                 int32_t flags, mgn_stream_t stream) {
    MGN_REQUIRE(reduce2, "reduce2 (two mgn_wgrad_reduce) required");
    if (!(flags & MGN_BWD_WGRAD_ONLY)) memset(reduce2, 0, 2 * sizeof(mgn_wgrad_reduce));
    BlockWs wl;
    if (int r = block_bwd_check(t, edge, node, de_out, ws_bytes, &wl)) return r;
    const bool chained = (chain_eligible(edge) && chain_node_eligible(node) && t->num_nodes > 0 && t->num_edges > 0) ||
                         ring_f32_eligible(t, edge, node) || gen1_eligible(t, edge, node);
    // a block whose weight gradients cannot be deferred (or keep = NULL) runs whole in its DATA_ONLY
    // call (reduced at once) and its WGRAD_ONLY call does nothing
    const int32_t part = flags & (MGN_BWD_DATA_ONLY | MGN_BWD_WGRAD_ONLY);
    MGN_REQUIRE(part != (MGN_BWD_DATA_ONLY | MGN_BWD_WGRAD_ONLY),
                "MGN_BWD_DATA_ONLY and MGN_BWD_WGRAD_ONLY exclude each other");
    if ((!chained || !keep) && part == MGN_BWD_WGRAD_ONLY) return 0;
    flags &= ~(MGN_BWD_DATA_ONLY | MGN_BWD_WGRAD_ONLY);
    if (!chained) {  // generic MLPs: reduced at once, nothing left for the caller
        MGN_REQUIRE(!flags, "pair-layout de (MGN_BWD_DE_*_PAIR) needs the chained bf16 h=128 edge and node MLPs");
        if (int r = block_backward_data_impl(t, edge, node, x, saved, dx_out, de_out, dx, de, node_grads, ws,
                                             ws_bytes, nullptr, stream))
            return r;
        return block_backward_wgrad_impl(t, edge, node, x, e, saved, de_out, edge_grads, node_grads, ws, ws_bytes,
                                         nullptr, nullptr, stream);
    }
    if (!keep) {  // reduced at once (mgn_block_backward with layout flags): reduce2 stays zeroed
        if (int r = block_backward_data_impl(t, edge, node, x, saved, dx_out, de_out, dx, de, node_grads, ws,
                                             ws_bytes, nullptr, stream, flags))
            return r;
        return block_backward_wgrad_impl(t, edge, node, x, e, saved, de_out, edge_grads, node_grads, ws, ws_bytes,
                                         nullptr, nullptr, stream);
    }
    MGN_REQUIRE(keep_bytes >= keep_layout(t, edge, node).total, "block backward keep buffer too small");
    if (part != MGN_BWD_WGRAD_ONLY) {
        if (int r = block_backward_data_impl(t, edge, node, x, saved, dx_out, de_out, dx, de, node_grads, ws, ws_bytes,
                                             keep, stream, flags))
            return r;
        if (part == MGN_BWD_DATA_ONLY) return 0;
    }
    RedDesc d[2];
    memset(d, 0, sizeof(d));
    if (int r = block_backward_wgrad_impl(t, edge, node, x, e, saved, de_out, edge_grads, node_grads, ws, ws_bytes,
                                          keep, d, stream))
        return r;
    memcpy(reduce2, d, sizeof(d));
    return 0;
}

int mgn_block_backward_deferred3(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node, const void* x,
                                 const void* e, const mgn_block_saved* saved, const void* dx_out, const void* de_out,
                                 void* dx, void* de, float* edge_grads, float* node_grads, void* ws,
                                 size_t ws_bytes, void* keep, size_t keep_bytes, mgn_wgrad_reduce* reduce2,
                                 int32_t flags, const mgn_call_opts* opts, mgn_stream_t stream) {
    MGN_REQUIRE(!opts || (opts->data_cus >= 0 && opts->wgrad_cus >= 0), "CU caps must be >= 0 (0 = no cap)");
    CallScope cs(opts);
    return mgn_block_backward_deferred2(t, edge, node, x, e, saved, dx_out, de_out, dx, de, edge_grads, node_grads, ws,
                                        ws_bytes, keep, keep_bytes, reduce2, flags, stream);
}

int mgn_wgrad_reduce_many(const mgn_wgrad_reduce* reds, int32_t n, mgn_stream_t stream) {
    MGN_REQUIRE(n >= 0 && (n == 0 || reds), "bad reduction list");
    std::vector<RedDesc> d;
    for (int32_t i = 0; i < n; ++i) {
        RedDesc x;
        memcpy(&x, &reds[i], sizeof(x));
        if (x.blocks > 0) d.push_back(x);
    }
    if (d.empty()) return 0;
    return launch_reduce2(d.data(), (int)d.size(), (hipStream_t)stream);
}

int mgn_block_backward(const mgn_topology* t, const mgn_mlp* edge, const mgn_mlp* node, const void* x, const void* e,
                       const mgn_block_saved* saved, const void* dx_out, const void* de_out, void* dx, void* de,
                       float* edge_grads, float* node_grads, void* ws, size_t ws_bytes, mgn_stream_t stream) {
    if (int r = mgn_block_backward_data(t, edge, node, x, e, saved, dx_out, de_out, dx, de, edge_grads, node_grads,
                                        ws, ws_bytes, stream))
        return r;
    return mgn_block_backward_wgrad(t, edge, node, x, e, saved, dx_out, de_out, dx, de, edge_grads, node_grads, ws,
                                    ws_bytes, stream);
}

}  // extern "C"
