// Shared device helpers for libmgn (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>
#include <cmath>

#include <string>

#include "mgn.h"

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define MGN_WAVE 64
#define MGN_THREADS 256
#define RMS_EPS 1e-8f

// --------------------------------------------------------------------------- MFMA traits
// D[i][j] += sum_k A[i][k] * B[k][j], 16x16 tile per wave.
//   f32  (v_mfma_f32_16x16x4_f32):   lane l holds A[l&15][l>>4],          B[l>>4][l&15]
//   bf16 (v_mfma_f32_16x16x32_bf16): lane l holds A[l&15][8(l>>4)+v],     B[8(l>>4)+v][l&15]
//   C/D (both): lane l, reg r ->  D[(l>>4)*4 + r][l&15]
template <class T>
struct Mf;
template <>
struct Mf<float> {
    static constexpr int VEC = 1, KSTEP = 4;
    typedef float frag;
    static __device__ __forceinline__ f4 mma(frag a, frag b, f4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
};
template <>
struct Mf<__bf16> {
    static constexpr int VEC = 8, KSTEP = 32;
    typedef bf16x8 frag;
    static __device__ __forceinline__ f4 mma(frag a, frag b, f4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
};

template <class T>
__device__ __forceinline__ typename Mf<T>::frag ld_frag(const T* p) {
    return *reinterpret_cast<const typename Mf<T>::frag*>(p);
}

// --------------------------------------------------------------------------- conversions
__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(__bf16 x) { return (float)x; }
template <class T>
__device__ __forceinline__ T from_f(float x);
template <>
__device__ __forceinline__ float from_f<float>(float x) { return x; }
template <>
__device__ __forceinline__ __bf16 from_f<__bf16>(float x) { return (__bf16)x; }

__device__ __forceinline__ float load_any(const void* p, int dtype, int64_t i) {
    return dtype == MGN_F32 ? reinterpret_cast<const float*>(p)[i]
                            : (float)reinterpret_cast<const __bf16*>(p)[i];
}

// 4 consecutive values <-> f4
__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }
__device__ __forceinline__ f4 ld4(const __bf16* p) {
    bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
    return f4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
// 4 consecutive fp32 with only 4-byte alignment guaranteed (parameters in an unpadded flat buffer)
__device__ __forceinline__ f4 ld4u(const float* p) { return f4{p[0], p[1], p[2], p[3]}; }
__device__ __forceinline__ void st4(float* p, f4 v) { *reinterpret_cast<f4*>(p) = v; }
__device__ __forceinline__ void st4(__bf16* p, f4 v) {
    bf16x4 o = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
    *reinterpret_cast<bf16x4*>(p) = o;
}

// 16-byte chunks: 4 floats or 8 bf16, returned as floats (up to 8)
template <class T>
struct Chunk;
template <>
struct Chunk<float> {
    static constexpr int N = 4;
    static __device__ __forceinline__ void load(const float* p, float* o) {
        f4 v = *reinterpret_cast<const f4*>(p);
        o[0] = v[0]; o[1] = v[1]; o[2] = v[2]; o[3] = v[3];
    }
    static __device__ __forceinline__ void store(float* p, const float* o) {
        *reinterpret_cast<f4*>(p) = f4{o[0], o[1], o[2], o[3]};
    }
};
template <>
struct Chunk<__bf16> {
    static constexpr int N = 8;
    static __device__ __forceinline__ void load(const __bf16* p, float* o) {
        bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (float)v[i];
    }
    static __device__ __forceinline__ void store(__bf16* p, const float* o) {
        bf16x8 v;
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = (__bf16)o[i];
        *reinterpret_cast<bf16x8*>(p) = v;
    }
};

__host__ __device__ __forceinline__ int cdiv(int a, int b) { return (a + b - 1) / b; }
__host__ __device__ __forceinline__ int64_t cdiv64(int64_t a, int64_t b) { return (a + b - 1) / b; }
__host__ __device__ __forceinline__ int rup(int a, int b) { return cdiv(a, b) * b; }

// --------------------------------------------------------------------------- packed weights
// Forward fragments of W[n][k] (nn.Linear weight [out, in]):
//   pack[((nt*KS + ks)*64 + lane)*VEC + v] = W[nt*16 + (lane&15)][ks*KSTEP + VEC*(lane>>4) + v]
// Transposed fragments (A operand of dX = dY·W):
//   packT[((kt*NS + ns)*64 + lane)*VEC + v] = W[ns*KSTEP + VEC*(lane>>4) + v][kt*16 + (lane&15)]
// kt runs over round_up(ceil(K/16), 8) tiles so a backward chunk of hidden/16 tiles never reads
// past the layer. Both use the same per-layer element count. An fp32 Linear with n == 128 and k a
// multiple of 128 also carries a 128x128 "chain image" of its first 128 input columns after the
// fragments of either region (the register-chained fp32 edge kernels' LDS-DMA source, mgn_mlp.hip):
//   image[((nt*8 + t)*64 + lane)*4 + r]  = W[nt*16 + (lane&15)][t*16 + 4*(lane>>4) + r]   (forward)
//   imageT[((kt*8 + t)*64 + lane)*4 + r] = W[t*16 + 4*(lane>>4) + r][kt*16 + (lane&15)]   (transposed)
// — one such image per 128-column block of the input (round 5: the chained fp32 node MLP's layer 0
// reads both blocks of its [x ‖ aggr] weight, the next block's projections the x_i / x_j blocks of the
// edge W0), block b's image of columns 128b .. 128b + 127 at chain_image_off(n, k, b) (mgn_mlp.hip).
__host__ __device__ inline int chain_images(int n, int k, int dtype) {
    return dtype == MGN_F32 && n == 128 && k > 0 && k % 128 == 0 ? k / 128 : 0;
}
__host__ __device__ inline bool has_chain_image(int n, int k, int dtype) { return chain_images(n, k, dtype) > 0; }
__host__ __device__ inline int64_t linear_pack_elems(int n, int k, int dtype) {
    const int vec = dtype == MGN_BF16 ? 8 : 1, kstep = 4 * vec;
    int64_t fwd = (int64_t)cdiv(n, 16) * cdiv(k, kstep);
    int64_t bwd = (int64_t)rup(cdiv(k, 16), 8) * cdiv(n, kstep);
    return (fwd > bwd ? fwd : bwd) * 64 * vec + (int64_t)chain_images(n, k, dtype) * 128 * 128;
}

// Layer shapes of build_mlp(in, hidden, out, L)
__host__ __device__ inline void mlp_layer_shape(const mgn_mlp& m, int l, int* n, int* k) {
    *k = l == 0 ? m.in_dim : m.hidden;
    *n = l == m.n_layers - 1 ? m.out_dim : m.hidden;
}

// --------------------------------------------------------------------------- errors
void mgn_set_error(const std::string& s);
#define MGN_TRY(expr)                                                                  \
    do {                                                                               \
        hipError_t _e = (expr);                                                        \
        if (_e != hipSuccess) {                                                        \
            mgn_set_error(std::string(#expr) + ": " + hipGetErrorString(_e));          \
            return (int)_e;                                                            \
        }                                                                              \
    } while (0)
#define MGN_REQUIRE(cond, msg)                                                         \
    do {                                                                               \
        if (!(cond)) {                                                                 \
            mgn_set_error(msg);                                                        \
            return 1000;                                                               \
        }                                                                              \
    } while (0)
#define MGN_LAUNCH_CHECK() MGN_TRY(hipGetLastError())

// --------------------------------------------------------------------------- opt-in profiler
// Kernel classes timed by mgn_profile_* (HIP events on the launch stream; off by default).
enum MgnProfKind {
    PROF_FWD_EDGE = 0, PROF_FWD_NODE, PROF_FWD_DENSE, PROF_BWD_EDGE, PROF_BWD_NODE, PROF_BWD_DENSE,
    PROF_WGRAD, PROF_WGRAD_REDUCE, PROF_COMBINE, PROF_PACK, PROF_ADAMW, PROF_PROJ, PROF_WGRAD_DENSE, PROF_KINDS
};
int mgn_prof_begin(int kind, hipStream_t st);  // returns slot or -1 when disabled
void mgn_prof_end(int slot, hipStream_t st);
struct ProfScope {
    int slot;
    hipStream_t st;
    ProfScope(int kind, hipStream_t s) : slot(mgn_prof_begin(kind, s)), st(s) {}
    ~ProfScope() { mgn_prof_end(slot, st); }
};

// --------------------------------------------------------------------------- saved-activation layout
// Row-octet ("R8") layout of a [rows x cols] matrix: element (m, c) at ((m/8)*cols + c)*8 + m%8.
// Eight consecutive rows of one column are contiguous (16 B in bf16): exactly one MFMA operand
// fragment when the reduction runs over rows (weight gradients), so the weight-gradient GEMMs load
// operands straight from HBM/L2 with 16-byte loads and no LDS transposition.
__host__ __device__ __forceinline__ int64_t r8_index(int64_t m, int64_t c, int64_t cols) {
    return ((m >> 3) * cols + c) * 8 + (m & 7);
}
// Saved buffers cover rows padded to 64 (every tile, including pure-padding rows, is written).
// compute units of the current device (read once; 256 on MI355X)
// CUs the persistent kernels size their grids for. MGN_MAX_CUS (read once) caps it, so two streams
// can each run a persistent kernel on part of the chip at the same time (intra-GPU data parallelism
// experiments: tools/exp_dual.py).
// Per-call options (mgn_call_opts, ABI v17; replaces v13's process-global mgn_set_grid_cus): the CU
// caps of the persistent grids of every launch except the weight-gradient launches (data_cus) and of
// the weight-gradient launches (wgrad_cus; 0 = none), so a block's weight gradients can run on a stream
// of their own beside the next block's data gradients, each on its own share of the CUs; and the device
// error word the hand-off waits of the recomputed weight gradients report a timeout to. CallScope
// installs a call's options for the duration of that call only, on the calling thread (restored on
// return), so two models, streams or threads never see each other's caps. Read when a launch is issued
// (a captured graph keeps its grids).
struct MgnCallCtx {
    int data_cus, wgrad_cus;
    uint32_t* err_word;
};
extern thread_local MgnCallCtx g_call;
struct CallScope {
    MgnCallCtx saved;
    explicit CallScope(const mgn_call_opts* o) : saved(g_call) {
        g_call = MgnCallCtx{o ? o->data_cus : 0, o ? o->wgrad_cus : 0, o ? o->err_word : nullptr};
    }
    ~CallScope() { g_call = saved; }
};
inline int hw_cus();
inline int device_cus() {
    const int c = hw_cus();
    return g_call.data_cus > 0 && g_call.data_cus < c ? g_call.data_cus : c;
}
inline int wgrad_cus() {
    const int c = hw_cus();
    return g_call.wgrad_cus > 0 && g_call.wgrad_cus < c ? g_call.wgrad_cus : c;
}
inline int hw_cus() {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
            cus = n;
        else
            cus = 256;
        if (const char* e = getenv("MGN_MAX_CUS")) {
            const int c = atoi(e);
            if (c > 0 && c < cus) cus = c;
        }
    }
    return cus;
}
__host__ __device__ __forceinline__ int64_t rows_pad(int64_t M) { return (M + 63) / 64 * 64; }
// RMSNorm's d^(-1/2) (layers.py:59-74) of an MLP: the true feature count (norm_dim) of a padded MLP
inline float norm_dinv(const mgn_mlp* m) {
    const int d = m->norm_dim > 0 ? m->norm_dim : m->out_dim;
    return (float)(1.0 / sqrt((double)d));
}
__host__ __device__ __forceinline__ int kstep_of(int dtype) { return dtype == MGN_BF16 ? 32 : 4; }
// R8 column count of the saved INPUT of layer l (layer 0: padded MLP input; else padded hidden)
__host__ __device__ inline int act_cols(const mgn_mlp& m, int l) {
    const int ks = kstep_of(m.dtype);
    return l == 0 ? rup(m.in_dim, ks) : rup(m.hidden, ks);
}
// gathered != 0: MLP of a GraphNetBlock, whose layer-0 input ([e‖x_i‖x_j] or [x‖aggr]) is not
// saved (the weight-gradient kernel re-gathers it); layer 0's block then has zero size.
__host__ __device__ inline int64_t act_off(const mgn_mlp& m, int64_t M, int l, int gathered = 0) {
    int64_t o = 0;
    for (int j = 0; j < l; ++j) o += (gathered && j == 0) ? 0 : rows_pad(M) * act_cols(m, j);
    return o;
}
// ReLU masks of the hidden-layer outputs: per layer, per (16-row tile, 16-col tile), 4 ballot words
__host__ __device__ inline int64_t mask_words_per_layer(const mgn_mlp& m, int64_t M) {
    return rows_pad(M) / 16 * (m.hidden / 16) * 4;
}
