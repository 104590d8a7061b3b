// Topology build, row permutation, stand-alone segment sum, AdamW, status (gfx950).
//
// mgn_topology_build turns the reference's edge_index [2,E] int64 (row = source j, col = target
// i; PyG flow "source_to_target", reference graphphysics/models/layers.py:649,688) into:
//   target-sorted ("CSC") order by a STABLE radix sort on col — for a coalesced (row, col)-sorted
//   edge list (PyG to_undirected) every in-edge segment is then in increasing source order, which
//   is exactly the order the reference's scatter_add_ visits them, so fp32 sums match the
//   reference summation order;
//   col_ptr: in-edge segments (forward aggregation, backward of x[col]);
//   row_perm/row_ptr: the same edges stably sorted by source (backward of x[row]).
#include <hipcub/hipcub.hpp>

#include <cmath>
#include <cstring>

#include "mgn_common.h"

thread_local MgnCallCtx g_call = {0, 0, nullptr};  // CallScope (mgn_call_opts, ABI v17)

static thread_local std::string g_err;
void mgn_set_error(const std::string& s) { g_err = s; }

namespace {

__global__ void split_edge_index(const int64_t* __restrict__ ei, int64_t E, int64_t N, int32_t* __restrict__ src,
                                 int32_t* __restrict__ dst, int32_t* __restrict__ iota, unsigned* __restrict__ bad) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= E) return;
    const int64_t r = ei[k], c = ei[E + k];
    if (r < 0 || r >= N || c < 0 || c >= N) atomicOr(bad, MGN_ERR_EDGE_INDEX);
    src[k] = (int32_t)(r < 0 ? 0 : (r >= N ? N - 1 : r));
    dst[k] = (int32_t)(c < 0 ? 0 : (c >= N ? N - 1 : c));
    iota[k] = (int32_t)k;
}

__global__ void gather_i32(const int32_t* __restrict__ v, const int32_t* __restrict__ idx, int64_t n,
                           int32_t* __restrict__ out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) out[k] = v[idx[k]];
}

// ptr[i] = lower_bound(sorted, i) for i in [0, N]
__global__ void segment_ptr(const int32_t* __restrict__ sorted, int64_t E, int64_t N, int32_t* __restrict__ ptr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > N) return;
    int64_t lo = 0, hi = E;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (sorted[mid] < i) lo = mid + 1; else hi = mid;
    }
    ptr[i] = (int32_t)lo;
}

size_t radix_tmp_bytes(int64_t E) {
    size_t b = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, b, (const int32_t*)nullptr, (int32_t*)nullptr,
                                       (const int32_t*)nullptr, (int32_t*)nullptr, (int)E);
    return b;
}

size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

template <class T>
__global__ void permute_rows_kernel(const void* __restrict__ in, void* __restrict__ out,
                                    const int32_t* __restrict__ idx, int64_t rows, int cols, int in_dt,
                                    int scatter) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= rows * cols) return;
    const int64_t k = g / cols;
    const int c = (int)(g - k * cols);
    const int64_t src = scatter ? k : (int64_t)idx[k];
    const int64_t dst = scatter ? (int64_t)idx[k] : k;
    reinterpret_cast<T*>(out)[dst * cols + c] = from_f<T>(load_any(in, in_dt, src * cols + c));
}

template <class T>
__global__ void segment_sum_kernel(const T* __restrict__ src, const int32_t* __restrict__ ptr, int64_t S,
                                   int cols, T* __restrict__ out) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= S * cols) return;
    const int64_t s = g / cols;
    const int c = (int)(g - s * cols);
    float acc = 0.f;
    for (int k = ptr[s]; k < ptr[s + 1]; ++k) acc += to_f(src[(int64_t)k * cols + c]);
    out[g] = from_f<T>(acc);
}

// The same sums, one thread per (segment, 16-byte chunk of a row): the 16 (bf16) / 32 (fp32) threads
// of a row read it as one coalesced 256 / 512-byte line, 4 rows in flight per thread; each element is
// still summed over k in increasing order in fp32 (bit-identical to segment_sum_kernel).
template <class T>
__global__ __launch_bounds__(256) void segment_sum_vec_kernel(const T* __restrict__ src, const int32_t* __restrict__ ptr,
                                                              int64_t S, int cols, T* __restrict__ out) {
    constexpr int CH = Chunk<T>::N;
    const int cpr = cols / CH;
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= S * cpr) return;
    const int64_t s = g / cpr;
    const int c = (int)(g - s * cpr) * CH;
    const int kb = ptr[s], ke = ptr[s + 1];
    float acc[CH];
#pragma unroll
    for (int e = 0; e < CH; ++e) acc[e] = 0.f;
    int k = kb;
    for (; k + 4 <= ke; k += 4) {
        float t[4][CH];
#pragma unroll
        for (int u = 0; u < 4; ++u) Chunk<T>::load(src + (int64_t)(k + u) * cols + c, t[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int e = 0; e < CH; ++e) acc[e] += t[u][e];
    }
    for (; k < ke; ++k) {
        float t[CH];
        Chunk<T>::load(src + (int64_t)k * cols + c, t);
#pragma unroll
        for (int e = 0; e < CH; ++e) acc[e] += t[e];
    }
    Chunk<T>::store(out + s * cols + c, acc);
}

// torch.optim.AdamW (single-tensor path) op for op, fp32, no FMA contraction so the rounding
// sequence is the one ATen's CPU kernels produce.
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                    float decay, float w1, float beta2, float omb2,
                                                    float bc2_sqrt, float eps, float neg_step) {
#pragma clang fp contract(off)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        float pi = p[i] * decay;
        const float gi = g[i];
        float mi = m[i];
        mi = fmaf(w1, gi - mi, mi);  // lerp(exp_avg, grad, 1-beta1): ATen's vectorised fmadd form
        float vi = v[i] * beta2;
        vi = vi + (omb2 * gi) * gi;  // addcmul(value=1-beta2)
        const float den = sqrtf(vi) / bc2_sqrt + eps;
        pi = pi + neg_step * (mi / den);  // addcdiv(value=-step_size)
        p[i] = pi;
        m[i] = mi;
        v[i] = vi;
    }
}

// Same update with lr and step read from device memory (double[2] = {lr, step}) so a captured
// hipGraph replays correct schedules: the host refreshes the two doubles before each replay.
__global__ __launch_bounds__(256) void adamw_dev_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                        const double* __restrict__ hyper, double beta1,
                                                        double beta2, double eps, double wd, unsigned* err,
                                                        int count_skip) {
#pragma clang fp contract(off)
    if (err) {  // a pending validation error: the reference raised before its optimizer step
        const unsigned e = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (e & MGN_ERR_ANY) {
            if (blockIdx.x == 0 && threadIdx.x == 0) {
                // one count per optimizer STEP: of a step's launches (one per parameter group /
                // parameter) only the first has count_skip set (mgn_adamw_dev2)
                if (count_skip && (e & MGN_ERR_SKIP_MASK) != MGN_ERR_SKIP_MASK) atomicAdd(err, MGN_ERR_SKIP_ONE);
                atomicOr(err, MGN_ERR_STALE);
            }
            return;
        }
    }
    const double lr = hyper[0], step = hyper[1];
    const double bc1 = 1.0 - pow(beta1, step), bc2 = 1.0 - pow(beta2, step);
    const float decay = (float)(1.0 - lr * wd), w1 = (float)(1.0 - beta1), b2 = (float)beta2;
    const float omb2 = (float)(1.0 - beta2), bc2s = (float)sqrt(bc2), epsf = (float)eps;
    const float neg_step = (float)(-(lr / bc1));
    auto upd = [&](float& pi, float gi, float& mi, float& vi) {
        pi = pi * decay;
        mi = fmaf(w1, gi - mi, mi);
        vi = vi * b2;
        vi = vi + (omb2 * gi) * gi;
        const float den = sqrtf(vi) / bc2s + epsf;
        pi = pi + neg_step * (mi / den);
    };
    // 16-byte vectors, several per thread: the double-precision schedule setup above is per thread,
    // so each thread amortises it over many elements (scalar loop when a buffer is not 16-byte aligned)
    const bool vec = (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0;
    const int64_t n4 = vec ? n / 4 : 0, stride = (int64_t)gridDim.x * blockDim.x, t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int64_t i = t0; i < n4; i += stride) {
        f4 P = reinterpret_cast<f4*>(p)[i], M = reinterpret_cast<f4*>(m)[i], V = reinterpret_cast<f4*>(v)[i];
        const f4 G = reinterpret_cast<const f4*>(g)[i];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float pi = P[r], mi = M[r], vi = V[r];
            upd(pi, G[r], mi, vi);
            P[r] = pi, M[r] = mi, V[r] = vi;
        }
        reinterpret_cast<f4*>(p)[i] = P;
        reinterpret_cast<f4*>(m)[i] = M;
        reinterpret_cast<f4*>(v)[i] = V;
    }
    for (int64_t i = 4 * n4 + t0; i < n; i += stride) {
        float pi = p[i], mi = m[i], vi = v[i];
        upd(pi, g[i], mi, vi);
        p[i] = pi, m[i] = mi, v[i] = vi;
    }
}

}  // namespace


// Column statistics of a row-major fp32 matrix: per block, fixed row range, per-thread strided rows,
// LDS tree in fixed order -> part[block][2*cols] (sum, sum of squares); a one-block pass then sums
// the partials in block order. Deterministic for given (rows, cols).
constexpr int STAT_MAXC = 32;
constexpr int STAT_BLOCKS = 256;

__global__ __launch_bounds__(256) void colstats_partial(const float* __restrict__ x, int64_t rows, int cols, int64_t ld,
                                                        int64_t rows_per_block, float* __restrict__ part) {
    __shared__ float red[256];
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = r0 + rows_per_block < rows ? r0 + rows_per_block : rows;
    for (int c = 0; c < cols; ++c) {
        float s = 0.f, s2 = 0.f;
        for (int64_t r = r0 + threadIdx.x; r < r1; r += 256) {
            const float v = x[r * ld + c];
            s += v;
            s2 = fmaf(v, v, s2);
        }
        for (int pass = 0; pass < 2; ++pass) {
            red[threadIdx.x] = pass ? s2 : s;
            __syncthreads();
            for (int w = 128; w > 0; w >>= 1) {
                if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
                __syncthreads();
            }
            if (threadIdx.x == 0) part[(int64_t)blockIdx.x * 2 * cols + pass * cols + c] = red[0];
            __syncthreads();
        }
    }
}

// Σ_b part[b][i] over nblocks <= 256 partial rows by one wave: lane-strided partials, then a fixed
// xor butterfly (every lane ends with the same total; deterministic).
__device__ __forceinline__ float partial_total(const float* __restrict__ part, int nblocks, int cols, int i,
                                               int lane) {
    float t = 0.f;
    for (int b = lane; b < nblocks; b += 64) t += part[(int64_t)b * 2 * cols + i];
#pragma unroll
    for (int w = 32; w > 0; w >>= 1) t += __shfl_xor(t, w);
    return t;
}

// the 2*cols totals, one wave per output (4 waves)
__global__ __launch_bounds__(256) void colstats_final(const float* __restrict__ part, int nblocks, int cols,
                                                      float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x >> 6; i < 2 * cols; i += 4) {
        const float t = partial_total(part, nblocks, cols, i, lane);
        if (lane == 0) out[i] = t;
    }
}

// Normalizer.forward (reference layers.py:265-392): one block finishes the batch column sums
// (same block order as colstats_final) or takes the caller's pending {Σx, Σx², count}, applies
// _accumulate to the module's fp32 buffers exactly as the torch expressions do (acc += live ? s : 0,
// live = num_acc < max_acc), and leaves mean / max(sqrt(max(var, 0)), eps) per column in mstd for
// the elementwise pass.
__device__ __forceinline__ void normalizer_update_body(const float* __restrict__ part, int nblocks, int cols,
                                                       const float* __restrict__ pending, float rows_f,
                                                       int accumulate, float* acc_sum, float* acc_sum_sq,
                                                       float* acc_count, float* num_acc, float max_acc, float eps,
                                                       float* __restrict__ mstd, bool skip = false) {
#pragma clang fp contract(off)  // one rounding per torch op: no fused multiply-adds here
    __shared__ float tot[2 * 32];
    const int i = threadIdx.x;
    const float count_old = *acc_count, num_old = *num_acc;
    // skip: a validation error is pending on the device word — the reference raised before this
    // normalizer accumulated, so the buffers stay as they are (the outputs are never used)
    if (skip) accumulate = 0;
    if (accumulate && !pending)
        for (int o = threadIdx.x >> 6; o < 2 * cols; o += 4) {
            const float t = partial_total(part, nblocks, cols, o, threadIdx.x & 63);
            if ((threadIdx.x & 63) == 0) tot[o] = t;
        }
    __syncthreads();  // totals in LDS; every thread has read the old scalars before thread 0 writes them
    const bool live = accumulate && num_old < max_acc;
    float cnt = 0.f;
    if (accumulate) cnt = pending ? pending[2 * cols] : rows_f;
    const float count_new = count_old + (live ? cnt : 0.f);
    if (i < cols) {
        float sm = acc_sum[i], sq = acc_sum_sq[i];
        if (accumulate) {
            float s = 0.f, s2 = 0.f;
            if (pending) {
                s = pending[i];
                s2 = pending[cols + i];
            } else {
                s = tot[i];
                s2 = tot[cols + i];
            }
            sm = sm + (live ? s : 0.f);
            sq = sq + (live ? s2 : 0.f);
            acc_sum[i] = sm;
            acc_sum_sq[i] = sq;
        }
        const float c1 = count_new < 1.f ? 1.f : count_new;  // clamp(min=1)
        const float mean = sm / c1;
        const float var = sq / c1 - mean * mean;
        const float sd = sqrtf(var < 0.f ? 0.f : var);
        mstd[i] = mean;
        mstd[cols + i] = sd != sd ? sd : (sd < eps ? eps : sd);  // torch.max: NaN propagates
    }
    if (i == 0 && accumulate) {
        *acc_count = count_new;
        *num_acc = num_old + (live ? 1.f : 0.f);
    }
}

__global__ __launch_bounds__(256) void normalizer_update(const float* __restrict__ part, int nblocks, int cols,
                                                        const float* __restrict__ pending, float rows_f,
                                                        int accumulate, float* acc_sum, float* acc_sum_sq,
                                                        float* acc_count, float* num_acc, float max_acc, float eps,
                                                        float* __restrict__ mstd) {
    normalizer_update_body(part, nblocks, cols, pending, rows_f, accumulate, acc_sum, acc_sum_sq, acc_count, num_acc,
                           max_acc, eps, mstd);
}

// ----------------------------------------------------------------------- fused Simulator preamble
// The three Normalizer.forward calls of Simulator._build_input_graph (simulator.py:206-290) on
// "virtual" matrices read straight from x / y / edge_attr: source 0 = target delta y - x[:, os:oe],
// source 1 = node features [x[:, fs:fe] ‖ one_hot(x[:, nti], n_types)], source 2 = edge_attr. Each
// source's statistics use mgn_column_stats' partition and order, so every sum, buffer and output is
// bit-identical to the unfused torch + mgn_normalizer_forward path; 3 launches instead of ~15.
struct PreSrc {
    const float* a;     // src 0: y, 1: x, 2: edge_attr
    const float* b;     // src 0: x (pre-target), else unused
    int64_t rows, lda, ldb;
    int32_t cols, off_a, off_b, nf, nti, ntypes;  // src 1: nf feature columns at off_a, type column nti
    int64_t rpb;        // rows per statistics block
    int32_t nb, blk0;   // statistics blocks, first block index in the launch
    float* part;        // [nb][2*cols]
    float* mstd;        // [2*cols]
    float* out;         // [rows][cols]
    const float* pending;
    float *acc_sum, *acc_sum_sq, *acc_count, *num_acc;
    float max_acc, eps;
};
struct PreArgs {
    PreSrc s[3];
    unsigned* err;  // device error word (MGN_ERR_TYPE_*), or NULL
    int32_t nsrc, accumulate;
    int64_t apply0[4];  // flat element offsets of the sources in the apply launch
};

__device__ __forceinline__ float pre_value(const PreSrc& q, int which, int64_t r, int c) {
    if (which == 0) return q.a[r * q.lda + q.off_a + c] - q.b[r * q.ldb + q.off_b + c];
    if (which == 1) {
        if (c < q.nf) return q.a[r * q.lda + q.off_a + c];
        const int64_t t = (int64_t)q.a[r * q.lda + q.nti];  // node_type.long() (truncation)
        return t == (int64_t)(c - q.nf) ? 1.f : 0.f;
    }
    return q.a[r * q.lda + c];
}

// F.one_hot(node_type.long(), n_types) validation (reference simulator.py one-hot; ATen raises
// "Class values must be non-negative." / "... smaller than num_classes."): flag the error word
// instead of reading back to the host; the row's one-hot stays all-zero, so every access is in range.
__device__ __forceinline__ void check_type(const PreSrc& q, int64_t r, unsigned* err) {
    if (!err) return;
    const float t = truncf(q.a[r * q.lda + q.nti]);
    if (!(t >= 0.f)) atomicOr(err, MGN_ERR_TYPE_NEG);  // negative or NaN
    else if (t >= (float)q.ntypes) atomicOr(err, MGN_ERR_TYPE_BIG);
}

__global__ __launch_bounds__(256) void preamble_stats(PreArgs a) {
    // colstats_partial's per-column arithmetic and tree order, all columns' trees advanced together
    // (one barrier per level instead of two trees per column)
    __shared__ float red[2 * STAT_MAXC][256];
    int w = 0;
    while (w + 1 < a.nsrc && (int)blockIdx.x >= a.s[w + 1].blk0) ++w;
    const PreSrc& q = a.s[w];
    const int64_t b = (int64_t)blockIdx.x - q.blk0;
    const int64_t r0 = b * q.rpb;
    const int64_t r1 = r0 + q.rpb < q.rows ? r0 + q.rpb : q.rows;
    const int cols = q.cols;
    for (int c = 0; c < cols; ++c) {
        float s = 0.f, s2 = 0.f;
        for (int64_t r = r0 + threadIdx.x; r < r1; r += 256) {
            const float v = pre_value(q, w, r, c);
            s += v;
            s2 = fmaf(v, v, s2);
        }
        if (w == 1 && c == q.nf)
            for (int64_t r = r0 + threadIdx.x; r < r1; r += 256) check_type(q, r, a.err);
        red[c][threadIdx.x] = s;
        red[cols + c][threadIdx.x] = s2;
    }
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k)
            for (int c = 0; c < 2 * cols; ++c) red[c][threadIdx.x] += red[c][threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x < 2 * cols) q.part[b * 2 * cols + threadIdx.x] = red[threadIdx.x][0];
}

__device__ __forceinline__ unsigned load_err(const unsigned* err) {
    return err ? __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
}

__global__ __launch_bounds__(256) void preamble_update(PreArgs a) {
    const PreSrc& q = a.s[blockIdx.x];
    // reference order (simulator.py _build_input_graph): the output normalizer accumulates, THEN
    // F.one_hot validates the node types, then the node / edge normalizers accumulate. An error of
    // THIS step (type bits set by preamble_stats, or an earlier unraised one) stops the node / edge
    // updates; the output normalizer stops only for an error of an earlier step (MGN_ERR_STALE).
    const unsigned e = load_err(a.err);
    const bool skip = blockIdx.x == 0 ? (e & MGN_ERR_STALE) != 0u : (e & (MGN_ERR_ANY | MGN_ERR_STALE)) != 0u;
    normalizer_update_body(q.part, q.nb, q.cols, q.pending, (float)q.rows, a.accumulate, q.acc_sum, q.acc_sum_sq,
                           q.acc_count, q.num_acc, q.max_acc, q.eps, q.mstd, skip);
}

// batch statistics only (the data-parallel prologue): per source {Σx, Σx², rows}, packed in source
// order, with colstats_final's order over the partial rows
__global__ __launch_bounds__(256) void preamble_stats_final(PreArgs a, float* __restrict__ packed) {
    const PreSrc& q = a.s[blockIdx.x];
    int64_t off = 0;
    for (int i = 0; i < (int)blockIdx.x; ++i) off += 2 * a.s[i].cols + 1;
    const int lane = threadIdx.x & 63;
    for (int o = threadIdx.x >> 6; o < 2 * q.cols; o += 4) {
        const float t = partial_total(q.part, q.nb, q.cols, o, lane);
        if (lane == 0) packed[off + o] = t;
    }
    if (threadIdx.x == 0) packed[off + 2 * q.cols] = (float)q.rows;
}

__global__ __launch_bounds__(256) void preamble_apply(PreArgs a) {
#pragma clang fp contract(off)
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.apply0[a.nsrc]) return;
    int w = 0;
    while (w + 1 < a.nsrc && k >= a.apply0[w + 1]) ++w;
    const PreSrc& q = a.s[w];
    const int64_t i = k - a.apply0[w];
    const int64_t r = i / q.cols;
    const int c = (int)(i - r * q.cols);
    if (w == 1 && c == q.nf) check_type(q, r, a.err);
    q.out[i] = (pre_value(q, w, r, c) - q.mstd[c]) / q.mstd[q.cols + c];
}

__global__ __launch_bounds__(256) void normalizer_apply(const float* __restrict__ x, int64_t rows, int cols,
                                                        int64_t ld, const float* __restrict__ mstd,
                                                        float* __restrict__ out) {
#pragma clang fp contract(off)
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= rows * cols) return;
    const int64_t r = k / cols;
    const int c = (int)(k - r * cols);
    out[k] = (x[r * ld + c] - mstd[c]) / mstd[cols + c];
}

// Masked L2 loss (reference utils/loss.py:10-65 in its masked_mse form): one block, rows strided
// over the threads, fixed-order tree: deterministic.
__device__ __forceinline__ float type_mask_of(const float* nt, int64_t ld, int64_t r, unsigned tmask) {
    const float v = nt[r * ld];
    const int t = (int)v;
    return (v == (float)t && t >= 0 && t < 32 && ((tmask >> t) & 1u)) ? 1.f : 0.f;
}

// partial sums per block (fixed row range, strided threads, LDS tree) -> part[block] = {Σ m·err, Σ m}
constexpr int MSE_BLOCKS = 64;
__global__ __launch_bounds__(256) void masked_mse_partial(const float* __restrict__ pred,
                                                          const float* __restrict__ tgt, int64_t rows, int cols,
                                                          const float* __restrict__ nt, int64_t nt_ld,
                                                          unsigned tmask, int64_t rows_per_block,
                                                          float* __restrict__ part) {
    __shared__ float ra[256], rc[256];
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = r0 + rows_per_block < rows ? r0 + rows_per_block : rows;
    float acc = 0.f, cnt = 0.f;
    for (int64_t r = r0 + threadIdx.x; r < r1; r += 256) {
        const float m = type_mask_of(nt, nt_ld, r, tmask);
        float e = 0.f;
        for (int c = 0; c < cols; ++c) {
            const float d = pred[r * cols + c] - tgt[r * cols + c];
            e += d * d;
        }
        acc += m * e;
        cnt += m;
    }
    ra[threadIdx.x] = acc;
    rc[threadIdx.x] = cnt;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            ra[threadIdx.x] += ra[threadIdx.x + w];
            rc[threadIdx.x] += rc[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = ra[0];
        part[2 * blockIdx.x + 1] = rc[0];
    }
}

__global__ __launch_bounds__(64) void masked_mse_final(const float* __restrict__ part, int nblocks, int cols,
                                                       const float* count_dev, float* loss, float* count_out) {
    const int lane = threadIdx.x;
    float a = 0.f, c = 0.f;
    for (int b = lane; b < nblocks; b += 64) {
        a += part[2 * b];
        c += part[2 * b + 1];
    }
#pragma unroll
    for (int w = 32; w > 0; w >>= 1) {
        a += __shfl_xor(a, w);
        c += __shfl_xor(c, w);
    }
    if (lane == 0) {
        const float cc = count_dev ? *count_dev : c;
        *loss = a / (cc * (float)cols);
        if (count_out) *count_out = cc;
    }
}

__global__ __launch_bounds__(256) void masked_mse_bwd(const float* __restrict__ pred, const float* __restrict__ tgt,
                                                      int64_t rows, int cols, const float* __restrict__ nt,
                                                      int64_t nt_ld, unsigned tmask, const float* count,
                                                      const float* gout, float* __restrict__ grad) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= rows * cols) return;
    const int64_t r = k / cols;
    const float m = type_mask_of(nt, nt_ld, r, tmask);
    const float scale = (gout ? *gout : 1.f) / (*count * (float)cols);
    grad[k] = m != 0.f ? scale * (2.f * (pred[k] - tgt[k])) : 0.f;
}

extern "C" {

int mgn_adamw_dev2(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                   const double* hyper, double beta1, double beta2, double eps, double weight_decay,
                   uint32_t* err_word, int32_t count_skip, mgn_stream_t stream) {
    if (n == 0) return 0;
    int64_t blocks = cdiv64(cdiv64(n, 4), 256);
    if (blocks > 512) blocks = 512;
    ProfScope ps(PROF_ADAMW, (hipStream_t)stream);
    hipLaunchKernelGGL(adamw_dev_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, param, grad,
                       exp_avg, exp_avg_sq, n, hyper, beta1, beta2, eps, weight_decay, (unsigned*)err_word,
                       (int)(count_skip != 0));
    MGN_LAUNCH_CHECK();
    return 0;
}

int mgn_adamw_dev(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                  const double* hyper, double beta1, double beta2, double eps, double weight_decay,
                  uint32_t* err_word, mgn_stream_t stream) {
    return mgn_adamw_dev2(param, grad, exp_avg, exp_avg_sq, n, hyper, beta1, beta2, eps, weight_decay, err_word, 1,
                          stream);
}

int mgn_abi_version(void) { return MGN_ABI_VERSION; }
const char* mgn_last_error(void) { return g_err.c_str(); }

size_t mgn_topology_workspace_bytes(int64_t E, int64_t N) {
    (void)N;
    return al(sizeof(unsigned)) + 4 * al((size_t)E * 4) + al(radix_tmp_bytes(E));
}

// edge_index validation flags MGN_ERR_EDGE_INDEX into the caller's device word (no host read-back);
// out-of-range indices are clamped into [0, N) so every later kernel stays in bounds.
int mgn_topology_build_async(const int64_t* edge_index, int64_t E, int64_t N, int32_t* csc_src, int32_t* csc_dst,
                             int32_t* csc_eid, int32_t* col_ptr, int32_t* row_ptr, int32_t* row_perm, void* ws,
                             size_t ws_bytes, uint32_t* err_word, mgn_stream_t stream) {
    MGN_REQUIRE(N >= 0 && E >= 0 && N < (1ll << 31) && E < (1ll << 31), "graph too large for int32 indices");
    MGN_REQUIRE(N > 0 || E == 0, "edge_index out of range (edges on a graph without nodes)");
    MGN_REQUIRE(err_word, "topology: NULL error word");
    MGN_REQUIRE(ws_bytes >= mgn_topology_workspace_bytes(E, N), "topology workspace too small");
    hipStream_t st = (hipStream_t)stream;
    char* w = reinterpret_cast<char*>(ws);
    w += al(sizeof(unsigned));
    int32_t* src = reinterpret_cast<int32_t*>(w); w += al((size_t)E * 4);
    int32_t* dst = reinterpret_cast<int32_t*>(w); w += al((size_t)E * 4);
    int32_t* iota = reinterpret_cast<int32_t*>(w); w += al((size_t)E * 4);
    int32_t* tmpk = reinterpret_cast<int32_t*>(w); w += al((size_t)E * 4);
    void* tmp = w;
    size_t tmp_bytes = radix_tmp_bytes(E);
    const unsigned eb = (unsigned)cdiv64(E, 256);
    if (E > 0) {
        hipLaunchKernelGGL(split_edge_index, dim3(eb), dim3(256), 0, st, edge_index, E, N, src, dst, iota,
                           (unsigned*)err_word);
        MGN_LAUNCH_CHECK();
        // target-sorted order: stable sort of (col, eid)
        MGN_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, dst, csc_dst, iota, csc_eid, (int)E, 0, 32, st));
        hipLaunchKernelGGL(gather_i32, dim3(eb), dim3(256), 0, st, src, csc_eid, E, csc_src);
        MGN_LAUNCH_CHECK();
        // out-edge order: stable sort of target-sorted positions (iota) by source
        MGN_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, csc_src, tmpk, iota, row_perm, (int)E, 0, 32, st));
    }
    const unsigned nb = (unsigned)cdiv64(N + 1, 256);
    hipLaunchKernelGGL(segment_ptr, dim3(nb), dim3(256), 0, st, csc_dst, E, N, col_ptr);
    MGN_LAUNCH_CHECK();
    hipLaunchKernelGGL(segment_ptr, dim3(nb), dim3(256), 0, st, tmpk, E, N, row_ptr);
    MGN_LAUNCH_CHECK();
    return 0;
}

int mgn_topology_build(const int64_t* edge_index, int64_t E, int64_t N, int32_t* csc_src, int32_t* csc_dst,
                       int32_t* csc_eid, int32_t* col_ptr, int32_t* row_ptr, int32_t* row_perm, void* ws,
                       size_t ws_bytes, mgn_stream_t stream) {
    MGN_REQUIRE(ws_bytes >= mgn_topology_workspace_bytes(E, N), "topology workspace too small");
    hipStream_t st = (hipStream_t)stream;
    unsigned* bad = reinterpret_cast<unsigned*>(ws);  // the workspace's first word
    MGN_TRY(hipMemsetAsync(bad, 0, sizeof(unsigned), st));
    const int rc = mgn_topology_build_async(edge_index, E, N, csc_src, csc_dst, csc_eid, col_ptr, row_ptr, row_perm,
                                            ws, ws_bytes, bad, stream);
    if (rc) return rc;
    unsigned hbad = 0;
    MGN_TRY(hipMemcpyAsync(&hbad, bad, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    MGN_TRY(hipStreamSynchronize(st));
    MGN_REQUIRE(hbad == 0, "edge_index out of range");
    return 0;
}

int mgn_permute_rows(const void* in, void* out, const int32_t* idx, int64_t rows, int32_t cols, int32_t in_dtype,
                     int32_t out_dtype, int32_t scatter, mgn_stream_t stream) {
    const int64_t tot = rows * cols;
    if (tot == 0) return 0;
    const unsigned b = (unsigned)cdiv64(tot, 256);
    if (out_dtype == MGN_F32)
        hipLaunchKernelGGL(permute_rows_kernel<float>, dim3(b), dim3(256), 0, (hipStream_t)stream, in, out, idx, rows,
                           cols, in_dtype, scatter);
    else
        hipLaunchKernelGGL(permute_rows_kernel<__bf16>, dim3(b), dim3(256), 0, (hipStream_t)stream, in, out, idx,
                           rows, cols, in_dtype, scatter);
    MGN_LAUNCH_CHECK();
    return 0;
}

int mgn_segment_sum(const void* src, const int32_t* seg_ptr, int64_t S, int32_t cols, int32_t dtype, void* out,
                    mgn_stream_t stream) {
    const int64_t tot = S * cols;
    if (tot == 0) return 0;
    const int ch = dtype == MGN_F32 ? 4 : 8;
    if (cols % ch == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)out & 15) == 0) {
        const unsigned bv = (unsigned)cdiv64(tot / ch, 256);
        if (dtype == MGN_F32)
            hipLaunchKernelGGL(segment_sum_vec_kernel<float>, dim3(bv), dim3(256), 0, (hipStream_t)stream,
                               (const float*)src, seg_ptr, S, cols, (float*)out);
        else
            hipLaunchKernelGGL(segment_sum_vec_kernel<__bf16>, dim3(bv), dim3(256), 0, (hipStream_t)stream,
                               (const __bf16*)src, seg_ptr, S, cols, (__bf16*)out);
        MGN_LAUNCH_CHECK();
        return 0;
    }
    const unsigned b = (unsigned)cdiv64(tot, 256);
    if (dtype == MGN_F32)
        hipLaunchKernelGGL(segment_sum_kernel<float>, dim3(b), dim3(256), 0, (hipStream_t)stream, (const float*)src,
                           seg_ptr, S, cols, (float*)out);
    else
        hipLaunchKernelGGL(segment_sum_kernel<__bf16>, dim3(b), dim3(256), 0, (hipStream_t)stream,
                           (const __bf16*)src, seg_ptr, S, cols, (__bf16*)out);
    MGN_LAUNCH_CHECK();
    return 0;
}

int mgn_adamw(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, double lr, double beta1,
              double beta2, double eps, double weight_decay, int64_t step, mgn_stream_t stream) {
    if (n == 0) return 0;
    MGN_REQUIRE(step >= 1, "AdamW step must be >= 1");
    // host-side scalars exactly as torch/optim/adamw.py computes them (Python doubles)
    const double bc1 = 1.0 - std::pow(beta1, (double)step);
    const double bc2 = 1.0 - std::pow(beta2, (double)step);
    const double step_size = lr / bc1;
    const double bc2_sqrt = std::sqrt(bc2);
    const float decay = (float)(1.0 - lr * weight_decay);
    int64_t blocks = cdiv64(n, 256);
    if (blocks > 4096) blocks = 4096;
    ProfScope ps(PROF_ADAMW, (hipStream_t)stream);
    hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, param, grad, exp_avg,
                       exp_avg_sq, n, decay, (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2),
                       (float)bc2_sqrt, (float)eps, (float)(-step_size));
    MGN_LAUNCH_CHECK();
    return 0;
}


size_t mgn_column_stats_workspace_bytes(int64_t rows, int32_t cols) {
    (void)rows;
    return (size_t)STAT_BLOCKS * 2 * (cols > 0 ? cols : 1) * sizeof(float);
}

int mgn_column_stats(const float* x, int64_t rows, int32_t cols, int64_t ld, float* sums, void* ws, size_t ws_bytes,
                     mgn_stream_t stream) {
    MGN_REQUIRE(cols >= 1 && cols <= STAT_MAXC, "column_stats: cols must be in [1, 32]");
    MGN_REQUIRE(ld >= cols, "column_stats: ld < cols");
    MGN_REQUIRE(ws_bytes >= mgn_column_stats_workspace_bytes(rows, cols), "column_stats: workspace too small");
    hipStream_t st = (hipStream_t)stream;
    int64_t rpb = cdiv64(rows > 0 ? rows : 1, STAT_BLOCKS);
    if (rpb < 256) rpb = 256;
    const int nb = (int)cdiv64(rows > 0 ? rows : 1, rpb);
    float* part = reinterpret_cast<float*>(ws);
    hipLaunchKernelGGL(colstats_partial, dim3(nb), dim3(256), 0, st, x, rows, (int)cols, ld, rpb, part);
    MGN_LAUNCH_CHECK();
    hipLaunchKernelGGL(colstats_final, dim3(1), dim3(256), 0, st, (const float*)part, nb, (int)cols, sums);
    MGN_LAUNCH_CHECK();
    return 0;
}

size_t mgn_normalizer_workspace_bytes(int64_t rows, int32_t cols) {
    return mgn_column_stats_workspace_bytes(rows, cols) + 256;
}

int mgn_normalizer_forward(const float* x, int64_t rows, int32_t cols, int64_t ld, int32_t accumulate,
                           const float* pending, float* acc_sum, float* acc_sum_sq, float* acc_count, float* num_acc,
                           float max_acc, float eps, float* out, void* ws, size_t ws_bytes, mgn_stream_t stream) {
    MGN_REQUIRE(cols >= 1 && cols <= STAT_MAXC, "normalizer: cols must be in [1, 32]");
    MGN_REQUIRE(ld >= cols, "normalizer: ld < cols");
    MGN_REQUIRE(ws_bytes >= mgn_normalizer_workspace_bytes(rows, cols), "normalizer: workspace too small");
    hipStream_t st = (hipStream_t)stream;
    float* mstd = reinterpret_cast<float*>(ws);  // [2 * cols] (256 B)
    float* part = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + 256);
    int nb = 0;
    if (accumulate && !pending && rows > 0) {
        int64_t rpb = cdiv64(rows, STAT_BLOCKS);
        if (rpb < 256) rpb = 256;
        nb = (int)cdiv64(rows, rpb);
        hipLaunchKernelGGL(colstats_partial, dim3(nb), dim3(256), 0, st, x, rows, (int)cols, ld, rpb, part);
        MGN_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(normalizer_update, dim3(1), dim3(256), 0, st, (const float*)part, nb, (int)cols, pending,
                       (float)rows, (int)accumulate, acc_sum, acc_sum_sq, acc_count, num_acc, max_acc, eps, mstd);
    MGN_LAUNCH_CHECK();
    if (rows * cols > 0) {
        hipLaunchKernelGGL(normalizer_apply, dim3((unsigned)cdiv64(rows * cols, 256)), dim3(256), 0, st, x, rows,
                           (int)cols, ld, (const float*)mstd, out);
        MGN_LAUNCH_CHECK();
    }
    return 0;
}

size_t mgn_simulator_preamble_workspace_bytes(int64_t num_nodes, int64_t num_edges) {
    (void)num_nodes;
    (void)num_edges;
    return 3 * (256 + (size_t)STAT_BLOCKS * 2 * STAT_MAXC * sizeof(float));
}

int mgn_simulator_statistics(const float* x, int64_t N, int64_t ldx, int32_t feat_start, int32_t feat_end,
                             int32_t type_index, int32_t n_types, int32_t out_start, int32_t out_end, const float* y,
                             int64_t ldy, const float* edge_attr, int64_t E, int32_t edge_cols, int64_t lde,
                             float* packed, uint32_t* err_word, void* ws, size_t ws_bytes, mgn_stream_t stream) {
    const int nf = feat_end - feat_start, no = out_end - out_start;
    MGN_REQUIRE(x && y && packed, "simulator statistics: NULL argument");
    MGN_REQUIRE(nf >= 0 && n_types >= 1 && nf + n_types <= STAT_MAXC && no >= 1 && no <= STAT_MAXC,
                "simulator statistics: node features and targets must have 1..32 columns");
    MGN_REQUIRE(feat_end <= ldx && out_end <= ldx && type_index >= 0 && type_index < ldx && ldy >= no,
                "simulator statistics: column ranges outside the rows");
    MGN_REQUIRE(!edge_attr || (edge_cols >= 1 && edge_cols <= STAT_MAXC && lde >= edge_cols),
                "simulator statistics: edge_attr must be [E, 1..32]");
    MGN_REQUIRE(ws_bytes >= mgn_simulator_preamble_workspace_bytes(N, E), "simulator statistics: workspace too small");
    hipStream_t st = (hipStream_t)stream;
    PreArgs a;
    memset(&a, 0, sizeof(a));
    a.err = err_word;
    a.nsrc = edge_attr ? 3 : 2;
    char* w = reinterpret_cast<char*>(ws);
    int blocks = 0;
    for (int i = 0; i < a.nsrc; ++i) {
        PreSrc& q = a.s[i];
        if (i == 0) {
            q.a = y, q.b = x, q.rows = N, q.lda = ldy, q.ldb = ldx, q.cols = no, q.off_b = out_start;
        } else if (i == 1) {
            q.a = x, q.rows = N, q.lda = ldx, q.cols = nf + n_types, q.off_a = feat_start, q.nf = nf;
            q.nti = type_index, q.ntypes = n_types;
        } else {
            q.a = edge_attr, q.rows = E, q.lda = lde, q.cols = edge_cols;
        }
        q.part = reinterpret_cast<float*>(w + i * (256 + (size_t)STAT_BLOCKS * 2 * STAT_MAXC * sizeof(float))) + 64;
        q.blk0 = blocks;
        if (q.rows > 0) {  // mgn_column_stats' partition
            q.rpb = cdiv64(q.rows, STAT_BLOCKS);
            if (q.rpb < 256) q.rpb = 256;
            q.nb = (int)cdiv64(q.rows, q.rpb);
        }
        blocks += q.nb;
    }
    if (blocks > 0) {
        hipLaunchKernelGGL(preamble_stats, dim3(blocks), dim3(256), 0, st, a);
        MGN_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(preamble_stats_final, dim3(a.nsrc), dim3(256), 0, st, a, packed);
    MGN_LAUNCH_CHECK();
    return 0;
}

int mgn_simulator_preamble(const float* x, int64_t N, int64_t ldx, int32_t feat_start, int32_t feat_end,
                           int32_t type_index, int32_t n_types, int32_t out_start, int32_t out_end, const float* y,
                           int64_t ldy, const float* edge_attr, int64_t E, int32_t edge_cols, int64_t lde,
                           int32_t accumulate, const mgn_normalizer_state* out_norm,
                           const mgn_normalizer_state* node_norm, const mgn_normalizer_state* edge_norm,
                           float* target_out, float* node_out, float* edge_out, uint32_t* err_word, void* ws,
                           size_t ws_bytes, mgn_stream_t stream) {
    const int nf = feat_end - feat_start, no = out_end - out_start;
    MGN_REQUIRE(x && y && out_norm && node_norm && target_out && node_out, "simulator preamble: NULL argument");
    MGN_REQUIRE(nf >= 0 && n_types >= 1 && nf + n_types <= STAT_MAXC && no >= 1 && no <= STAT_MAXC,
                "simulator preamble: node features and targets must have 1..32 columns");
    MGN_REQUIRE(feat_end <= ldx && out_end <= ldx && type_index >= 0 && type_index < ldx && ldy >= no,
                "simulator preamble: column ranges outside the rows");
    MGN_REQUIRE(!edge_norm || (edge_attr && edge_out && edge_cols >= 1 && edge_cols <= STAT_MAXC && lde >= edge_cols),
                "simulator preamble: edge normalizer needs edge_attr [E, 1..32]");
    MGN_REQUIRE(ws_bytes >= mgn_simulator_preamble_workspace_bytes(N, E), "simulator preamble: workspace too small");
    hipStream_t st = (hipStream_t)stream;
    PreArgs a;
    memset(&a, 0, sizeof(a));
    a.err = err_word;
    a.accumulate = accumulate;
    const mgn_normalizer_state* ns[3] = {out_norm, node_norm, edge_norm};
    a.nsrc = edge_norm ? 3 : 2;
    char* w = reinterpret_cast<char*>(ws);
    int blocks = 0;
    int64_t flat = 0;
    for (int i = 0; i < a.nsrc; ++i) {
        PreSrc& q = a.s[i];
        const mgn_normalizer_state* n = ns[i];
        if (i == 0) {
            q.a = y, q.b = x, q.rows = N, q.lda = ldy, q.ldb = ldx, q.cols = no, q.off_a = 0, q.off_b = out_start;
            q.out = target_out;
        } else if (i == 1) {
            q.a = x, q.rows = N, q.lda = ldx, q.cols = nf + n_types, q.off_a = feat_start, q.nf = nf;
            q.nti = type_index, q.ntypes = n_types, q.out = node_out;
        } else {
            q.a = edge_attr, q.rows = E, q.lda = lde, q.cols = edge_cols, q.out = edge_out;
        }
        q.mstd = reinterpret_cast<float*>(w + i * (256 + (size_t)STAT_BLOCKS * 2 * STAT_MAXC * sizeof(float)));
        q.part = q.mstd + 64;
        q.pending = n->pending;
        q.acc_sum = n->acc_sum, q.acc_sum_sq = n->acc_sum_sq, q.acc_count = n->acc_count, q.num_acc = n->num_acc;
        q.max_acc = n->max_acc, q.eps = n->eps;
        q.blk0 = blocks;
        if (accumulate && !n->pending && q.rows > 0) {  // mgn_column_stats' partition
            q.rpb = cdiv64(q.rows, STAT_BLOCKS);
            if (q.rpb < 256) q.rpb = 256;
            q.nb = (int)cdiv64(q.rows, q.rpb);
        }
        blocks += q.nb;
        a.apply0[i] = flat;
        flat += q.rows * q.cols;
    }
    a.apply0[a.nsrc] = flat;
    for (int i = a.nsrc + 1; i < 4; ++i) a.apply0[i] = flat;
    if (blocks > 0) {
        hipLaunchKernelGGL(preamble_stats, dim3(blocks), dim3(256), 0, st, a);
        MGN_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(preamble_update, dim3(a.nsrc), dim3(256), 0, st, a);
    MGN_LAUNCH_CHECK();
    if (flat > 0) {
        hipLaunchKernelGGL(preamble_apply, dim3((unsigned)cdiv64(flat, 256)), dim3(256), 0, st, a);
        MGN_LAUNCH_CHECK();
    }
    return 0;
}

size_t mgn_masked_mse_workspace_bytes(int64_t rows) {
    (void)rows;
    return 2 * MSE_BLOCKS * sizeof(float);
}

int mgn_masked_mse(const float* pred, const float* target, int64_t rows, int32_t cols, const float* node_type,
                   int64_t nt_ld, uint32_t type_mask, const float* count, float* loss, float* count_out, void* ws,
                   size_t ws_bytes, mgn_stream_t stream) {
    MGN_REQUIRE(cols >= 1, "masked_mse: cols must be >= 1");
    MGN_REQUIRE(ws_bytes >= mgn_masked_mse_workspace_bytes(rows), "masked_mse: workspace too small");
    hipStream_t st = (hipStream_t)stream;
    float* part = reinterpret_cast<float*>(ws);
    int64_t rpb = cdiv64(rows > 0 ? rows : 1, MSE_BLOCKS);
    if (rpb < 256) rpb = 256;
    const int nb = (int)cdiv64(rows > 0 ? rows : 1, rpb);
    hipLaunchKernelGGL(masked_mse_partial, dim3(nb), dim3(256), 0, st, pred, target, rows, (int)cols, node_type,
                       nt_ld, type_mask, rpb, part);
    MGN_LAUNCH_CHECK();
    hipLaunchKernelGGL(masked_mse_final, dim3(1), dim3(64), 0, st, (const float*)part, nb, (int)cols, count, loss,
                       count_out);
    MGN_LAUNCH_CHECK();
    return 0;
}

int mgn_masked_mse_backward(const float* pred, const float* target, int64_t rows, int32_t cols,
                            const float* node_type, int64_t nt_ld, uint32_t type_mask, const float* count,
                            const float* grad_loss, float* grad, mgn_stream_t stream) {
    if (rows * cols == 0) return 0;
    hipLaunchKernelGGL(masked_mse_bwd, dim3((unsigned)cdiv64(rows * cols, 256)), dim3(256), 0, (hipStream_t)stream,
                       pred, target, rows, (int)cols, node_type, nt_ld, type_mask, count, grad_loss, grad);
    MGN_LAUNCH_CHECK();
    return 0;
}

}  // extern "C"
