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

static thread_local std::string g_err;
void mgn_set_error(const std::string& s) { g_err = s; }

namespace {

__global__ void split_edge_index(const int64_t* __restrict__ ei, int64_t E, int64_t N, int32_t* __restrict__ src,
                                 int32_t* __restrict__ dst, int32_t* __restrict__ iota, unsigned* __restrict__ bad) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= E) return;
    const int64_t r = ei[k], c = ei[E + k];
    if (r < 0 || r >= N || c < 0 || c >= N) atomicOr(bad, 1u);
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
                                                        double beta2, double eps, double wd) {
#pragma clang fp contract(off)
    const double lr = hyper[0], step = hyper[1];
    const double bc1 = 1.0 - pow(beta1, step), bc2 = 1.0 - pow(beta2, step);
    const float decay = (float)(1.0 - lr * wd), w1 = (float)(1.0 - beta1), b2 = (float)beta2;
    const float omb2 = (float)(1.0 - beta2), bc2s = (float)sqrt(bc2), epsf = (float)eps;
    const float neg_step = (float)(-(lr / bc1));
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        float pi = p[i] * decay;
        const float gi = g[i];
        float mi = fmaf(w1, gi - m[i], m[i]);
        float vi = v[i] * b2;
        vi = vi + (omb2 * gi) * gi;
        const float den = sqrtf(vi) / bc2s + epsf;
        pi = pi + neg_step * (mi / den);
        p[i] = pi;
        m[i] = mi;
        v[i] = vi;
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

__global__ __launch_bounds__(64) void colstats_final(const float* __restrict__ part, int nblocks, int cols,
                                                     float* __restrict__ out) {
    const int i = threadIdx.x;
    if (i >= 2 * cols) return;
    float t = 0.f;
    for (int b = 0; b < nblocks; ++b) t += part[(int64_t)b * 2 * cols + i];
    out[i] = t;
}

extern "C" {

int mgn_adamw_dev(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                  const double* hyper, double beta1, double beta2, double eps, double weight_decay,
                  mgn_stream_t stream) {
    if (n == 0) return 0;
    int64_t blocks = cdiv64(n, 256);
    if (blocks > 4096) blocks = 4096;
    ProfScope ps(PROF_ADAMW, (hipStream_t)stream);
    hipLaunchKernelGGL(adamw_dev_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, param, grad,
                       exp_avg, exp_avg_sq, n, hyper, beta1, beta2, eps, weight_decay);
    MGN_LAUNCH_CHECK();
    return 0;
}

int mgn_abi_version(void) { return MGN_ABI_VERSION; }
const char* mgn_last_error(void) { return g_err.c_str(); }

size_t mgn_topology_workspace_bytes(int64_t E, int64_t N) {
    (void)N;
    return al(sizeof(unsigned)) + 4 * al((size_t)E * 4) + al(radix_tmp_bytes(E));
}

int mgn_topology_build(const int64_t* edge_index, int64_t E, int64_t N, int32_t* csc_src, int32_t* csc_dst,
                       int32_t* csc_eid, int32_t* col_ptr, int32_t* row_ptr, int32_t* row_perm, void* ws,
                       size_t ws_bytes, mgn_stream_t stream) {
    MGN_REQUIRE(N >= 0 && E >= 0 && N < (1ll << 31) && E < (1ll << 31), "graph too large for int32 indices");
    MGN_REQUIRE(ws_bytes >= mgn_topology_workspace_bytes(E, N), "topology workspace too small");
    hipStream_t st = (hipStream_t)stream;
    char* w = reinterpret_cast<char*>(ws);
    unsigned* bad = reinterpret_cast<unsigned*>(w);
    w += al(sizeof(unsigned));
    int32_t* src = reinterpret_cast<int32_t*>(w); w += al((size_t)E * 4);
    int32_t* dst = reinterpret_cast<int32_t*>(w); w += al((size_t)E * 4);
    int32_t* iota = reinterpret_cast<int32_t*>(w); w += al((size_t)E * 4);
    int32_t* tmpk = reinterpret_cast<int32_t*>(w); w += al((size_t)E * 4);
    void* tmp = w;
    size_t tmp_bytes = radix_tmp_bytes(E);
    MGN_TRY(hipMemsetAsync(bad, 0, sizeof(unsigned), st));
    const unsigned eb = (unsigned)cdiv64(E, 256);
    if (E > 0) {
        hipLaunchKernelGGL(split_edge_index, dim3(eb), dim3(256), 0, st, edge_index, E, N, src, dst, iota, bad);
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
    hipLaunchKernelGGL(colstats_final, dim3(1), dim3(64), 0, st, (const float*)part, nb, (int)cols, sums);
    MGN_LAUNCH_CHECK();
    return 0;
}

}  // extern "C"
