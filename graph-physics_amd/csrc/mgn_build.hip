// On-device graph construction, gfx950.
//
// The reference builds every training sample's graph on the host, per sample, with
// torch-geometric 2.6.1 transforms and torch.sparse / scipy:
//   FaceToEdge(remove_faces=False) → to_undirected       preprocessing.py:16-23,410-431
//       (tetrahedra first split into 4 triangles         torch_graph.py:171-186)
//   k-hop augmentation  A_k ← coalesce(A_k + A_k·A), self loops dropped   torch_graph.py:16-53
//   Cartesian(norm=False) ‖ Distance(norm=False)         preprocessing.py:16-23
//   add_world_pos_features (relative world pos + norm)   preprocessing.py:143-174
//   add_world_edges: cKDTree.query_pairs(r) filtered to OBSTACLE–NORMAL pairs, then
//       to_undirected                                     preprocessing.py:92-140
//
// Here all of it is integer/byte work on HBM-resident arrays: every edge set is a list of 64-bit
// keys row·N + col, and "coalesce" is one radix sort of the keys + a flag/select pass + a split
// into the reference's [2, E] int64 layout (sorted by (row, col), duplicates removed — exactly the
// order torch's coalesce() and PyG's to_undirected produce). k-hop expands A_k·A by a CSR walk of
// A (one thread per A_k edge, degree-length runs), radius pairs use a uniform grid of cell size r
// sorted by cell key (27-cell queries, fp64 distance like cKDTree). No GEMM, no floating-point
// reduction order to match: results are bit-identical to the reference's index sets.
//
// Output sizes are data-dependent: each entry point returns the count to the host (one
// synchronisation, as the reference's own .coalesce()/.nonzero() do).
#include <hipcub/hipcub.hpp>

#include <cmath>

#include "mgn_common.h"

namespace {

size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

int key_bits(int64_t n) {  // bits of the largest key n·n − 1
    if (n <= 1) return 1;
    const unsigned long long mx = (unsigned long long)(n - 1) * (unsigned long long)n + (unsigned long long)(n - 1);
    int b = 0;
    while (b < 64 && (mx >> b) != 0) ++b;
    return b;
}

// ---------------------------------------------------------------------------------- key kernels
// cells [k, C] row-major (reference Data.face / tetra layout). k = 3: PyG FaceToEdge pairs
// (face[0],face[1]), (face[1],face[2]), (face[0],face[2]); k = 4: the reference's 4 triangles
// [c0c1c2], [c1c2c3], [c2c3c0], [c3c0c1] (torch_graph.py:173-181), each giving those 3 pairs.
// Every pair is emitted in both directions (to_undirected).
__global__ void cells_to_keys(const int64_t* __restrict__ cells, int k, int64_t C, int64_t N,
                              unsigned long long* __restrict__ keys, unsigned* __restrict__ bad) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    int64_t v[4];
    bool ok = true;
    for (int i = 0; i < k; ++i) {
        v[i] = cells[(int64_t)i * C + c];
        if (v[i] < 0 || v[i] >= N) { ok = false; v[i] = 0; }
    }
    if (!ok) atomicOr(bad, 1u);
    const int nf = k == 4 ? 4 : 1;
    unsigned long long* o = keys + c * (int64_t)(6 * nf);
    for (int f = 0; f < nf; ++f) {
        int64_t a, b, d;
        if (k == 3) { a = v[0]; b = v[1]; d = v[2]; }
        else if (f == 0) { a = v[0]; b = v[1]; d = v[2]; }
        else if (f == 1) { a = v[1]; b = v[2]; d = v[3]; }
        else if (f == 2) { a = v[2]; b = v[3]; d = v[0]; }
        else { a = v[3]; b = v[0]; d = v[1]; }
        const int64_t pr[3][2] = {{a, b}, {b, d}, {a, d}};
        for (int p = 0; p < 3; ++p) {
            o[6 * f + 2 * p] = (unsigned long long)(pr[p][0] * N + pr[p][1]);
            o[6 * f + 2 * p + 1] = (unsigned long long)(pr[p][1] * N + pr[p][0]);
        }
    }
}

// edge_index [2, E] → keys (and the reversed keys at [E, 2E) when symmetrizing)
__global__ void edges_to_keys(const int64_t* __restrict__ ei, int64_t E, int64_t N, int sym,
                              unsigned long long* __restrict__ keys, unsigned* __restrict__ bad) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= E) return;
    int64_t r = ei[k], c = ei[E + k];
    if (r < 0 || r >= N || c < 0 || c >= N) { atomicOr(bad, 1u); r = 0; c = 0; }
    keys[k] = (unsigned long long)(r * N + c);
    if (sym) keys[E + k] = (unsigned long long)(c * N + r);
}

// keep the first of every run of equal sorted keys; optionally drop the diagonal
__global__ void unique_flags(const unsigned long long* __restrict__ s, int64_t M, int64_t N, int drop_self,
                             unsigned char* __restrict__ flag) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= M) return;
    const unsigned long long v = s[k];
    bool keep = k == 0 || s[k - 1] != v;
    if (drop_self && (int64_t)(v / (unsigned long long)N) == (int64_t)(v % (unsigned long long)N)) keep = false;
    flag[k] = keep ? 1 : 0;
}

// unique keys → [2, E] int64 (row block then col block), E read on the device
__global__ void split_keys(const unsigned long long* __restrict__ u, const int* __restrict__ num, int64_t M,
                           int64_t N, int64_t* __restrict__ out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t E = *num;
    if (k >= E || k >= M) return;
    const unsigned long long v = u[k];
    out[k] = (int64_t)(v / (unsigned long long)N);
    out[E + k] = (int64_t)(v % (unsigned long long)N);
}

// ptr[i] = lower_bound(rows, i), i in [0, N]  (rows = edge_index[0] of a coalesced edge list)
__global__ void row_ptr_i64(const int64_t* __restrict__ rows, int64_t E, int64_t N, int64_t* __restrict__ ptr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > N) return;
    int64_t lo = 0, hi = E;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (rows[mid] < i) lo = mid + 1; else hi = mid;
    }
    ptr[i] = lo;
}

// candidates of one hop for A_k edge k = (r, c): itself + (r, A.col[t]) for t in A's row c
__global__ void khop_count(const int64_t* __restrict__ eik, int64_t Ek, const int64_t* __restrict__ aptr, int64_t N,
                           int64_t* __restrict__ cnt, unsigned* __restrict__ bad) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= Ek) return;
    const int64_t r = eik[k], c = eik[Ek + k];
    if (r < 0 || r >= N || c < 0 || c >= N) { atomicOr(bad, 1u); cnt[k] = 0; return; }
    cnt[k] = 1 + aptr[c + 1] - aptr[c];
}

__global__ void khop_expand(const int64_t* __restrict__ eik, int64_t Ek, const int64_t* __restrict__ acol,
                            const int64_t* __restrict__ aptr, const int64_t* __restrict__ off, int64_t N,
                            unsigned long long* __restrict__ keys) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= Ek) return;
    const int64_t r = eik[k], c = eik[Ek + k];
    if (r < 0 || r >= N || c < 0 || c >= N) return;  // flagged by khop_count; no candidates
    unsigned long long* o = keys + off[k];
    const unsigned long long base = (unsigned long long)(r * N);
    o[0] = base + (unsigned long long)c;
    const int64_t b = aptr[c], e = aptr[c + 1];
    for (int64_t t = b; t < e; ++t) o[1 + t - b] = base + (unsigned long long)acol[t];
}

// --------------------------------------------------------------------------------- edge features
// out[k, 0:dim] = pos[row] − pos[col]; out[k, dim] = ‖·‖₂   (Cartesian(norm=False) ‖ Distance(norm=False);
// add_world_pos_features: world_pos[senders] − world_pos[receivers] ‖ norm, preprocessing.py:163-167)
__global__ void edge_features_kernel(const float* __restrict__ pos, int64_t ld, int dim,
                                     const int64_t* __restrict__ ei, int64_t E, float* __restrict__ out,
                                     int64_t out_ld) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= E) return;
    const int64_t r = ei[k], c = ei[E + k];
    float s = 0.f;
    for (int d = 0; d < dim; ++d) {
        const float v = pos[r * ld + d] - pos[c * ld + d];
        out[k * out_ld + d] = v;
        s += v * v;
    }
    out[k * out_ld + dim] = sqrtf(s);
}

__global__ void check_edge_range(const int64_t* __restrict__ ei, int64_t E, int64_t N, unsigned* __restrict__ bad) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= E) return;
    const int64_t r = ei[k], c = ei[E + k];
    if (r < 0 || r >= N || c < 0 || c >= N) atomicOr(bad, 1u);
}

// ---------------------------------------------------------------------------------- radius pairs
// bounding box of pos[:, 0:dim] (one workgroup, fixed order: exact min/max are order-free anyway)
__global__ __launch_bounds__(1024) void bbox_kernel(const float* __restrict__ pos, int64_t ld, int dim, int64_t N,
                                                    float* __restrict__ box) {
    __shared__ float lo[3][1024], hi[3][1024];
    float l[3] = {INFINITY, INFINITY, INFINITY}, h[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = threadIdx.x; i < N; i += 1024)
        for (int d = 0; d < dim; ++d) {
            const float v = pos[i * ld + d];
            l[d] = fminf(l[d], v);
            h[d] = fmaxf(h[d], v);
        }
    for (int d = 0; d < 3; ++d) { lo[d][threadIdx.x] = l[d]; hi[d][threadIdx.x] = h[d]; }
    __syncthreads();
    for (int s = 512; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s)
            for (int d = 0; d < 3; ++d) {
                lo[d][threadIdx.x] = fminf(lo[d][threadIdx.x], lo[d][threadIdx.x + s]);
                hi[d][threadIdx.x] = fmaxf(hi[d][threadIdx.x], hi[d][threadIdx.x + s]);
            }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        for (int d = 0; d < 3; ++d) { box[d] = lo[d][0]; box[3 + d] = hi[d][0]; }
}

struct Grid {
    double o[3], inv;  // origin, 1 / cell size
    int64_t n[3];      // cells per dim
    int dim;
};

__device__ __forceinline__ void cell_of(const Grid& g, const float* p, int64_t* c) {
    for (int d = 0; d < 3; ++d) {
        if (d < g.dim) {
            int64_t v = (int64_t)floor(((double)p[d] - g.o[d]) * g.inv);
            c[d] = v < 0 ? 0 : (v >= g.n[d] ? g.n[d] - 1 : v);
        } else {
            c[d] = 0;
        }
    }
}

__global__ void cell_keys(const float* __restrict__ pos, int64_t ld, int64_t N, Grid g, int64_t* __restrict__ key,
                          int32_t* __restrict__ iota) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    int64_t c[3];
    cell_of(g, pos + i * ld, c);
    key[i] = (c[2] * g.n[1] + c[1]) * g.n[0] + c[0];
    iota[i] = (int32_t)i;
}

__device__ __forceinline__ int64_t lower_bound_i64(const int64_t* a, int64_t n, int64_t v) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ bool type_ok(const float* nt, int64_t ntld, int filter, int64_t i, int64_t j) {
    if (!filter) return true;
    const float a = nt[i * ntld], b = nt[j * ntld];
    // OBSTACLE (1) – NORMAL (0) in either order (preprocessing.py:123-132)
    return (a == 1.f && b == 0.f) || (a == 0.f && b == 1.f);
}

// mode 0: count pairs (i, j), j > i, ‖p_i − p_j‖ ≤ r; mode 1: write them at off[i]
__global__ void radius_pairs_kernel(const float* __restrict__ pos, int64_t ld, int64_t N, Grid g, double r2,
                                    const int64_t* __restrict__ skey, const int32_t* __restrict__ sid,
                                    const float* __restrict__ nt, int64_t ntld, int filter, int mode,
                                    int64_t* __restrict__ cnt, const int64_t* __restrict__ off,
                                    int64_t* __restrict__ out, int64_t total) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    if (filter) {
        const float a = nt[i * ntld];
        if (a != 0.f && a != 1.f) { if (mode == 0) cnt[i] = 0; return; }
    }
    const float* pi = pos + i * ld;
    int64_t c[3];
    cell_of(g, pi, c);
    int64_t n = 0, w = mode ? off[i] : 0;
    const int zs = g.dim > 2 ? 1 : 0, ys = g.dim > 1 ? 1 : 0;
    for (int dz = -zs; dz <= zs; ++dz) {
        const int64_t cz = c[2] + dz;
        if (cz < 0 || cz >= g.n[2]) continue;
        for (int dy = -ys; dy <= ys; ++dy) {
            const int64_t cy = c[1] + dy;
            if (cy < 0 || cy >= g.n[1]) continue;
            // the dx = -1..1 cells are consecutive keys: one contiguous run of the sorted array
            const int64_t x0 = c[0] > 0 ? c[0] - 1 : 0, x1 = c[0] + 1 < g.n[0] ? c[0] + 1 : g.n[0] - 1;
            const int64_t kb = (cz * g.n[1] + cy) * g.n[0];
            const int64_t b = lower_bound_i64(skey, N, kb + x0), e = lower_bound_i64(skey, N, kb + x1 + 1);
            for (int64_t t = b; t < e; ++t) {
                const int64_t j = sid[t];
                if (j <= i || !type_ok(nt, ntld, filter, i, j)) continue;
                const float* pj = pos + j * ld;
                double d2 = 0.0;
                for (int d = 0; d < g.dim; ++d) {
                    const double v = (double)pi[d] - (double)pj[d];
                    d2 += v * v;
                }
                if (d2 <= r2) {
                    if (mode && w < total) { out[w] = i; out[total + w] = j; }
                    ++n;
                    ++w;
                }
            }
        }
    }
    if (mode == 0) cnt[i] = n;
}

// ------------------------------------------------------------------------------ shared tail
size_t coalesce_tmp_bytes(int64_t M) {
    size_t a = 0, b = 0;
    hipcub::DeviceRadixSort::SortKeys(nullptr, a, (const unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                      (int)M);
    hipcub::DeviceSelect::Flagged(nullptr, b, (const unsigned long long*)nullptr, (const unsigned char*)nullptr,
                                  (unsigned long long*)nullptr, (int*)nullptr, (int)M);
    return a > b ? a : b;
}

// workspace: bad | num | keys[M] | sorted[M] | flags[M] | tmp ; unique keys reuse `keys`
size_t coalesce_ws(int64_t M) {
    return 2 * al(sizeof(int64_t)) + 2 * al((size_t)M * 8) + al((size_t)M) + al(coalesce_tmp_bytes(M));
}

struct CoalesceWs {
    unsigned* bad;
    int* num;
    unsigned long long* keys;
    unsigned long long* sorted;
    unsigned char* flags;
    void* tmp;
    size_t tmp_bytes;
};

CoalesceWs carve(void* ws, int64_t M) {
    char* w = reinterpret_cast<char*>(ws);
    CoalesceWs c;
    c.bad = reinterpret_cast<unsigned*>(w); w += al(sizeof(int64_t));
    c.num = reinterpret_cast<int*>(w); w += al(sizeof(int64_t));
    c.keys = reinterpret_cast<unsigned long long*>(w); w += al((size_t)M * 8);
    c.sorted = reinterpret_cast<unsigned long long*>(w); w += al((size_t)M * 8);
    c.flags = reinterpret_cast<unsigned char*>(w); w += al((size_t)M);
    c.tmp = w;
    c.tmp_bytes = coalesce_tmp_bytes(M);
    return c;
}

// keys (already in c.keys, M of them) → sorted unique [2, E] in out; *num_out = E (host)
int coalesce_tail(CoalesceWs& c, int64_t M, int64_t N, int drop_self, int64_t* out, int64_t* num_out, hipStream_t st) {
    unsigned hbad = 0;
    int hnum = 0;
    if (M > 0) {
        MGN_TRY(hipcub::DeviceRadixSort::SortKeys(c.tmp, c.tmp_bytes, c.keys, c.sorted, (int)M, 0, key_bits(N), st));
        const unsigned b = (unsigned)cdiv64(M, 256);
        hipLaunchKernelGGL(unique_flags, dim3(b), dim3(256), 0, st, c.sorted, M, N, drop_self, c.flags);
        MGN_LAUNCH_CHECK();
        MGN_TRY(hipcub::DeviceSelect::Flagged(c.tmp, c.tmp_bytes, c.sorted, c.flags, c.keys, c.num, (int)M, st));
        hipLaunchKernelGGL(split_keys, dim3(b), dim3(256), 0, st, c.keys, c.num, M, N, out);
        MGN_LAUNCH_CHECK();
        MGN_TRY(hipMemcpyAsync(&hnum, c.num, sizeof(int), hipMemcpyDeviceToHost, st));
    }
    MGN_TRY(hipMemcpyAsync(&hbad, c.bad, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    MGN_TRY(hipStreamSynchronize(st));
    MGN_REQUIRE(hbad == 0, "edge_index out of range");
    *num_out = hnum;
    return 0;
}

size_t khop_tmp_bytes(int64_t Ek) {
    size_t a = 0, b = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, a, (const int64_t*)nullptr, (int64_t*)nullptr, (int)Ek);
    hipcub::DeviceReduce::Sum(nullptr, b, (const int64_t*)nullptr, (int64_t*)nullptr, (int)Ek);
    return a > b ? a : b;
}

}  // namespace

extern "C" {

size_t mgn_coalesce_workspace_bytes(int64_t num_keys) { return coalesce_ws(num_keys < 1 ? 1 : num_keys); }

int64_t mgn_face_to_edge_keys(int32_t verts_per_cell, int64_t num_cells) {
    return (verts_per_cell == 4 ? 24 : 6) * num_cells;
}

int mgn_face_to_edge(const int64_t* cells, int32_t verts_per_cell, int64_t num_cells, int64_t num_nodes,
                     int64_t* edge_index, int64_t* num_edges, void* ws, size_t ws_bytes, mgn_stream_t stream) {
    MGN_REQUIRE(verts_per_cell == 3 || verts_per_cell == 4, "face_to_edge: cells must be [3, C] or [4, C]");
    MGN_REQUIRE(num_cells >= 0 && num_nodes >= 0 && num_nodes < (1ll << 31), "face_to_edge: bad sizes");
    const int64_t M = mgn_face_to_edge_keys(verts_per_cell, num_cells);
    MGN_REQUIRE(M < (1ll << 31), "face_to_edge: too many cells");
    MGN_REQUIRE(ws_bytes >= mgn_coalesce_workspace_bytes(M), "face_to_edge workspace too small");
    hipStream_t st = (hipStream_t)stream;
    CoalesceWs c = carve(ws, M < 1 ? 1 : M);
    MGN_TRY(hipMemsetAsync(c.bad, 0, sizeof(unsigned), st));
    if (num_cells > 0) {
        hipLaunchKernelGGL(cells_to_keys, dim3((unsigned)cdiv64(num_cells, 256)), dim3(256), 0, st, cells,
                           verts_per_cell, num_cells, num_nodes, c.keys, c.bad);
        MGN_LAUNCH_CHECK();
    }
    return coalesce_tail(c, M, num_nodes, 0, edge_index, num_edges, st);
}

int mgn_coalesce(const int64_t* edge_index, int64_t num_edges, int64_t num_nodes, int32_t flags, int64_t* out,
                 int64_t* num_out, void* ws, size_t ws_bytes, mgn_stream_t stream) {
    MGN_REQUIRE(num_edges >= 0 && num_nodes >= 0 && num_nodes < (1ll << 31), "coalesce: bad sizes");
    const int sym = (flags & MGN_COALESCE_SYMMETRIZE) != 0;
    const int64_t M = num_edges * (sym ? 2 : 1);
    MGN_REQUIRE(M < (1ll << 31), "coalesce: too many edges");
    MGN_REQUIRE(ws_bytes >= mgn_coalesce_workspace_bytes(M), "coalesce workspace too small");
    hipStream_t st = (hipStream_t)stream;
    CoalesceWs c = carve(ws, M < 1 ? 1 : M);
    MGN_TRY(hipMemsetAsync(c.bad, 0, sizeof(unsigned), st));
    if (num_edges > 0) {
        hipLaunchKernelGGL(edges_to_keys, dim3((unsigned)cdiv64(num_edges, 256)), dim3(256), 0, st, edge_index,
                           num_edges, num_nodes, sym, c.keys, c.bad);
        MGN_LAUNCH_CHECK();
    }
    return coalesce_tail(c, M, num_nodes, (flags & MGN_COALESCE_DROP_SELF_LOOPS) != 0, out, num_out, st);
}

size_t mgn_khop_count_workspace_bytes(int64_t num_edges_k, int64_t num_edges_a, int64_t num_nodes) {
    (void)num_edges_a;
    const int64_t ek = num_edges_k < 1 ? 1 : num_edges_k;
    return 2 * al(sizeof(int64_t)) + al((size_t)(num_nodes + 1) * 8) + 2 * al((size_t)ek * 8) + al(khop_tmp_bytes(ek));
}

// shared front of both k-hop calls: A's row pointers, per-edge candidate counts
static int khop_front(const int64_t* eik, int64_t Ek, const int64_t* eia, int64_t Ea, int64_t N, char*& w,
                      unsigned*& bad, int64_t*& total, int64_t*& aptr, int64_t*& cnt, int64_t*& off, void*& tmp,
                      size_t& tmp_bytes, hipStream_t st) {
    const int64_t ek = Ek < 1 ? 1 : Ek;
    bad = reinterpret_cast<unsigned*>(w); w += al(sizeof(int64_t));
    total = reinterpret_cast<int64_t*>(w); w += al(sizeof(int64_t));
    aptr = reinterpret_cast<int64_t*>(w); w += al((size_t)(N + 1) * 8);
    cnt = reinterpret_cast<int64_t*>(w); w += al((size_t)ek * 8);
    off = reinterpret_cast<int64_t*>(w); w += al((size_t)ek * 8);
    tmp = w;
    tmp_bytes = khop_tmp_bytes(ek);
    w += al(tmp_bytes);
    MGN_TRY(hipMemsetAsync(bad, 0, sizeof(unsigned), st));
    MGN_TRY(hipMemsetAsync(total, 0, sizeof(int64_t), st));
    if (Ea > 0) {
        hipLaunchKernelGGL(check_edge_range, dim3((unsigned)cdiv64(Ea, 256)), dim3(256), 0, st, eia, Ea, N, bad);
        MGN_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(row_ptr_i64, dim3((unsigned)cdiv64(N + 1, 256)), dim3(256), 0, st, eia, Ea, N, aptr);
    MGN_LAUNCH_CHECK();
    if (Ek > 0) {
        hipLaunchKernelGGL(khop_count, dim3((unsigned)cdiv64(Ek, 256)), dim3(256), 0, st, eik, Ek, aptr, N, cnt, bad);
        MGN_LAUNCH_CHECK();
    }
    return 0;
}

int mgn_khop_count(const int64_t* edge_index_k, int64_t num_edges_k, const int64_t* edge_index_a,
                   int64_t num_edges_a, int64_t num_nodes, int64_t* num_keys, void* ws, size_t ws_bytes,
                   mgn_stream_t stream) {
    MGN_REQUIRE(num_edges_k >= 0 && num_edges_a >= 0 && num_nodes >= 0 && num_nodes < (1ll << 31) &&
                    num_edges_k < (1ll << 31), "khop: bad sizes");
    MGN_REQUIRE(ws_bytes >= mgn_khop_count_workspace_bytes(num_edges_k, num_edges_a, num_nodes),
                "khop count workspace too small");
    hipStream_t st = (hipStream_t)stream;
    char* w = reinterpret_cast<char*>(ws);
    unsigned* bad;
    int64_t *total, *aptr, *cnt, *off;
    void* tmp;
    size_t tmp_bytes;
    int rc = khop_front(edge_index_k, num_edges_k, edge_index_a, num_edges_a, num_nodes, w, bad, total, aptr, cnt, off,
                        tmp, tmp_bytes, st);
    if (rc) return rc;
    if (num_edges_k > 0) MGN_TRY(hipcub::DeviceReduce::Sum(tmp, tmp_bytes, cnt, total, (int)num_edges_k, st));
    unsigned hbad = 0;
    int64_t htot = 0;
    MGN_TRY(hipMemcpyAsync(&hbad, bad, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    MGN_TRY(hipMemcpyAsync(&htot, total, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    MGN_TRY(hipStreamSynchronize(st));
    MGN_REQUIRE(hbad == 0, "edge_index out of range");
    *num_keys = htot;
    return 0;
}

size_t mgn_khop_workspace_bytes(int64_t num_keys, int64_t num_edges_k, int64_t num_nodes) {
    return mgn_khop_count_workspace_bytes(num_edges_k, 0, num_nodes) + mgn_coalesce_workspace_bytes(num_keys);
}

int mgn_khop_hop(const int64_t* edge_index_k, int64_t num_edges_k, const int64_t* edge_index_a, int64_t num_edges_a,
                 int64_t num_nodes, int64_t num_keys, int64_t* out, int64_t* num_out, void* ws, size_t ws_bytes,
                 mgn_stream_t stream) {
    MGN_REQUIRE(num_edges_k >= 0 && num_edges_a >= 0 && num_nodes >= 0 && num_nodes < (1ll << 31) &&
                    num_edges_k < (1ll << 31) && num_keys >= 0 && num_keys < (1ll << 31), "khop: bad sizes");
    MGN_REQUIRE(ws_bytes >= mgn_khop_workspace_bytes(num_keys, num_edges_k, num_nodes), "khop workspace too small");
    hipStream_t st = (hipStream_t)stream;
    char* w = reinterpret_cast<char*>(ws);
    unsigned* bad;
    int64_t *total, *aptr, *cnt, *off;
    void* tmp;
    size_t tmp_bytes;
    int rc = khop_front(edge_index_k, num_edges_k, edge_index_a, num_edges_a, num_nodes, w, bad, total, aptr, cnt, off,
                        tmp, tmp_bytes, st);
    if (rc) return rc;
    CoalesceWs c = carve(w, num_keys < 1 ? 1 : num_keys);
    MGN_TRY(hipMemsetAsync(c.bad, 0, sizeof(unsigned), st));
    if (num_edges_k > 0) {
        MGN_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, cnt, off, (int)num_edges_k, st));
        MGN_TRY(hipcub::DeviceReduce::Sum(tmp, tmp_bytes, cnt, total, (int)num_edges_k, st));
        int64_t htot = 0;
        MGN_TRY(hipMemcpyAsync(&htot, total, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        MGN_TRY(hipStreamSynchronize(st));
        MGN_REQUIRE(htot == num_keys, "khop: num_keys does not match mgn_khop_count for these inputs");
        hipLaunchKernelGGL(khop_expand, dim3((unsigned)cdiv64(num_edges_k, 256)), dim3(256), 0, st, edge_index_k,
                           num_edges_k, edge_index_a + num_edges_a, aptr, off, num_nodes, c.keys);
        MGN_LAUNCH_CHECK();
    }
    unsigned hbad = 0;
    MGN_TRY(hipMemcpyAsync(&hbad, bad, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    MGN_TRY(hipStreamSynchronize(st));
    MGN_REQUIRE(hbad == 0, "edge_index out of range");
    return coalesce_tail(c, num_keys, num_nodes, 1, out, num_out, st);
}

int mgn_edge_features(const float* pos, int64_t pos_ld, int32_t dim, const int64_t* edge_index, int64_t num_edges,
                      int64_t num_nodes, float* out, int64_t out_ld, void* ws, size_t ws_bytes, mgn_stream_t stream) {
    MGN_REQUIRE(dim >= 1 && dim <= 3 && pos_ld >= dim && out_ld >= dim + 1, "edge_features: bad shapes");
    MGN_REQUIRE(ws_bytes >= sizeof(unsigned), "edge_features workspace too small");
    if (num_edges == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    unsigned* bad = reinterpret_cast<unsigned*>(ws);
    MGN_TRY(hipMemsetAsync(bad, 0, sizeof(unsigned), st));
    const unsigned b = (unsigned)cdiv64(num_edges, 256);
    hipLaunchKernelGGL(check_edge_range, dim3(b), dim3(256), 0, st, edge_index, num_edges, num_nodes, bad);
    MGN_LAUNCH_CHECK();
    unsigned hbad = 0;
    MGN_TRY(hipMemcpyAsync(&hbad, bad, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    MGN_TRY(hipStreamSynchronize(st));
    MGN_REQUIRE(hbad == 0, "edge_index out of range");
    hipLaunchKernelGGL(edge_features_kernel, dim3(b), dim3(256), 0, st, pos, pos_ld, dim, edge_index, num_edges, out,
                       out_ld);
    MGN_LAUNCH_CHECK();
    return 0;
}

size_t mgn_radius_pairs_workspace_bytes(int64_t num_nodes) {
    const int64_t n = num_nodes < 1 ? 1 : num_nodes;
    size_t sort_tmp = 0, scan_tmp = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, (const int64_t*)nullptr, (int64_t*)nullptr,
                                       (const int32_t*)nullptr, (int32_t*)nullptr, (int)n);
    hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tmp, (const int64_t*)nullptr, (int64_t*)nullptr, (int)n);
    hipcub::DeviceReduce::Sum(nullptr, scan_tmp > sort_tmp ? sort_tmp : scan_tmp, (const int64_t*)nullptr,
                              (int64_t*)nullptr, (int)n);
    size_t red_tmp = 0;
    hipcub::DeviceReduce::Sum(nullptr, red_tmp, (const int64_t*)nullptr, (int64_t*)nullptr, (int)n);
    size_t t = sort_tmp > scan_tmp ? sort_tmp : scan_tmp;
    t = t > red_tmp ? t : red_tmp;
    return al(8 * sizeof(float)) + al(sizeof(int64_t)) + 2 * al((size_t)n * 8) + 2 * al((size_t)n * 4) +
           2 * al((size_t)n * 8) + al(t);
}

int mgn_radius_pairs(const float* pos, int64_t pos_ld, int32_t dim, int64_t num_nodes, double radius,
                     const float* node_type, int64_t node_type_ld, int64_t* out, int64_t capacity,
                     int64_t* num_pairs, void* ws, size_t ws_bytes, mgn_stream_t stream) {
    MGN_REQUIRE(dim >= 1 && dim <= 3 && pos_ld >= dim, "radius_pairs: bad shapes");
    MGN_REQUIRE(radius > 0.0 && std::isfinite(radius), "radius_pairs: radius must be positive");
    MGN_REQUIRE(num_nodes >= 0 && num_nodes < (1ll << 31), "radius_pairs: bad sizes");
    MGN_REQUIRE(ws_bytes >= mgn_radius_pairs_workspace_bytes(num_nodes), "radius_pairs workspace too small");
    *num_pairs = 0;
    if (num_nodes < 2) return 0;
    hipStream_t st = (hipStream_t)stream;
    const int64_t n = num_nodes;
    char* w = reinterpret_cast<char*>(ws);
    float* box = reinterpret_cast<float*>(w); w += al(8 * sizeof(float));
    int64_t* total = reinterpret_cast<int64_t*>(w); w += al(sizeof(int64_t));
    int64_t* key = reinterpret_cast<int64_t*>(w); w += al((size_t)n * 8);
    int64_t* skey = reinterpret_cast<int64_t*>(w); w += al((size_t)n * 8);
    int32_t* iota = reinterpret_cast<int32_t*>(w); w += al((size_t)n * 4);
    int32_t* sid = reinterpret_cast<int32_t*>(w); w += al((size_t)n * 4);
    int64_t* cnt = reinterpret_cast<int64_t*>(w); w += al((size_t)n * 8);
    int64_t* off = reinterpret_cast<int64_t*>(w); w += al((size_t)n * 8);
    void* tmp = w;
    size_t tmp_bytes = ws_bytes - (size_t)(w - reinterpret_cast<char*>(ws));

    hipLaunchKernelGGL(bbox_kernel, dim3(1), dim3(1024), 0, st, pos, pos_ld, dim, n, box);
    MGN_LAUNCH_CHECK();
    float hbox[6];
    MGN_TRY(hipMemcpyAsync(hbox, box, sizeof(hbox), hipMemcpyDeviceToHost, st));
    MGN_TRY(hipStreamSynchronize(st));
    Grid g;
    g.dim = dim;
    // cell edge slightly above r: points within r are never more than one cell apart after rounding
    double cell = radius * (1.0 + 1e-6);
    for (;;) {
        double cells = 1.0;
        for (int d = 0; d < 3; ++d) {
            if (d < dim) {
                MGN_REQUIRE(std::isfinite(hbox[d]) && std::isfinite(hbox[3 + d]), "radius_pairs: non-finite positions");
                g.o[d] = hbox[d];
                g.n[d] = (int64_t)std::floor(((double)hbox[3 + d] - (double)hbox[d]) / cell) + 1;
            } else {
                g.o[d] = 0.0;
                g.n[d] = 1;
            }
            cells *= (double)g.n[d];
        }
        if (cells < (double)(1ll << 40)) break;
        cell *= 2.0;  // sparse cloud in a huge box: coarser cells, same 27-cell query, still exact
    }
    g.inv = 1.0 / cell;
    const unsigned b = (unsigned)cdiv64(n, 256);
    hipLaunchKernelGGL(cell_keys, dim3(b), dim3(256), 0, st, pos, pos_ld, n, g, key, iota);
    MGN_LAUNCH_CHECK();
    MGN_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, key, skey, iota, sid, (int)n, 0, 64, st));
    const double r2 = radius * radius;
    const int filter = node_type != nullptr;
    hipLaunchKernelGGL(radius_pairs_kernel, dim3(b), dim3(256), 0, st, pos, pos_ld, n, g, r2, skey, sid, node_type,
                       node_type_ld, filter, 0, cnt, (const int64_t*)nullptr, (int64_t*)nullptr, (int64_t)0);
    MGN_LAUNCH_CHECK();
    MGN_TRY(hipcub::DeviceReduce::Sum(tmp, tmp_bytes, cnt, total, (int)n, st));
    int64_t htot = 0;
    MGN_TRY(hipMemcpyAsync(&htot, total, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    MGN_TRY(hipStreamSynchronize(st));
    *num_pairs = htot;
    if (htot == 0 || htot > capacity || out == nullptr) return 0;  // caller re-calls with capacity >= *num_pairs
    MGN_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, cnt, off, (int)n, st));
    hipLaunchKernelGGL(radius_pairs_kernel, dim3(b), dim3(256), 0, st, pos, pos_ld, n, g, r2, skey, sid, node_type,
                       node_type_ld, filter, 1, (int64_t*)nullptr, off, out, htot);
    MGN_LAUNCH_CHECK();
    return 0;
}

}  // extern "C"
