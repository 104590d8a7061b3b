// Device helpers shared by the register-chained bf16 h=128 kernels (mgn_chain16.hip) and the recomputed
// edge weight gradients (mgn_rew.hip, compiled without -amdgpu-mfma-vgpr-form: its weight-gradient
// accumulators live in the AGPR file). Everything is in an anonymous namespace: one copy per TU.
#pragma once
#include <mutex>

#include "mgn_chain.h"

#ifndef MGN_ABLATE
#define MGN_ABLATE 0
#endif

namespace {

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int H = 128;
constexpr int TR = 16;                 // edges per wave tile
constexpr int NW = 8;                  // waves per workgroup (2 per SIMD)
constexpr int FRAG = 512;              // bf16 per 16x16x32 operand fragment (64 lanes x 8)
constexpr int LFR = 32;                // fragments per layer: 8 out-tiles x 4 k-steps

__device__ __forceinline__ f4 mfma16(const bf16x8& a, const bf16x8& b, const f4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ f4 bf4(u32x2 v) {
    const bf16x4 b = __builtin_bit_cast(bf16x4, v);
    return f4{(float)b[0], (float)b[1], (float)b[2], (float)b[3]};
}

// Weight image: fragment (l, t, s) lane (r, g) element j = A_l[16t + r][32s + 16(j>>2) + 4g + (j&3)]
// (A = W forward, Wᵀ backward). Linear walk over libmgn's 16x16x32 packs (16-byte coalesced loads):
// a source chunk holds 8 consecutive reduction indices 32s + 8q .. +7 of one row; its halves go to
// lane groups g = 2(q&1) + half, element group jg = q>>1.
template <int NL = 4, int NT = NW * 64>
__device__ __forceinline__ void stage16(__bf16* W, const __bf16* pack, const int64_t* woff, const int* wks,
                                        bool transposed, int tid = -1) {
    constexpr int TOT = NL * 2048, PER = (TOT + NT - 1) / NT;  // 16 chunks per thread (4 layers, 512 threads)
    if (tid < 0) tid = threadIdx.x;
    u32x4 v[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int it = tid + u * NT;
        if (TOT % NT != 0 && it >= TOT) break;
        const int l = it >> 11, c = it & 2047;
        const int tile = c >> 6, lane16 = c & 63;
        const int rt = tile >> 2, ks = tile & 3;
        const int ksl = transposed ? 4 : wks[l];
        if (MGN_ABLATE & 4) {
            v[u] = u32x4{0u, 0u, 0u, 0u};
            continue;
        }
        v[u] = *reinterpret_cast<const u32x4*>(pack + woff[l] + ((int64_t)(rt * ksl + ks) * 64 + lane16) * 8);
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int it = tid + u * NT;
        if (TOT % NT != 0 && it >= TOT) break;
        const int l = it >> 11, c = it & 2047;
        const int tile = c >> 6, lane16 = c & 63;
        const int rt = tile >> 2, ks = tile & 3;
        const int r = lane16 & 15, q = lane16 >> 4;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const int g = (2 * q + half) & 3, jg = q >> 1;
            const u32x2 w = {v[u][2 * half], v[u][2 * half + 1]};
            *reinterpret_cast<u32x2*>(W + ((size_t)((l * 8 + rt) * 4 + ks) * 64 + r + 16 * g) * 8 + jg * 4) = w;
        }
    }
}

__device__ __forceinline__ bf16x8 wfrag(const __bf16* W, int l, int t, int s, int lane) {
    return *reinterpret_cast<const bf16x8*>(W + ((size_t)((l * 8 + t) * 4 + s) * 64 + lane) * 8);
}

// acc = bias (LDS vector, features 16t + 4g..; nullptr: 0) + W_l · B: the bias rides in the MFMA
// accumulator instead of one v_add per output element after it
__device__ __forceinline__ void acc_init(f4 (&acc)[8], const float* bias, int lane) {
#pragma unroll
    for (int t = 0; t < 8; ++t)
        acc[t] = bias ? *reinterpret_cast<const f4*>(bias + 16 * t + 4 * (lane >> 4)) : f4{0.f, 0.f, 0.f, 0.f};
}

__device__ __forceinline__ void gemm16(f4 (&acc)[8], const __bf16* W, int l, const bf16x8 (&B)[4], int lane,
                                       const float* bias = nullptr) {
    acc_init(acc, bias, lane);
    // one k-step's 8 fragments in flight at a time (the other wave on the SIMD covers the LDS
    // latency); without the fence the scheduler hoists all 32 reads and the backward spills
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = mfma16(wfrag(W, l, t, s, lane), B[s], acc[t]);
        __builtin_amdgcn_sched_barrier(0);
    }
}

__device__ __forceinline__ void to_operand(const f4 (&v)[8], bf16x8 (&B)[4]) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) B[s][j] = (__bf16)v[2 * s + (j >> 2)][j & 3];
}

// Pair layout (P2) of a bf16 row of 128 features, for rows this library both writes and gathers
// back in the accumulator layout (node projections P, the edge MLP's z, the node MLP's z, d_aggr):
// feature 16t + 4g + r sits at 32(t>>1) + 8g + 4(t&1) + r, so the two quads of lane group g for the
// tile pair (2i, 2i+1) are one 16-byte load (4 loads of 16 B per row and lane instead of 8 of 8 B).
template <bool P2>
__device__ __forceinline__ int col_of(int t, int g) {
    return P2 ? 32 * (t >> 1) + 8 * g + 4 * (t & 1) : 16 * t + 4 * g;
}
// the 8 accumulator-layout quads (features 16t + 4g .. +3) of a P2 row
__device__ __forceinline__ void load_p2(u32x2 (&o)[8], const __bf16* row, int g) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const u32x4 w = *reinterpret_cast<const u32x4*>(row + 32 * i + 8 * g);
        o[2 * i] = u32x2{w[0], w[1]};
        o[2 * i + 1] = u32x2{w[2], w[3]};
    }
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

int set_lds_once(const void* fn, size_t bytes) {
    static std::mutex mu;
    static const void* done[32] = {};
    std::lock_guard<std::mutex> lk(mu);
    for (const void* d : done)
        if (d == fn) return 0;
    MGN_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    for (const void*& d : done)
        if (!d) {
            d = fn;
            break;
        }
    return 0;
}

}  // namespace
