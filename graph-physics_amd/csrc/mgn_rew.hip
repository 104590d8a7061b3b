// Recomputed edge-MLP weight gradients (round 5) — see the comment below. Its own translation unit:
// the pipeline's waves run at two per SIMD (256 registers each), with none of mgn_chain16.hip's
// register-chained kernels' flags.
#include <cstring>

#include "mgn_chain16_dev.h"

namespace {

// ------------------------------------------------------------------------------------ recomputed weight gradients
// Round 5 (the save/re-read traffic): the edge MLP's hidden-layer weight gradients
// WITHOUT the forward's R8 layer-input saves. Measured before building it (tools/dev/r05_saves.py, the
// training vs the inference forward): the saves are 73 MB of the edge forward's 157 MB at Cfg B (33.9
// vs 25.4 µs) and 1.1 GB of its 2.54 GB at Cfg E (549 vs 257 µs), and the ring reads them back. Here one
// workgroup per row chunk re-runs layers 0..2 on its rows — the forward's own operations in its order
// (the stage16 image, gemm16's k-steps, P_i + P_j, ReLU, bf16): bit-identical X1..X3 — and accumulates
// dW_l = dZ_lᵀ·X_l and db_l = Σ dZ_l for l = 1..3 from the backward's R8 dZ saves. Twelve waves
// (three per SIMD, 168 registers each), every one with 32 MFMAs per step, in a pipeline through LDS:
//   waves 2i, 2i + 1 (i = 0..2): layer i on one 16-row tile each -> X_{i+1} (image i); layer 0 from e
//     rows and the P gathers, layers 1, 2 from image i - 1
//   waves 6 + 2(l-1) + hf (l = 1..3): image l - 1 -> output-feature half hf of dW_l, db_l (64x128 fp32)
// (A wave that both runs a layer and holds a weight-gradient accumulator has no registers left to keep
// its weight-fragment LDS reads in flight: measured 10k cycles per step against 1.5k.)
// Steps of 32 rows (one 16x16x32 k-step of the weight-gradient MFMAs); double-buffered hand-off images
// counted with ready / freed step counters in LDS. Weight-gradient operands: X_l from the row-major
// images by ds_read_b64_tr_b16 (the ring's XOR swizzle), dZ_l straight from the R8 saves (one 16-byte
// load per fragment). The e block of W0, the node MLP and W0's x blocks stay on the ring.
constexpr int REW_WAVES = 12;
constexpr int REW_FLAGS = 16;
constexpr int REW_SR = 32;                   // rows per step
constexpr int REW_IMG = REW_SR * H * 2;      // one 32-row bf16 image (8 KiB)
constexpr size_t REW_LDS_W = (size_t)3 * LFR * FRAG * 2;  // layers 0..2 (96 KiB)
static_assert((REW_LDS_W + 4 * H * 4) % 256 == 0 && REW_IMG % 256 == 0, "images on 256-byte boundaries (rew_get_tr's XOR)");
constexpr size_t REW_LDS = REW_LDS_W + 4 * H * 4 + (size_t)6 * REW_IMG + 4 * REW_FLAGS;
// Bounded hand-off waits: MGN_REW_SPIN polls (s_sleep 1 each, ~0.5 s at 2.4 GHz) before a wait gives
// up — a correct pipeline never comes near. The environment variable of the same name overrides it
// (diagnostics: MGN_REW_SPIN=0 makes every wait fail, tests/test_step_gpu.py). A wait that gives up
// ends its wave's loop (every wave still reaches the end of the kernel: the waits it would have served
// give up in turn), ORs MGN_ERR_HANDOFF into the call's error word and makes the workgroup's slab
// regions NaN instead of partial sums, so a timeout can never become a silently wrong gradient.
#ifndef MGN_REW_SPIN
#define MGN_REW_SPIN (1u << 24)
#endif

__device__ __forceinline__ int rew_slot(int r, int ch) { return r * (H * 2) + 16 * (ch ^ ((((r & 3) << 2) | ((r >> 2) & 3)))); }

// output tiles t0 .. t0 + NT - 1 of tile u (16 rows) of a C-layout activation into an image as bf16
// (the bits to_operand makes)
template <int NT>
__device__ __forceinline__ void rew_put(char* img, const f4 (&v)[NT], int u, int t0, int lane) {
    const int m = lane & 15, g = lane >> 4, r = u * 16 + m;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        const int t = t0 + i;
        const bf16x4 w = {(__bf16)v[i][0], (__bf16)v[i][1], (__bf16)v[i][2], (__bf16)v[i][3]};
        *reinterpret_cast<bf16x4*>(img + rew_slot(r, 2 * t + (g >> 1)) + 8 * (g & 1)) = w;
    }
}
// tile u's B operand in to_operand's layout (lane (m, g), k-step s: features 32s + 4g.., 32s + 16 + 4g..)
__device__ __forceinline__ void rew_get_op(const char* img, bf16x8 (&B)[4], int u, int lane) {
    const int m = lane & 15, g = lane >> 4, r = u * 16 + m;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const u32x2 lo = *reinterpret_cast<const u32x2*>(img + rew_slot(r, 4 * s + (g >> 1)) + 8 * (g & 1));
        const u32x2 hi = *reinterpret_cast<const u32x2*>(img + rew_slot(r, 4 * s + 2 + (g >> 1)) + 8 * (g & 1));
        B[s] = __builtin_bit_cast(bf16x8, u32x4{lo[0], lo[1], hi[0], hi[1]});
    }
}
// the 16x16x32 operand fragment of columns 16kt .. 16kt + 15 over the image's 32 rows (K): transposed
// LDS reads (mlp_wgrad_kernel's re-gathered-input path; K order = the R8 dZ fragment's rows). The
// lane's two byte offsets for k-tile 0 (rew_tr_base) become k-tile kt's by XOR with 32kt: the swizzle
// permutes 16-byte chunks by r-dependent XOR, so chunk 2kt + c sits at 32(kt ^ (swz >> 1)) + ...; one
// v_xor per read instead of 16 loop-invariant addresses held in registers.
typedef __attribute__((address_space(3))) char lds_char;
__device__ __forceinline__ uint32_t lds_u32(const char* p) {
    return (uint32_t)(uintptr_t)((const lds_char*)p);
}
__device__ __forceinline__ void rew_tr_base(int lane, uint32_t& blo, uint32_t& bhi) {
    const int i = lane & 15, q = i >> 2, p = i & 3;
    const int r0 = 8 * (lane >> 4) + q;
    blo = (uint32_t)(rew_slot(r0, p >> 1) + 8 * (p & 1));
    bhi = (uint32_t)(rew_slot(r0 + 4, p >> 1) + 8 * (p & 1));
}
__device__ __forceinline__ bf16x8 rew_get_tr(uint32_t lo_addr, uint32_t hi_addr, int kt) {
    typedef short s4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) s4 lds_s4;
    typedef short s8 __attribute__((ext_vector_type(8)));
    const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(uintptr_t)(lo_addr ^ (uint32_t)(kt << 5)));
    const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(uintptr_t)(hi_addr ^ (uint32_t)(kt << 5)));
    const s8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
}
// gemm16 (bias in the accumulator, per-tile k order: bit-identical) with two k-steps' 16 weight
// fragments in flight: half the exposed LDS latencies of gemm16 for waves with the registers
__device__ __forceinline__ void gemm16_k2(f4 (&acc)[8], const __bf16* W, int l, const bf16x8 (&B)[4], int lane,
                                          const float* bias) {
    acc_init(acc, bias, lane);
#pragma unroll
    for (int k = 0; k < 4; k += 2) {
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = mfma16(wfrag(W, l, t, k, lane), B[k], acc[t]);
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = mfma16(wfrag(W, l, t, k + 1, lane), B[k + 1], acc[t]);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Hand-off counters in LDS. Relaxed atomics with explicit LDS fences: a wave's LDS operations complete
// in order, so "image stores; s_waitcnt lgkmcnt(0); counter store" publishes the image, and the reader's
// counter load completes before its image loads issue. (A release / acquire at workgroup scope would
// also wait for the wave's outstanding global loads — the next step's prefetch — at every hand-off.)
__device__ __forceinline__ bool rew_wait(const unsigned* f, unsigned target, unsigned spin) {
    for (unsigned n = 0; n < spin; ++n) {
        if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            return true;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    return false;
}
// a wait gave up: report it on the call's device error word (a vector atomic from one lane)
__device__ __forceinline__ void rew_fail(const ChainRewArgs& a, int lane) {
    if (lane == 0 && a.err != nullptr) atomicOr(a.err, (unsigned)MGN_ERR_HANDOFF);
}
__device__ __forceinline__ void rew_signal(unsigned* f, unsigned v, int lane) {
    lds_fence();
    if (lane == 0) __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
}

// Diagnostics (-DMGN_STAMPS, tools/build_variant.sh ... mgn_rew.hip): per-phase s_memtime sums of every
// wave of workgroup 0, printed once per launch. Not in normal builds.
#ifdef MGN_STAMPS
#define RS_DECL unsigned long long rs_prev = __builtin_amdgcn_s_memtime(), rs_ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define RS(i)                                                                                           \
    do {                                                                                                \
        __builtin_amdgcn_sched_barrier(0);                                                              \
        unsigned long long rs_t;                                                                        \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(rs_t)::"memory");                   \
        __builtin_amdgcn_sched_barrier(0);                                                              \
        rs_ph[i] += rs_t - rs_prev;                                                                     \
        rs_prev = rs_t;                                                                                 \
    } while (0)
#define RS_PRINT(w, n)                                                                                  \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0)                                                     \
    printf("rew w%d steps %d %llu %llu %llu %llu %llu %llu %llu %llu\n", w, n, rs_ph[0], rs_ph[1], rs_ph[2],  \
           rs_ph[3], rs_ph[4], rs_ph[5], rs_ph[6], rs_ph[7])
#else
#define RS_DECL
#define RS(i)
#define RS_PRINT(w, n)
#endif

__global__ __launch_bounds__(REW_WAVES * 64, 1) void chain16_rew_kernel(ChainRewArgs a) {
    RS_DECL;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __bf16* W = reinterpret_cast<__bf16*>(smem);
    float* vec = reinterpret_cast<float*>(smem + REW_LDS_W);       // biases [4][H]
    char* hb = reinterpret_cast<char*>(vec + 4 * H);               // images H1, H2, H3 x 2 slots
    unsigned* flg = reinterpret_cast<unsigned*>(hb + 6 * REW_IMG);  // hand-off step counters
    const int lane = threadIdx.x & 63, m = lane & 15, g = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t r0 = (int64_t)blockIdx.x * a.rows_per_chunk;
    const int64_t r1 = r0 + a.rows_per_chunk < a.RP ? r0 + a.rows_per_chunk : a.RP;
    const int nsteps = r0 < r1 ? (int)((r1 - r0) / REW_SR) : 0;
    stage16<3, REW_WAVES * 64>(W, a.wpack, a.woff, a.wks, false);
    for (int i = threadIdx.x; i < 4 * H; i += REW_WAVES * 64) vec[i] = a.bias[i / H][i % H];
    if (threadIdx.x < REW_FLAGS) flg[threadIdx.x] = 0u;
    __syncthreads();
    RS(7);
    // image i (0: H1 = X1, 1: H2, 2: H3), slot s & 1; step counters:
    //   RD(i, u)  tile u of image i written (its producer)
    //   FD(i, hf) image i read by the weight-gradient wave of layer i + 1, half hf
    //   FC(i, u)  tile u of image i read by the producer of image i + 1 (i < 2)
    auto img = [&](int i, int s) { return hb + (size_t)(2 * i + (s & 1)) * REW_IMG; };
    unsigned* RD = flg;       // [3][2]
    unsigned* FD = flg + 6;   // [3][2]
    unsigned* FC = flg + 12;  // [2][2]
    auto prev = [](int s) { return (unsigned)(s > 0 ? s - 1 : 0); };  // a slot is rewritten 2 steps on
    if (wave < 6) {
        // ---- producers: image i, tile u (16 rows) of every 32-row step
        const int i = wave >> 1, u = wave & 1;
        auto slot_free = [&](int s) -> bool {
            if (!rew_wait(FD + 2 * i, prev(s), a.spin) || !rew_wait(FD + 2 * i + 1, prev(s), a.spin)) return false;
            return i == 2 || rew_wait(FC + 2 * i + u, prev(s), a.spin);
        };
        if (i == 0) {
            // layer 0 (chain16_fwd_kernel's operations: e·W0a, + P_i + P_j, ReLU). A step's operands
            // are loaded one step ahead and their gather indices two steps ahead
            const int64_t last = a.M - 1;
            auto rowof = [&](int s) {
                const int64_t r = r0 + (int64_t)s * REW_SR + 16 * u + m;
                return r < a.M ? r : last;
            };
            auto idx = [&](int s, int& di, int& dj) {
                const int64_t row = rowof(s < nsteps ? s : 0);
                di = a.proj_i[row];
                dj = a.proj_j[row];
            };
            auto load_e = [&](int s, bf16x8 (&eb)[4]) {
                const __bf16* e = a.e + rowof(s) * H + 4 * g;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const u32x2 lo = *reinterpret_cast<const u32x2*>(e + 32 * k);
                    const u32x2 hi = *reinterpret_cast<const u32x2*>(e + 32 * k + 16);
                    eb[k] = __builtin_bit_cast(bf16x8, u32x4{lo[0], lo[1], hi[0], hi[1]});
                }
            };
            // e rows one step ahead (before the MFMAs that consume the current ones), the P rows as
            // soon as the current ones are added (a put, the hand-off waits and the next step's MFMAs
            // cover them), gather indices two steps ahead
            bf16x8 eb[4], ebn[4];
            u32x2 pi[8], pj[8];
            int di = 0, dj = 0;
            if (nsteps > 0) {
                idx(0, di, dj);
                load_e(0, eb);
                load_p2(pi, a.proj + (int64_t)di * (2 * H), g);
                load_p2(pj, a.proj + (int64_t)dj * (2 * H) + H, g);
                idx(1, di, dj);
            }
            // ping-pong e buffers (two steps per iteration): the next step's rows land in the other
            // buffer's registers, no copy waiting for them
            auto step = [&](int s, const bf16x8 (&cur)[4], bf16x8 (&nxt)[4]) -> bool {
                load_e(s + 1 < nsteps ? s + 1 : s, nxt);
                RS(0);
                f4 x[8];
                gemm16(x, W, 0, cur, lane);  // (two e buffers + P leave no room for gemm16_k2)
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const f4 b = bf4(pi[t]) + bf4(pj[t]);
#pragma unroll
                    for (int r = 0; r < 4; ++r) x[t][r] = fmaxf(x[t][r] + b[r], 0.f);
                }
                if (s + 1 < nsteps) {
                    load_p2(pi, a.proj + (int64_t)di * (2 * H), g);
                    load_p2(pj, a.proj + (int64_t)dj * (2 * H) + H, g);
                    idx(s + 2, di, dj);
                }
                RS(1);
                if (!slot_free(s)) return false;
                rew_put<8>(img(0, s), x, u, 0, lane);
                rew_signal(RD + u, (unsigned)(s + 1), lane);
                RS(2);
                return true;
            };
            int s = 0;
            bool ok = true;
            for (; s + 1 < nsteps; s += 2)
                if (!step(s, eb, ebn) || !step(s + 1, ebn, eb)) {
                    ok = false;
                    break;
                }
            if (ok && s + 1 == nsteps) ok = step(s, eb, ebn);
            if (!ok) rew_fail(a, lane);
        } else {
            // layer i on X_i (tile u of image i - 1): + b_i, ReLU -> X_{i+1}
            for (int s = 0; s < nsteps; ++s) {
                if (!rew_wait(RD + 2 * (i - 1) + u, (unsigned)(s + 1), a.spin)) {
                    rew_fail(a, lane);
                    break;
                }
                RS(0);
                bf16x8 X[4];
                rew_get_op(img(i - 1, s), X, u, lane);
                rew_signal(FC + 2 * (i - 1) + u, (unsigned)(s + 1), lane);
                f4 x[8];
                gemm16_k2(x, W, i, X, lane, vec + i * H);
#pragma unroll
                for (int t = 0; t < 8; ++t)
#pragma unroll
                    for (int r = 0; r < 4; ++r) x[t][r] = fmaxf(x[t][r], 0.f);
                RS(1);
                if (!slot_free(s)) {
                    rew_fail(a, lane);
                    break;
                }
                rew_put<8>(img(i, s), x, u, 0, lane);
                rew_signal(RD + 2 * i + u, (unsigned)(s + 1), lane);
                RS(2);
            }
        }
        RS_PRINT(wave, nsteps);
        return;
    }
    // ---- weight-gradient waves: layer l = 1..3 (image l - 1), output-feature half hf:
    // dW_l[n][k] += Σ_rows dZ_l[row][n]·X_l[row][k], db_l[n] += Σ_rows dZ_l[row][n]
    const int l = 1 + (wave - 6) / 2, hf = (wave - 6) & 1;
    const __bf16* dz = a.dz8 + (int64_t)l * a.RP * H;
    f4 acc[4][8];  // acc[nt][kt]: the dWᵀ tile (k 16kt.., n 64hf + 16nt..)
    float bs[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        bs[nt] = 0.f;
#pragma unroll
        for (int kt = 0; kt < 8; ++kt) acc[nt][kt] = f4{0.f, 0.f, 0.f, 0.f};
    }
    // dZ_l fragments: R8 octets (r8_index): rows base + 8(lane >> 4) .. + 7 of column 64hf + 16nt + m sit
    // at dz + base·H + r8_index(8(lane >> 4), 64hf + m) + 128nt — one lane pointer, immediate offsets
    bf16x8 A[4];
    const __bf16* dzw = dz + r0 * H;  // wave-uniform
    const int dzo = (int)r8_index(8 * (lane >> 4), 64 * hf + m, H);
    auto loadA = [&](int s) {
        const __bf16* p = dzw + (int64_t)s * REW_SR * H + dzo;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) A[nt] = ld_frag(p + 128 * nt);
    };
    uint32_t tlo, thi;
    rew_tr_base(lane, tlo, thi);
    if (nsteps > 0) loadA(0);
    bool ok = true;
    for (int s = 0; s < nsteps; ++s) {
        if (!rew_wait(RD + 2 * (l - 1), (unsigned)(s + 1), a.spin) ||
            !rew_wait(RD + 2 * (l - 1) + 1, (unsigned)(s + 1), a.spin)) {
            ok = false;
            break;
        }
        RS(0);
        // db first: A is then dead after the MFMAs and the next step's loads land in its registers
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
            for (int v = 0; v < 8; ++v) bs[nt] += (float)A[nt][v];
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t hin = lds_u32(img(l - 1, s)), alo = hin + tlo, ahi = hin + thi;
        // two k-tiles' operands in flight at a time (the accumulator leaves ~40 registers)
#pragma unroll
        for (int kt = 0; kt < 8; kt += 2) {
            const bf16x8 b0 = rew_get_tr(alo, ahi, kt), b1 = rew_get_tr(alo, ahi, kt + 1);
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) acc[nt][kt] = mfma16(b0, A[nt], acc[nt][kt]);
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) acc[nt][kt + 1] = mfma16(b1, A[nt], acc[nt][kt + 1]);
            __builtin_amdgcn_sched_barrier(0);
        }
        rew_signal(FD + 2 * (l - 1) + hf, (unsigned)(s + 1), lane);
        RS(1);
        // unconditional (the last step reloads its own rows): the loads land in A's registers, no
        // copy that would wait for them at the end of the step
        loadA(s + 1 < nsteps ? s + 1 : s);
        RS(2);
    }
    // this wave's rows of layer l's slab regions: dW [128][128] and db. The MFMAs computed dWᵀ tiles
    // (X fragments as the row operand): lane (m, g) holds dW[64hf + 16nt + m][16kt + 4g .. + 3], one
    // 16-byte store. A timed-out wait (here or in a producer wave, whose failure makes this wave's waits
    // time out in turn) stores NaN, never the partial sums
    if (!ok) {
        rew_fail(a, lane);
        const float nan = __builtin_nanf("");
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            bs[nt] = nan;
#pragma unroll
            for (int kt = 0; kt < 8; ++kt) acc[nt][kt] = f4{nan, nan, nan, nan};
        }
    }
    float* slab = a.part + (int64_t)blockIdx.x * a.G;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int kt = 0; kt < 8; ++kt)
            *reinterpret_cast<f4*>(slab + a.w_off[l] + (int64_t)(64 * hf + 16 * nt + m) * H + 16 * kt + 4 * g) =
                acc[nt][kt];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        float t = bs[nt];
        t += __shfl_xor(t, 16);
        t += __shfl_xor(t, 32);
        if (g == 0) slab[a.b_off[l] + 64 * hf + 16 * nt + m] = t;
    }
    RS(6);
    RS_PRINT(wave, nsteps);
}

}  // namespace

int chain16_edge_wgrad_recompute(const mgn_mlp* m, const void* e, const void* proj, const int32_t* pi, const int32_t* pj,
                                 int64_t M, const void* dz8, float* part, int64_t G, int rows_per_chunk, int nchunks,
                                 hipStream_t st) {
    ChainRewArgs a;
    memset(&a, 0, sizeof(a));
    a.e = reinterpret_cast<const __bf16*>(e);
    a.proj = reinterpret_cast<const __bf16*>(proj);
    a.proj_i = pi;
    a.proj_j = pj;
    a.wpack = reinterpret_cast<const __bf16*>(m->wpack);
    layer_offsets(m, a.woff, a.wks);
    for (int l = 0; l < 4; ++l) a.bias[l] = m->bias[l];
    a.dz8 = reinterpret_cast<const __bf16*>(dz8);
    a.M = M;
    a.RP = rows_pad(M);
    a.rows_per_chunk = rows_per_chunk;
    a.nchunks = nchunks;
    a.part = part;
    a.G = G;
    a.err = g_call.err_word;
    a.spin = MGN_REW_SPIN;
    if (const char* v = getenv("MGN_REW_SPIN")) a.spin = (uint32_t)strtoul(v, nullptr, 0);
    int64_t o = 0;
    for (int l = 0; l < 4; ++l) {
        int n, k;
        mlp_layer_shape(*m, l, &n, &k);
        a.w_off[l] = o;
        a.b_off[l] = o + (int64_t)n * k;
        o += (int64_t)n * k + n;
    }
    MGN_REQUIRE(rows_per_chunk % REW_SR == 0 && nchunks > 0, "recomputed weight gradients: chunks of 32-row steps");
    MGN_REQUIRE(G % 4 == 0 && a.w_off[1] % 4 == 0 && ((uintptr_t)part & 15) == 0,
                "recomputed weight gradients: 16-byte aligned slab rows");
    if (M == 0) return 0;
    if (int e2 = set_lds_once((const void*)chain16_rew_kernel, REW_LDS)) return e2;
    ProfScope ps(PROF_WGRAD, st);
    hipLaunchKernelGGL(chain16_rew_kernel, dim3(nchunks), dim3(REW_WAVES * 64), REW_LDS, st, a);
    MGN_LAUNCH_CHECK();
    return 0;
}

