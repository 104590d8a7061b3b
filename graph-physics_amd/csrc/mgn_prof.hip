// Opt-in kernel profiler: HIP events recorded on the launch stream around each kernel class, so
// bench.py can report a kernel's average duration over the timed region without a tracer.
// (hipExtLaunchKernel's start/stop events were tried: hipEventElapsedTime rejects them on ROCm 7.2.)
#include <mutex>
#include <vector>

#include "mgn_common.h"

namespace {
struct Rec {
    hipEvent_t a, b;
    int kind;
};
std::mutex g_mu;
bool g_on = false;
std::vector<Rec> g_recs;
std::vector<hipEvent_t> g_pool;

hipEvent_t take() {
    if (!g_pool.empty()) {
        hipEvent_t e = g_pool.back();
        g_pool.pop_back();
        return e;
    }
    // timing-only events without the system-scope release: no L2 writeback / invalidate around the
    // profiled kernels (with it, every profiled kernel starts on flushed caches: the edge backward
    // read 47 us against 42 us in the rocprofv3 trace of the replayed step)
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
    return e;
}
}  // namespace

int mgn_prof_begin(int kind, hipStream_t st) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_on) return -1;
    Rec r{take(), take(), kind};
    if (!r.a || !r.b) return -1;
    hipEventRecord(r.a, st);
    g_recs.push_back(r);
    return (int)g_recs.size() - 1;
}

void mgn_prof_end(int slot, hipStream_t st) {
    if (slot < 0) return;
    std::lock_guard<std::mutex> lk(g_mu);
    if (slot < (int)g_recs.size()) hipEventRecord(g_recs[slot].b, st);
}

extern "C" {

/* Enable/disable the profiler; enabling also discards previous records. */
int mgn_profile_enable(int on) {
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto& r : g_recs) {
        g_pool.push_back(r.a);
        g_pool.push_back(r.b);
    }
    g_recs.clear();
    g_on = on != 0;
    return 0;
}

/* Total milliseconds and launch count of one kernel class since the last enable (synchronises
 * on the recorded events). */
int mgn_profile_collect(int kind, double* total_ms, int64_t* count) {
    std::lock_guard<std::mutex> lk(g_mu);
    double t = 0.0;
    int64_t c = 0;
    for (auto& r : g_recs) {
        if (r.kind != kind) continue;
        MGN_TRY(hipEventSynchronize(r.b));
        float ms = 0.f;
        MGN_TRY(hipEventElapsedTime(&ms, r.a, r.b));
        t += ms;
        ++c;
    }
    *total_ms = t;
    *count = c;
    return 0;
}

}  // extern "C"
