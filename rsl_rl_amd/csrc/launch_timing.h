// Live launch timing (rslrl_launch_timing_*, bench.py's roofline): while armed, each launch of a timed hot-path kernel
// is bound to a (start, stop) event pair through hipExtLaunchKernelGGL, so the elapsed time is the dispatch's own
// begin / end -- the duration rocprofv3 reports -- rather than a marker-event span around the C-ABI call (which adds
// the dispatch latency of the markers, ~3-5 us per call).  Never bound while the stream is being captured.  Each bound
// launch carries a tag (the kernel it timed), read back per tag.  One state for the library (ppo_loss.hip defines it).
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <mutex>
#include <vector>

namespace rslrl {

enum LaunchTag : int32_t { kTagPpoLoss = 0, kTagRolloutRecord = 1, kTagGatherRecords = 2, kNumLaunchTags = 3 };

struct LaunchTiming {
    struct Slot {
        hipEvent_t start, stop;
        int32_t tag;
    };
    std::mutex mu;
    std::vector<Slot> pool;
    size_t used = 0, cap = 0;
    std::atomic<bool> on{false};
};

LaunchTiming& launch_timing();

template <typename K, typename... Args>
void launch_timed(int32_t tag, K kernel, dim3 g, dim3 b, size_t shmem, hipStream_t st, Args... args) {
    LaunchTiming& t = launch_timing();
    if (t.on.load(std::memory_order_relaxed)) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone) {
            hipEvent_t e0 = nullptr, e1 = nullptr;
            {
                std::lock_guard<std::mutex> lk(t.mu);
                if (t.used < t.cap) {
                    e0 = t.pool[t.used].start;
                    e1 = t.pool[t.used].stop;
                    t.pool[t.used].tag = tag;
                    ++t.used;
                }
            }
            if (e0) {
                hipExtLaunchKernelGGL(kernel, g, b, static_cast<uint32_t>(shmem), st, e0, e1, 0, args...);
                return;
            }
        }
    }
    hipLaunchKernelGGL(kernel, g, b, shmem, st, args...);
}

}  // namespace rslrl
