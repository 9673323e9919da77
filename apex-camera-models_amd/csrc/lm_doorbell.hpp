// lm_doorbell.hpp -- the doorbell of the LM's pre-queued evaluation (r06,
// ACM_TUNE_LM_HOST_RESULT 3).
//
// The host queues evaluation k + 1's normal-equations kernel (and its
// epilogue) while evaluation k runs.  When k's results are in and the LM
// wants another point, the host writes the camera into a mailbox in pinned
// host memory and then its sequence number; the kernel is already resident:
//   * the first wave of workgroup 0 polls the sequence word (bounded by a
//     wall-clock timeout), copies the camera to device memory with vector
//     stores and publishes a device-memory flag;
//   * thread 0 of every workgroup waits on that flag (bounded as well), so
//     only one wave reads host memory while the grid waits;
//   * every workgroup then reads the camera and runs the normal equations.
// Workgroup 0 never waits on another workgroup, so the wait ends whether or
// not the rest of the grid is resident.  A cancelled or timed-out evaluation
// computes nothing; the host learns which from the acknowledgement word.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "acm.h"

namespace acm {

struct LmMailbox {
    unsigned long long seq;  // host: written last (release)
    unsigned long long ack;  // device: seq when served, else seq | kLmNotServed
    acm_camera cam;          // host: the parameters to evaluate
};
constexpr unsigned long long kLmCancel = 1ull << 62;     // host: no evaluation after all
constexpr unsigned long long kLmNotServed = 1ull << 63;  // device: cancelled or timed out

struct LmDoorbell {
    const LmMailbox* mb;         // pinned host memory
    acm_camera* cam;             // device copy of the camera
    unsigned long long* flag;    // device: seq (served) or seq | kLmNotServed
    unsigned long long seq;
    unsigned long long timeout;  // wall-clock ticks
};

__device__ __forceinline__ unsigned long long lm_uniform64(unsigned long long v) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
}

// true: the camera is at d.cam and the evaluation runs; uniform over the
// workgroup
__device__ __forceinline__ bool lm_doorbell_wait(const LmDoorbell& d) {
    __shared__ int s_go;
    const unsigned t = threadIdx.x;
    if (blockIdx.x == 0 && t < 64) {
        const unsigned long long t0 = wall_clock64();
        bool served = false;
        for (;;) {
            const unsigned long long u = lm_uniform64(
                __hip_atomic_load(&d.mb->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
            if (u == d.seq) {
                served = true;
                break;
            }
            if (u == (d.seq | kLmCancel) || wall_clock64() - t0 > d.timeout) break;
            __builtin_amdgcn_s_sleep(4);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the host's camera before its seq
        constexpr unsigned kWords = (unsigned)(sizeof(acm_camera) / 4);
        if (served && t < kWords)
            reinterpret_cast<unsigned*>(d.cam)[t] =
                __hip_atomic_load(reinterpret_cast<const unsigned*>(&d.mb->cam) + t,
                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (t == 0) {
            const unsigned long long v = served ? d.seq : (d.seq | kLmNotServed);
            __hip_atomic_store(d.flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(const_cast<unsigned long long*>(&d.mb->ack), v, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    if (t == 0) {
        const unsigned long long t0 = wall_clock64();
        int go = 0;
        // relaxed polls, and no acquire afterwards: an acquire (per poll or
        // once per workgroup) invalidates the caches it must see through,
        // from every workgroup of the grid (r06j: +11 us per evaluation).
        // The camera is then read with coherent (agent-scope atomic) loads
        // issued only after the flag's value is known.
        for (;;) {
            const unsigned long long v =
                __hip_atomic_load(d.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((v & ~kLmNotServed) == d.seq) {
                go = (v & kLmNotServed) ? 0 : 1;
                break;
            }
            // workgroup 0 publishes within d.timeout; twice that is a
            // backstop, so that no wave can wait unboundedly
            if (wall_clock64() - t0 > 2 * d.timeout) break;
            __builtin_amdgcn_s_sleep(8);
        }
        s_go = go;
    }
    __syncthreads();
    return s_go != 0;
}

// The camera workgroup 0 copied, read after the flag (atomic loads cannot be
// hoisted above the wait) and made uniform (SGPRs, as a kernel argument is)
__device__ __forceinline__ acm_camera lm_doorbell_camera(const acm_camera* src) {
    constexpr int kWords = (int)(sizeof(acm_camera) / 4);
    unsigned w[kWords];
#pragma unroll
    for (int i = 0; i < kWords; ++i)
        w[i] = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(reinterpret_cast<const unsigned*>(src) + i, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT));
    acm_camera c;
    __builtin_memcpy(&c, w, sizeof(c));
    return c;
}

}  // namespace acm
