// Inter-workgroup hand-offs inside one launch on gfx950 (8 XCDs with
// private L2s, per-CU L1s never refreshed by other CUs' stores), following
// the agent-scope release/acquire rules of the CDNA4 guide: payload stored
// write-through (sc1, no release fence needed), every storing wave drains
// (s_waitcnt vmcnt(0)) before the flag or ticket, the consumer polls with
// relaxed agent-scope loads, takes ONE agent-scope acquire, then reads.
#pragma once

#include "internal.hpp"

namespace mpg {

// Last-arriver hand-off (one GPU): every workgroup stores its partials
// write-through (sc1, so no release fence is needed for them), drains its
// stores, and one lane draws a ticket; the workgroup that draws the last one
// takes an agent-scope acquire and combines all partials in a fixed order
// (deterministic, placement-independent). The counter is re-armed by the
// last arriver; it starts zeroed (hipMemset at plan creation).
typedef __attribute__((address_space(1))) unsigned int gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

__device__ __forceinline__ void store_wt(double* p, double v) {
    __hip_atomic_store((gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// true in every thread of the last-arriving of `expected` workgroups that
// share the counter (after its acquire); last_arriver: of the whole grid
__device__ __forceinline__ bool last_arriver_of(unsigned* cnt, unsigned expected) {
    __shared__ int last_s;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t = __hip_atomic_fetch_add((gu32*)cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = t == expected - 1;
        if (last) {
            __hip_atomic_store((gu32*)cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        last_s = last;
    }
    __syncthreads();
    return last_s != 0;
}
__device__ __forceinline__ bool last_arriver(unsigned* cnt) { return last_arriver_of(cnt, gridDim.x); }


__device__ __forceinline__ void store_wt(float* p, float v) {
    __hip_atomic_store((gu32*)p, (unsigned)__float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wait until *flag != 0 (lane-local; relaxed agent-scope polls with
// s_sleep). Bounded by the 100 MHz real-time counter: after `bound` ticks
// (default ~2 s) it records a fault in *err and returns false, so a
// scheduling fault ends the launch instead of hanging the GPU.
constexpr uint64_t kWaitBound = 200000000ull;
__device__ __forceinline__ bool wait_flag(const int* flag, int* err, uint64_t bound = kWaitBound) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load((const gu32*)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        __builtin_amdgcn_s_sleep(2);
        if (__builtin_amdgcn_s_memrealtime() - t0 > bound) {
            __hip_atomic_store((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
    }
    return true;
}

__device__ __forceinline__ void set_flag(int* flag) {
    __hip_atomic_store((gu32*)flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ void acquire_agent() {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// LDS written by some lanes of a wave and read by others of the same wave
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace mpg
