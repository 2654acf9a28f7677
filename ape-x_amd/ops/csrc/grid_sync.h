// Grid-wide barrier for kernels whose whole grid is co-resident (the launcher checks the
// occupancy: grid <= CUs x resident workgroups per CU), used to run several dependent
// phases of a learner step in ONE launch instead of one launch per phase.
//
// bar[0] counts arrivals, bar[1] is the generation.  Thread 0 of every workgroup releases
// the workgroup's writes (agent-scope fence: the XCD's L2 written back), arrives, and the
// last arrival resets the count and bumps the generation; the others poll the generation
// (agent-scope loads, s_sleep between polls), then acquire (L2 / L1 invalidated) before the
// workgroup barrier lets the other waves read what other workgroups wrote.
//
// Every wait is bounded: after `kGridSyncTimeoutTicks` of the 100 MHz wall clock, or as
// soon as another workgroup has timed out, the wait gives up and sets *err -- the kernel
// then always drains (wrong results, flagged) instead of hanging the device if the grid
// was not co-resident after all.
#pragma once

#include <hip/hip_runtime.h>

namespace apex {

constexpr unsigned long long kGridSyncTimeoutTicks = 100000000ull;  // 1 s at 100 MHz

__device__ __forceinline__ void grid_sync(unsigned* bar, unsigned nblocks, int* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned gen = __hip_atomic_load(bar + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned arrived = __hip_atomic_fetch_add(bar, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (arrived == nblocks - 1) {
      __hip_atomic_store(bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(bar + 1, gen + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const unsigned long long t0 = wall_clock64();
      while (__hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen) {
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) break;
        if (wall_clock64() - t0 > kGridSyncTimeoutTicks) {
          __hip_atomic_fetch_or(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __threadfence();
  }
  __syncthreads();
}

}  // namespace apex
