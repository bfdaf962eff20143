// Descriptor staging copies fused into another launch (stage_copy.h): a batch's copy jobs ride in the first
// kernel of the UE DL chain (ofdm_rx_kernel) instead of one stage_copy_kernel launch each.  A job copies
// pinned host descriptors to their device slot, optionally zeroes a word range, and its last workgroup stores
// the batch's sequence number into the slot's fence word -- exactly what stage_copy_kernel does.
#ifndef SRSRAN_AMD_STAGE_JOBS_H
#define SRSRAN_AMD_STAGE_JOBS_H
#include <hip/hip_runtime.h>

#include <cstdint>

namespace srsran_amd {

struct CopyJob {
  uint4*       dst;
  const uint4* src;    // device alias of pinned host memory
  uint32_t     n16;
  uint32_t     nz;
  uint32_t*    zero;   // nz words zeroed (optional)
  uint32_t*    fence;  // fence word of the slot (optional)
  uint32_t*    count;  // the fence's workgroup counter (device, zero between launches)
  uint32_t     seq;
};
constexpr int kMaxFusedJobs = 4;
struct CopyJobs {
  CopyJob  job[kMaxFusedJobs];
  uint32_t n;
};

// every workgroup of the launch takes its share of each job (grid-stride), then counts itself done per job;
// the last one of a job publishes its fence.  Call with all threads of the workgroup (it has a barrier).
__device__ __forceinline__ void run_copy_jobs(const CopyJobs& js)
{
  if (js.n == 0) {
    return;
  }
  const uint32_t nt = blockDim.x, gs = gridDim.x * nt, t0 = blockIdx.x * nt + threadIdx.x;
  for (uint32_t j = 0; j < js.n; j++) {
    const CopyJob& c = js.job[j];
    for (uint32_t i = t0; i < c.n16; i += gs) {
      c.dst[i] = c.src[i];
    }
    for (uint32_t i = t0; i < c.nz; i += gs) {
      c.zero[i] = 0;
    }
  }
  // this workgroup's loads have returned (their values were stored) once every thread passed the barrier; the
  // count needs no fence (nothing is published through it: the consumers are later kernels) and the fence word
  // is a relaxed store to uncached host memory -- a release here would write back the L2 the launch is filling
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t j = 0; j < js.n; j++) {
      const CopyJob& c = js.job[j];
      if (c.fence && atomicAdd(c.count, 1u) == gridDim.x - 1) {
        __hip_atomic_store(c.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(c.fence, c.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

}  // namespace srsran_amd
#endif
