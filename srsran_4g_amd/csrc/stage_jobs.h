// Descriptor staging copies fused into another launch (stage_copy.h): a batch's copy jobs ride in the UE DL
// chain's estimator launch (chest_kernel) instead of one stage_copy_kernel launch each.  A job copies
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
constexpr int kMaxFusedJobs = 2;  // the UE DL batch: PDSCH and DL-SCH descriptors
struct CopyJobs {
  CopyJob  job[kMaxFusedJobs];
  uint32_t n;
};

// Two halves, so that a launch can issue the PCIe reads early and consume them late (their latency under its
// own work): copy_jobs_issue loads element t0 = bid * blockDim.x + threadIdx.x of every job into registers
// (bid / nblocks: the workgroup's linear index / the launch's workgroups); copy_jobs_finish stores them, copies
// the rest of each job (grid-stride from t0 + nblocks * blockDim.x) and zeroes, then the workgroup counts
// itself done per job; the last one of a job publishes its fence.  Call both with all threads of the
// workgroup (finish has a barrier).
struct CopyRegs {  // element t0 of job 0 / job 1 (kMaxFusedJobs = 2), plain registers
  uint4 v0, v1;
};
static_assert(kMaxFusedJobs == 2, "CopyRegs holds one element of each of two jobs");
__device__ __forceinline__ void copy_jobs_issue(const CopyJobs& js, CopyRegs& r, uint32_t bid)
{
  const uint32_t t0 = bid * blockDim.x + threadIdx.x;
  if (js.n > 0 && t0 < js.job[0].n16) {
    r.v0 = js.job[0].src[t0];
  }
  if (js.n > 1 && t0 < js.job[1].n16) {
    r.v1 = js.job[1].src[t0];
  }
}
__device__ __forceinline__ void copy_job_rest(const CopyJob& c, uint4 v, uint32_t t0, uint32_t gs)
{
  if (t0 < c.n16) {
    c.dst[t0] = v;
  }
  for (uint32_t i = t0 + gs; i < c.n16; i += gs) {
    c.dst[i] = c.src[i];
  }
  for (uint32_t i = t0; i < c.nz; i += gs) {
    c.zero[i] = 0;
  }
}
__device__ __forceinline__ void copy_job_done(const CopyJob& c, uint32_t nblocks)
{
  if (c.fence && atomicAdd(c.count, 1u) == nblocks - 1) {
    __hip_atomic_store(c.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(c.fence, c.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
__device__ __forceinline__ void copy_jobs_finish(const CopyJobs& js, const CopyRegs& r, uint32_t bid, uint32_t nblocks)
{
  if (js.n == 0) {
    return;
  }
  const uint32_t nt = blockDim.x, gs = nblocks * nt, t0 = bid * nt + threadIdx.x;
  copy_job_rest(js.job[0], r.v0, t0, gs);
  if (js.n > 1) {
    copy_job_rest(js.job[1], r.v1, t0, gs);
  }
  // this workgroup's loads have returned (their values were stored) once every thread passed the barrier; the
  // count needs no fence (nothing is published through it: the consumers are later kernels) and the fence word
  // is a relaxed store to uncached host memory -- a release here would write back the L2 the launch is filling
  __syncthreads();
  if (threadIdx.x == 0) {
    copy_job_done(js.job[0], nblocks);
    if (js.n > 1) {
      copy_job_done(js.job[1], nblocks);
    }
  }
}

}  // namespace srsran_amd
#endif
