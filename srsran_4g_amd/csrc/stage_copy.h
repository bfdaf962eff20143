// Descriptor staging for the batch APIs: the host writes a batch's descriptors into pinned coherent host
// memory (a ring slot) and one small kernel in the launch stream copies them to the slot's device copy.
// Replaces hipMemcpyAsync on a side stream + cross-stream event waits, whose copy launch and waits left
// the GPU idle ~10-20 us at each hand-over (gpurun_out r04j rocprof trace of the PDSCH chain).
#ifndef SRSRAN_AMD_STAGE_COPY_H
#define SRSRAN_AMD_STAGE_COPY_H
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace srsran_amd {

// pinned host memory the GPU reads in place (mapped, coherent: no stale L2 lines when a ring slot comes round)
// -> host pointer; *dev = its device alias
void* stage_host_alloc(size_t bytes, void** dev);
// dst (device) <- src_dev (device alias of stage_host_alloc memory), bytes rounded up to 16; the same launch
// zeroes zero_words 32-bit words at `zero` (optional: a per-batch accumulator, instead of a memset launch)
hipError_t stage_copy_launch(void* dst, const void* src_dev, size_t bytes, hipStream_t stream, uint32_t* zero = nullptr,
                             uint32_t zero_words = 0);
// Events that order work and free ring slots (never to publish GPU writes to host memory): device-scope release.
// A default event's system-scope release writes back and invalidates the caches when it is recorded, which left
// the GPU idle ~5.5 us at every record in the PDSCH chain (gpurun_out r04k rocprof trace: 5 records a batch)
inline hipError_t ring_event_create(hipEvent_t* e)
{
  return hipEventCreateWithFlags(e, hipEventDisableTiming | hipEventReleaseToDevice);
}
// SRSRAN_AMD_STAGE=side: the round-3 staging (hipMemcpyAsync on a side stream + event waits), for A/B runs
bool stage_side_copy();

}  // namespace srsran_amd
#endif
