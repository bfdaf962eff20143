// Descriptor staging for the batch APIs: the host writes a batch's descriptors into pinned coherent host
// memory (a ring slot) and one small kernel in the launch stream copies them to the slot's device copy.
// Replaces hipMemcpyAsync on a side stream + cross-stream event waits, whose copy launch and waits left
// the GPU idle ~10-20 us at each hand-over (gpurun_out r04j rocprof trace of the PDSCH chain).
//
// No events in the steady state: every event recorded into the stream left the GPU idle ~5-6 us (r04l trace,
// device-scope release or not), so
//  - the copy kernel itself tells the host when it has read a ring slot: its last workgroup stores the batch's
//    sequence number into a pinned coherent fence word, on which the host waits before refilling the slot;
//  - device-side reuse (the slot's device copy, scratch shared between batches) is ordered by the stream; only
//    when a batch comes on another stream than the object's previous one does `handoff` make the new stream
//    wait for everything queued on the old one.
#ifndef SRSRAN_AMD_STAGE_COPY_H
#define SRSRAN_AMD_STAGE_COPY_H
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <functional>
#include <utility>
#include <vector>

#include "stage_jobs.h"

namespace srsran_amd {

// pinned host memory the GPU reads in place (mapped, coherent: no stale L2 lines when a ring slot comes round)
// -> host pointer; *dev = its device alias
void* stage_host_alloc(size_t bytes, void** dev);

// Per-object ring fence: fence words in pinned coherent memory (one per slot) and the copy kernel's
// workgroup counter (device, zero between launches)
struct StageFence {
  volatile uint32_t* h     = nullptr;
  uint32_t*          d     = nullptr;  // device alias of h
  uint32_t*          count = nullptr;
  uint32_t           seq   = 0;  // last sequence number handed out
  bool               broken = false;  // a wait timed out: the ring's state is unknown, the object fails from then on
};
bool stage_fence_init(StageFence& f, int nslots);
void stage_fence_free(StageFence& f);
// blocks until slot's fence word has reached seq (wrap-safe); returns false after ~10 s (a GPU that stopped, or a
// staging copy that was never launched) and marks the fence broken: every later wait on it fails at once, so the
// object keeps returning SRSRAN_ERROR instead of spinning 10 s a call on a slot whose sequence it cannot recover
bool stage_fence_wait(StageFence& f, int slot, uint32_t seq);

// dst (device) <- src_dev (device alias of stage_host_alloc memory), bytes rounded up to 16; the same launch
// zeroes zero_words 32-bit words at `zero` (optional: a per-batch accumulator, instead of a memset launch) and,
// with a fence, stores seq into fence word `slot` once every workgroup has read its part
hipError_t stage_copy_launch(void* dst, const void* src_dev, size_t bytes, hipStream_t stream, uint32_t* zero = nullptr,
                             uint32_t zero_words = 0, const StageFence* fence = nullptr, int slot = 0,
                             uint32_t seq = 0);

// Events that order work and free ring slots (never to publish GPU writes to host memory): device-scope release.
inline hipError_t ring_event_create(hipEvent_t* e)
{
  return hipEventCreateWithFlags(e, hipEventDisableTiming | hipEventReleaseToDevice);
}

// A stream on a hardware queue of its own: HIP maps ordinary streams onto GPU_MAX_HW_QUEUES shared queues
// (least-used first, so the mapping depends on every stream created and freed before); a stream created with a CU
// mask -- here every CU -- gets a new queue.  For PHY workers whose batches must overlap.  Blocking with respect to
// the legacy NULL stream (HIP creates CU-masked streams without hipStreamNonBlocking).
hipError_t own_queue_stream(hipStream_t* s);

// Stream hand-over of an object's device state: a batch on stream s after batches on another stream waits (on
// the GPU) for everything queued on that stream so far.  No-op while the stream stays the same.
struct StreamHandoff {
  hipStream_t last = nullptr;
  bool        any  = false;
  hipEvent_t  ev   = nullptr;
};
hipError_t handoff(StreamHandoff& h, hipStream_t s);
// everything queued by the object so far is done (host wait; grow / free paths)
void handoff_drain(StreamHandoff& h);
void handoff_free(StreamHandoff& h);

// Deferred launches (UE DL batch): while a recorder is installed on the calling thread, the batch APIs record
// their staging copies as CopyJobs (to be fused into the chain's first kernel) and their kernel launches as
// closures, to be replayed in order once the kernels in front of them are enqueued
struct LaunchRecorder {
  std::vector<CopyJob>                  jobs;
  std::vector<std::function<hipError_t()>> launches;
};
LaunchRecorder*& launch_recorder();  // the calling thread's recorder; nullptr = launch immediately
template <class F>
hipError_t launch_or_record(F&& f)
{
  if (LaunchRecorder* r = launch_recorder()) {
    r->launches.emplace_back(std::forward<F>(f));
    return hipSuccess;
  }
  return f();
}
// stage_copy_launch, or the same as a recorded job
hipError_t stage_copy_or_record(void* dst, const void* src_dev, size_t bytes, hipStream_t stream, uint32_t* zero,
                                uint32_t zero_words, const StageFence* fence, int slot, uint32_t seq);
// a recorded job as its own stage_copy_kernel launch
hipError_t stage_copy_job(const CopyJob& j, hipStream_t stream);

// SRSRAN_AMD_STAGE=side: the round-3 staging (hipMemcpyAsync on a side stream + event waits), for A/B runs
bool stage_side_copy();

}  // namespace srsran_amd
#endif
