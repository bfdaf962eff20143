// srsran_4g_amd/csrc/stage_copy.cpp -- host side of the descriptor staging (stage_copy.h)
#include "stage_copy.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace srsran_amd {

void* stage_host_alloc(size_t bytes, void** dev)
{
  void* h = nullptr;
  *dev    = nullptr;
  if (hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    return nullptr;
  }
  if (hipHostGetDevicePointer(dev, h, 0) != hipSuccess) {
    hipHostFree(h);
    *dev = nullptr;
    return nullptr;
  }
  return h;
}

bool stage_fence_init(StageFence& f, int nslots)
{
  void* d = nullptr;
  void* h = stage_host_alloc((size_t)nslots * sizeof(uint32_t), &d);
  if (!h) {
    return false;
  }
  f.h = (volatile uint32_t*)h;
  f.d = (uint32_t*)d;
  for (int i = 0; i < nslots; i++) {
    f.h[i] = 0;
  }
  f.seq = 0;
  if (hipMalloc((void**)&f.count, sizeof(uint32_t)) != hipSuccess || hipMemset(f.count, 0, sizeof(uint32_t)) != hipSuccess) {
    return false;
  }
  return true;
}

void stage_fence_free(StageFence& f)
{
  if (f.h) {
    hipHostFree((void*)f.h);
  }
  if (f.count) {
    hipFree(f.count);
  }
  f = StageFence();
}

bool stage_fence_wait(StageFence& f, int slot, uint32_t seq)
{
  if (f.broken) {
    return false;
  }
  uint32_t spins = 0;
  auto     t0    = std::chrono::steady_clock::now();
  while ((int32_t)(f.h[slot] - seq) < 0) {
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
    if ((++spins & 0xfff) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
      fprintf(stderr, "[srsran_amd] staging ring slot %d: fence %u never reached %u; the object is unusable\n", slot,
              f.h[slot], seq);
      f.broken = true;
      return false;
    }
  }
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  return true;
}

hipError_t handoff(StreamHandoff& h, hipStream_t s)
{
  if (h.any && h.last != s) {
    if (!h.ev) {
      const hipError_t e = ring_event_create(&h.ev);
      if (e != hipSuccess) {
        return e;
      }
    }
    hipError_t e = hipEventRecord(h.ev, h.last);
    if (e == hipSuccess) {
      e = hipStreamWaitEvent(s, h.ev, 0);
    }
    if (e != hipSuccess) {
      return e;
    }
  }
  h.last = s;
  h.any  = true;
  return hipSuccess;
}

void handoff_drain(StreamHandoff& h)
{
  if (h.any) {
    hipStreamSynchronize(h.last);
  }
}

void handoff_free(StreamHandoff& h)
{
  if (h.ev) {
    hipEventDestroy(h.ev);
  }
  h = StreamHandoff();
}

LaunchRecorder*& launch_recorder()
{
  static thread_local LaunchRecorder* r = nullptr;
  return r;
}

hipError_t stage_copy_or_record(void* dst, const void* src_dev, size_t bytes, hipStream_t stream, uint32_t* zero,
                                uint32_t zero_words, const StageFence* fence, int slot, uint32_t seq)
{
  if (LaunchRecorder* r = launch_recorder()) {
    CopyJob j;
    j.dst   = (uint4*)dst;
    j.src   = (const uint4*)src_dev;
    j.n16   = (uint32_t)((bytes + 15) / 16);
    j.nz    = zero ? zero_words : 0;
    j.zero  = zero;
    j.fence = fence ? fence->d + slot : nullptr;
    j.count = fence ? fence->count : nullptr;
    j.seq   = seq;
    r->jobs.push_back(j);
    return hipSuccess;
  }
  return stage_copy_launch(dst, src_dev, bytes, stream, zero, zero_words, fence, slot, seq);
}

hipError_t own_queue_stream(hipStream_t* s)
{
  int             dev = 0;
  hipDeviceProp_t prop;
  hipError_t      e = hipGetDevice(&dev);
  if (e != hipSuccess || (e = hipGetDeviceProperties(&prop, dev)) != hipSuccess) {
    return e;
  }
  std::vector<uint32_t> mask((prop.multiProcessorCount + 31) / 32, ~0u);
  return hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data());
}

bool stage_side_copy()
{
  static const bool side = [] {
    const char* e = getenv("SRSRAN_AMD_STAGE");
    return e && strcmp(e, "side") == 0;
  }();
  return side;
}

}  // namespace srsran_amd
