// srsran_4g_amd/csrc/devkey.h -- the current HIP device, used to key every process-wide device table
// cache (QPP tables, rate de-matching tables, CRC shift tables, FFT twiddles, Gold jump tables,
// per-device streams).  One process may drive several GPUs, one host thread per GPU:
// a table built on device 0 must never be handed to a kernel launched on device 1.
#pragma once
#include <hip/hip_runtime.h>

namespace srsran_amd {

inline int cur_dev()
{
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) {
    return 0;
  }
  return d;
}

}  // namespace srsran_amd
