// Global-address-space views of device pointers that reach a kernel through a descriptor in memory
// (batch items, staged arrays).  Without them the compiler addresses such pointers with FLAT instructions,
// which count on both the vector-memory and the LDS counters: every LDS wait then also waits for the
// thread's outstanding stores, and the loads of a batched group serialise behind them.
#ifndef SRSRAN_AMD_GMEM_H
#define SRSRAN_AMD_GMEM_H
#include <hip/hip_runtime.h>

namespace srsran_amd {

#if defined(__HIP_DEVICE_COMPILE__)
template <typename T>
using gptr_t = __attribute__((address_space(1))) T*;
#else  // the host pass of a .hip file only parses device code: the qualifier has no meaning there
template <typename T>
using gptr_t = T*;
#endif

template <typename T>
__device__ __forceinline__ gptr_t<T> gptr(T* p)
{
  return (gptr_t<T>)p;
}

}  // namespace srsran_amd
#endif
