// tools/fetch_calib.hip -- FETCH_SIZE / WRITE_SIZE calibration for the access widths this repo's kernels
// use (developer tool; MI355X_MICROARCH.md "HBM": only 16-B-per-lane streaming reads are calibrated there).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE -- tools/fetch_calib      (then a second pass with WRITE_SIZE)
//
// Every launch streams a known byte count once, coalesced, over a buffer far larger than the 256 MiB
// Infinity Cache (1 GiB): reads of 2, 4, 8 and 16 bytes per lane (result folded into one word per
// workgroup), writes of the same widths, and one re-read launch (a 64 MiB slice read 8 times, the
// pattern of a decoder that re-reads its input every half-iteration).  The program prints the bytes
// of each launch in dispatch order; tools/fetch_calib.py divides the counters by them.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

namespace {

template <typename T>
__device__ __forceinline__ uint32_t fold(const T& v)
{
  const uint32_t* w = (const uint32_t*)&v;
  uint32_t        x = 0;
  for (unsigned i = 0; i < sizeof(T) / 4; i++) {
    x ^= w[i];
  }
  return x;
}

template <>
__device__ __forceinline__ uint32_t fold<uint16_t>(const uint16_t& v)
{
  return v;
}

template <typename T>
__global__ __launch_bounds__(256) void read_kernel(const T* __restrict__ in, size_t n, int passes, size_t n_slice,
                                                  uint32_t* __restrict__ out)
{
  uint32_t x = 0;
  for (int p = 0; p < passes; p++) {
    const size_t lim = passes > 1 ? n_slice : n;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < lim; i += (size_t)gridDim.x * blockDim.x) {
      x ^= fold(in[i]) + (uint32_t)p;
    }
  }
  __shared__ uint32_t red[256];
  red[threadIdx.x] = x;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      red[threadIdx.x] ^= red[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[blockIdx.x] = red[0];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void write_kernel(T* __restrict__ o, size_t n, uint32_t seed)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    T v;
    uint32_t* w = (uint32_t*)&v;
    if (sizeof(T) >= 4) {
      for (unsigned k = 0; k < sizeof(T) / 4; k++) {
        w[k] = seed ^ (uint32_t)i ^ k;
      }
    } else {
      *(uint16_t*)&v = (uint16_t)(seed ^ (uint32_t)i);
    }
    o[i] = v;
  }
}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr size_t kBytes = (size_t)1 << 30;
constexpr size_t kSlice = (size_t)64 << 20;
constexpr int    kGrid  = 4096;

template <typename T>
void run_read(const void* buf, uint32_t* out, int passes)
{
  const size_t n = kBytes / sizeof(T), ns = kSlice / sizeof(T);
  read_kernel<T><<<kGrid, 256>>>((const T*)buf, n, passes, ns, out);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  printf("{\"op\": \"read\", \"width\": %zu, \"passes\": %d, \"bytes\": %zu}\n", sizeof(T), passes,
         passes > 1 ? (size_t)passes * kSlice : kBytes);
}

template <typename T>
void run_write(void* buf)
{
  write_kernel<T><<<kGrid, 256>>>((T*)buf, kBytes / sizeof(T), 0x9e3779b9u);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  printf("{\"op\": \"write\", \"width\": %zu, \"passes\": 1, \"bytes\": %zu}\n", sizeof(T), kBytes);
}

}  // namespace

int main()
{
  void*     buf = nullptr;
  void*     flush = nullptr;
  uint32_t* out = nullptr;
  CK(hipMalloc(&buf, kBytes));
  CK(hipMalloc(&flush, kBytes / 2));
  CK(hipMalloc((void**)&out, kGrid * sizeof(uint32_t)));
  CK(hipMemset(buf, 0x5a, kBytes));
  // a 512 MiB store between launches evicts the Infinity Cache, so every read launch starts cold
  auto evict = [&]() {
    write_kernel<uint4><<<kGrid, 256>>>((uint4*)flush, kBytes / 2 / 16, 1u);
    CK(hipDeviceSynchronize());
    printf("{\"op\": \"evict\", \"width\": 16, \"passes\": 1, \"bytes\": %zu}\n", kBytes / 2);
  };
  evict();
  run_read<uint16_t>(buf, out, 1);
  evict();
  run_read<uint32_t>(buf, out, 1);
  evict();
  run_read<uint2>(buf, out, 1);
  evict();
  run_read<uint4>(buf, out, 1);
  evict();
  run_read<uint16_t>(buf, out, 8);
  evict();
  run_read<uint4>(buf, out, 8);
  run_write<uint16_t>(buf);
  run_write<uint32_t>(buf);
  run_write<uint2>(buf);
  run_write<uint4>(buf);
  CK(hipFree(buf));
  CK(hipFree(flush));
  CK(hipFree(out));
  return 0;
}
