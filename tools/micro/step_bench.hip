// Microbenchmark: cycles per packed trellis step (beta_step / alpha step+LLR) for
// C independent chains per wave, one wave per SIMD (and 2 waves/SIMD variant).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef short v2s __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2s u2v(uint32_t u) { return __builtin_bit_cast(v2s, u); }
__device__ __forceinline__ uint32_t v2u(v2s v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ v2s padd(v2s a, v2s b) { return __builtin_elementwise_add_sat(a, b); }
__device__ __forceinline__ v2s pmax(v2s a, v2s b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ v2s lo2(v2s a) { return __builtin_shufflevector(a, a, 0, 0); }
__device__ __forceinline__ v2s hi2(v2s a) { return __builtin_shufflevector(a, a, 1, 1); }
__device__ __forceinline__ v2s swp(v2s a) { return __builtin_shufflevector(a, a, 1, 0); }
__device__ __forceinline__ v2s perm(v2s h, v2s l, uint32_t sel) { return u2v(__builtin_amdgcn_perm(v2u(h), v2u(l), sel)); }
#define QP(a, b, c, d) ((a) | ((b) << 2) | ((c) << 4) | ((d) << 6))
template <int C> __device__ __forceinline__ v2s dpp(v2s a) { return u2v((uint32_t)__builtin_amdgcn_mov_dpp((int)v2u(a), C, 0xf, 0xf, false)); }

__device__ __forceinline__ v2s beta_step(v2s P, v2s xy, uint32_t s1, uint32_t rb) {
  const v2s xys = padd(xy, swp(xy));
  const v2s g1 = perm(xys, xy, s1);
  const v2s t1 = dpp<QP(0,0,1,1)>(P), t2 = dpp<QP(2,2,3,3)>(P);
  const v2s r = perm(t2, t1, rb);
  return pmax(padd(lo2(r), g1), padd(hi2(r), swp(g1)));
}
template <int C, int N>
__global__ __launch_bounds__(64) void k(const uint32_t* xin, uint32_t* out, unsigned long long* cyc) {
  const int lane = threadIdx.x;
  const uint32_t s1 = (lane & 3) == 0 ? 0x05040c0cu : 0x03020100u, rb = (lane & 1) ? 0x07060302u : 0x05040100u;
  v2s P[C];
  for (int c = 0; c < C; c++) P[c] = u2v(xin[lane + c]);
  v2s xy[16];
  for (int i = 0; i < 16; i++) xy[i] = u2v(xin[lane * 7 + i]);
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < N; it++) {
#pragma unroll
    for (int i = 0; i < 16; i++)
#pragma unroll
      for (int c = 0; c < C; c++) P[c] = beta_step(P[c], xy[(i + c) & 15], s1, rb);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t acc = 0;
  for (int c = 0; c < C; c++) acc ^= v2u(P[c]);
  out[blockIdx.x * 64 + lane] = acc;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int C, int N>
void run(int blocks, const char* tag) {
  uint32_t *x, *o; unsigned long long* cy;
  hipMalloc(&x, 4096 * 4); hipMalloc(&o, blocks * 64 * 4); hipMalloc(&cy, blocks * 8);
  hipMemset(x, 1, 4096 * 4);
  hipLaunchKernelGGL((k<C, N>), dim3(blocks), dim3(64), 0, 0, x, o, cy);
  hipLaunchKernelGGL((k<C, N>), dim3(blocks), dim3(64), 0, 0, x, o, cy);
  hipDeviceSynchronize();
  unsigned long long h[4096]; hipMemcpy(h, cy, blocks * 8, hipMemcpyDeviceToHost);
  double m = 0; for (int b = 0; b < blocks; b++) m += h[b]; m /= blocks;
  // s_memtime counts at the shader clock
  printf("%-28s chains=%d blocks=%5d  cycles/step-per-chain=%.1f  cycles/step(all chains)=%.1f\n", tag, C, blocks,
         m / (N * 16.0), m / (N * 16.0 * C));
  hipFree(x); hipFree(o); hipFree(cy);
}
int main() {
  run<1, 64>(256, "1 wave/CU");
  run<2, 64>(256, "1 wave/CU");
  run<4, 64>(256, "1 wave/CU");
  run<8, 64>(256, "1 wave/CU");
  run<1, 64>(1024, "1 wave/SIMD");
  run<2, 64>(1024, "1 wave/SIMD");
  run<1, 64>(2048, "2 waves/SIMD");
  run<2, 64>(2048, "2 waves/SIMD");
  run<4, 64>(2048, "2 waves/SIMD");
  run<1, 64>(4096, "4 waves/SIMD");
  run<2, 64>(4096, "4 waves/SIMD");
  return 0;
}
