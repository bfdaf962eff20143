// tools/valu_issue.hip -- VALU issue cost and dependent latency of the turbo decoder's instructions on
// gfx950 (developer micro-benchmark; standalone: hipcc --offload-arch=gfx950 -O3 tools/valu_issue.hip).
//
// Each kernel runs N_IT iterations of 32 instructions of one kind, either as 8 independent chains
// (issue cost) or as one chain (dependent latency), and lane 0 of every wave reports clock64 cycles
// per instruction.  Launched as one workgroup of 64 threads (one wave alone on its SIMD) and of 512
// threads (8 waves on 4 SIMDs: two waves a SIMD).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int N_IT = 4096;

#define R8(OP)                                                                          \
  asm volatile(OP " %0, %0, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b)); \
  asm volatile(OP " %1, %1, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b)); \
  asm volatile(OP " %2, %2, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b)); \
  asm volatile(OP " %3, %3, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b)); \
  asm volatile(OP " %4, %4, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b)); \
  asm volatile(OP " %5, %5, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b)); \
  asm volatile(OP " %6, %6, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b)); \
  asm volatile(OP " %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));

#define R1(OP) asm volatile(OP " %0, %0, %1" : "+v"(a0) : "v"(b));

// independent: 8 chains, 32 instructions an iteration
#define INDEP_KERNEL(name, OP)                                                             \
  __global__ __launch_bounds__(512, 1) void name(unsigned long long* out, unsigned seed) \
  {                                                                                        \
    unsigned a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, \
             a7 = a0 * 19, b = seed ^ 0x00010001u;                                        \
    const unsigned long long t0 = clock64();                                              \
    for (int it = 0; it < N_IT; it++) {                                                   \
      R8(OP) R8(OP) R8(OP) R8(OP)                                                         \
    }                                                                                      \
    const unsigned long long t1 = clock64();                                              \
    if ((threadIdx.x & 63) == 0) out[threadIdx.x >> 6] = t1 - t0;                          \
    if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 0x12345u) out[63] = 1;                   \
  }

// dependent: one chain, 32 instructions an iteration
#define DEP_KERNEL(name, OP)                                                               \
  __global__ __launch_bounds__(512, 1) void name(unsigned long long* out, unsigned seed) \
  {                                                                                        \
    unsigned a0 = seed + threadIdx.x, b = seed ^ 0x00010001u;                              \
    const unsigned long long t0 = clock64();                                              \
    for (int it = 0; it < N_IT; it++) {                                                   \
      R1(OP) R1(OP) R1(OP) R1(OP) R1(OP) R1(OP) R1(OP) R1(OP)                             \
      R1(OP) R1(OP) R1(OP) R1(OP) R1(OP) R1(OP) R1(OP) R1(OP)                             \
      R1(OP) R1(OP) R1(OP) R1(OP) R1(OP) R1(OP) R1(OP) R1(OP)                             \
      R1(OP) R1(OP) R1(OP) R1(OP) R1(OP) R1(OP) R1(OP) R1(OP)                             \
    }                                                                                      \
    const unsigned long long t1 = clock64();                                              \
    if ((threadIdx.x & 63) == 0) out[threadIdx.x >> 6] = t1 - t0;                          \
    if (a0 == 0x12345u) out[63] = 1;                                                       \
  }

INDEP_KERNEL(i_add_u32, "v_add_u32")
INDEP_KERNEL(i_pk_add_i16, "v_pk_add_i16")
INDEP_KERNEL(i_pk_max_i16, "v_pk_max_i16")
INDEP_KERNEL(i_pk_sub_i16, "v_pk_sub_i16")
DEP_KERNEL(d_add_u32, "v_add_u32")
DEP_KERNEL(d_pk_add_i16, "v_pk_add_i16")
DEP_KERNEL(d_pk_max_i16, "v_pk_max_i16")

// the decoder's forms: clamp + op_sel, and v_perm_b32 (three operands)
#define R8C                                                                                \
  asm volatile("v_pk_add_i16 %0, %0, %8 op_sel:[1,0] op_sel_hi:[0,1] clamp\n\t"           \
               "v_pk_add_i16 %1, %1, %8 op_sel:[1,0] op_sel_hi:[0,1] clamp\n\t"           \
               "v_pk_add_i16 %2, %2, %8 op_sel:[1,0] op_sel_hi:[0,1] clamp\n\t"           \
               "v_pk_add_i16 %3, %3, %8 op_sel:[1,0] op_sel_hi:[0,1] clamp\n\t"           \
               "v_pk_add_i16 %4, %4, %8 op_sel:[1,0] op_sel_hi:[0,1] clamp\n\t"           \
               "v_pk_add_i16 %5, %5, %8 op_sel:[1,0] op_sel_hi:[0,1] clamp\n\t"           \
               "v_pk_add_i16 %6, %6, %8 op_sel:[1,0] op_sel_hi:[0,1] clamp\n\t"           \
               "v_pk_add_i16 %7, %7, %8 op_sel:[1,0] op_sel_hi:[0,1] clamp"               \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
#define R8P                                                                                \
  asm volatile("v_perm_b32 %0, %0, %8, %9\n\t"                                             \
               "v_perm_b32 %1, %1, %8, %9\n\t"                                             \
               "v_perm_b32 %2, %2, %8, %9\n\t"                                             \
               "v_perm_b32 %3, %3, %8, %9\n\t"                                             \
               "v_perm_b32 %4, %4, %8, %9\n\t"                                             \
               "v_perm_b32 %5, %5, %8, %9\n\t"                                             \
               "v_perm_b32 %6, %6, %8, %9\n\t"                                             \
               "v_perm_b32 %7, %7, %8, %9"                                                 \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "s"(sel));

__global__ __launch_bounds__(512, 1) void i_pk_add_clamp_opsel(unsigned long long* out, unsigned seed)
{
  unsigned a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17,
           a7 = a0 * 19, b = seed ^ 0x00010001u;
  const unsigned long long t0 = clock64();
  for (int it = 0; it < N_IT; it++) {
    R8C R8C R8C R8C
  }
  const unsigned long long t1 = clock64();
  if ((threadIdx.x & 63) == 0) out[threadIdx.x >> 6] = t1 - t0;
  if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 0x12345u) out[63] = 1;
}

__global__ __launch_bounds__(512, 1) void i_perm_b32(unsigned long long* out, unsigned seed)
{
  unsigned a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17,
           a7 = a0 * 19, b = seed ^ 0x00010001u;
  const unsigned sel = 0x05040100u ^ (seed & 0x01000000u);
  const unsigned long long t0 = clock64();
  for (int it = 0; it < N_IT; it++) {
    R8P R8P R8P R8P
  }
  const unsigned long long t1 = clock64();
  if ((threadIdx.x & 63) == 0) out[threadIdx.x >> 6] = t1 - t0;
  if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 0x12345u) out[63] = 1;
}

typedef void (*Kern)(unsigned long long*, unsigned);

int main()
{
  struct K {
    const char* name;
    Kern        k;
  } ks[] = {{"indep v_add_u32", i_add_u32},
            {"indep v_pk_add_i16", i_pk_add_i16},
            {"indep v_pk_add_i16 op_sel clamp", i_pk_add_clamp_opsel},
            {"indep v_pk_max_i16", i_pk_max_i16},
            {"indep v_pk_sub_i16", i_pk_sub_i16},
            {"indep v_perm_b32", i_perm_b32},
            {"dep v_add_u32", d_add_u32},
            {"dep v_pk_add_i16", d_pk_add_i16},
            {"dep v_pk_max_i16", d_pk_max_i16}};
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, 64 * sizeof(unsigned long long)) != hipSuccess) {
    return 1;
  }
  for (const K& k : ks) {
    for (int threads : {64, 512}) {
      hipMemset(d, 0, 64 * sizeof(unsigned long long));
      hipLaunchKernelGGL(k.k, dim3(1), dim3(threads), 0, 0, d, 7u);  // warm
      hipLaunchKernelGGL(k.k, dim3(1), dim3(threads), 0, 0, d, 7u);
      if (hipDeviceSynchronize() != hipSuccess) {
        return 2;
      }
      std::vector<unsigned long long> h(64);
      hipMemcpy(h.data(), d, 64 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
      const int    nw  = threads / 64;
      double       sum = 0;
      for (int w = 0; w < nw; w++) {
        sum += (double)h[w];
      }
      printf("{\"kernel\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_instruction\": %.2f}\n", k.name,
             threads == 64 ? 1 : 2, sum / nw / (N_IT * 32.0));
    }
  }
  hipFree(d);
  return 0;
}
