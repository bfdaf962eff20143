// tools/micro/ifetch.hip -- does instruction delivery bound a long straight-line VALU stream on gfx950?
// (developer micro-benchmark, standalone: hipcc --offload-arch=gfx950 -O3 tools/micro/ifetch.hip -o ifetch)
//
// A body of BODY independent instructions (8 chains), looped N_IT times, on EVERY CU at once with 1, 2 and
// 4 waves per SIMD (one workgroup per CU, forced by its LDS reservation).  Variants: 8-byte VOP3P
// v_pk_add_i16 clamp (the turbo decoder's instruction), 4-byte VOP2 v_add_u32, and the VOP3P form in a short
// body (32 instructions: served from the wave's instruction buffer).  Reports cycles per instruction per wave
// and VALU instructions per SIMD-cycle.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define STR2(x) #x
#define STR(x) STR2(x)

template <int KIND, int BODY>
__global__ __launch_bounds__(1024) void k(unsigned long long* out, unsigned seed, int n_it)
{
  extern __shared__ unsigned lds[];
  unsigned a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17,
           a7 = a0 * 19, b = seed ^ 0x00010001u;
  const unsigned long long t0 = clock64();
  for (int it = 0; it < n_it; it++) {
    if constexpr (KIND == 0) {
      asm volatile(".rept %[n]\n\t"
                   "v_pk_add_i16 %0, %0, %8 op_sel:[1,0] op_sel_hi:[0,1] clamp\n\t"
                   "v_pk_add_i16 %1, %1, %8 op_sel:[1,0] op_sel_hi:[0,1] clamp\n\t"
                   "v_pk_add_i16 %2, %2, %8 op_sel:[1,0] op_sel_hi:[0,1] clamp\n\t"
                   "v_pk_add_i16 %3, %3, %8 op_sel:[1,0] op_sel_hi:[0,1] clamp\n\t"
                   "v_pk_add_i16 %4, %4, %8 op_sel:[1,0] op_sel_hi:[0,1] clamp\n\t"
                   "v_pk_add_i16 %5, %5, %8 op_sel:[1,0] op_sel_hi:[0,1] clamp\n\t"
                   "v_pk_add_i16 %6, %6, %8 op_sel:[1,0] op_sel_hi:[0,1] clamp\n\t"
                   "v_pk_add_i16 %7, %7, %8 op_sel:[1,0] op_sel_hi:[0,1] clamp\n\t"
                   ".endr"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(b), [n] "i"(BODY / 8));
    } else {
      asm volatile(".rept %[n]\n\t"
                   "v_add_u32 %0, %0, %8\n\t"
                   "v_add_u32 %1, %1, %8\n\t"
                   "v_add_u32 %2, %2, %8\n\t"
                   "v_add_u32 %3, %3, %8\n\t"
                   "v_add_u32 %4, %4, %8\n\t"
                   "v_add_u32 %5, %5, %8\n\t"
                   "v_add_u32 %6, %6, %8\n\t"
                   "v_add_u32 %7, %7, %8\n\t"
                   ".endr"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(b), [n] "i"(BODY / 8));
    }
  }
  const unsigned long long t1 = clock64();
  const unsigned           w  = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0) {
    out[w] = t1 - t0;
  }
  if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 0x12345u) {
    lds[0] = 1;
    out[0] = lds[0];
  }
}

typedef void (*Kern)(unsigned long long*, unsigned, int);

int main()
{
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  struct K {
    const char* name;
    Kern        k;
    int         body;
  } ks[] = {{"vop3p pk_add_i16 clamp, body 2048 (16 KB)", k<0, 2048>, 2048},
            {"vop3p pk_add_i16 clamp, body 32", k<0, 32>, 32},
            {"vop2 add_u32, body 2048 (8 KB)", k<1, 2048>, 2048},
            {"vop2 add_u32, body 32", k<1, 32>, 32}};
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, 64 * 4096 * sizeof(unsigned long long)) != hipSuccess) {
    return 1;
  }
  const size_t lds = 100 * 1024;  // one workgroup a CU
  for (const K& kk : ks) {
    hipFuncSetAttribute((const void*)kk.k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    const int n_it = 65536 / kk.body * 8;
    for (int wps : {1, 2, 4}) {
      const int threads = 64 * 4 * wps;
      if (threads > 256 && wps > 1) {
        // 512 / 1024 threads a workgroup
      }
      hipLaunchKernelGGL(kk.k, dim3(ncu), dim3(threads), lds, 0, d, 7u, 16);  // warm
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(kk.k, dim3(ncu), dim3(threads), lds, 0, d, 7u, n_it);
      hipEventRecord(e1, 0);
      if (hipDeviceSynchronize() != hipSuccess) {
        printf("launch failed\n");
        return 2;
      }
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const int                       nw = ncu * threads / 64;
      std::vector<unsigned long long> h(nw);
      hipMemcpy(h.data(), d, nw * sizeof(unsigned long long), hipMemcpyDeviceToHost);
      double sum = 0;
      for (int w = 0; w < nw; w++) {
        sum += (double)h[w];
      }
      const double insts = (double)n_it * kk.body;
      const double cpi   = sum / nw / insts;
      printf("{\"kernel\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_inst_per_wave\": %.3f, \"insts_per_simd_cycle\": %.4f, \"ms\": %.4f}\n",
             kk.name, wps, cpi, wps / cpi, ms);
    }
  }
  return 0;
}
