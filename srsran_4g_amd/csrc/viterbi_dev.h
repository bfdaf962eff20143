// srsran_4g_amd/csrc/viterbi_dev.h -- the rate-1/3, K = 7 tail-biting Viterbi decoder of the
// reference's AVX2 16-bit build (viterbi.c:546-605, viterbi37_avx2_16bit.c:176-313) as a device
// function for one 64-lane wave: lane = trellis state.  Shared by the PDCCH candidates
// (pdcch_kernel.hip) and the long CQI on PUSCH (uci_kernel.hip).
//
// sym: 3 F quantised soft bits (uint16, 32767 = erasure) in LDS.  The trellis runs over five copies
// of the frame (TB_ITER = 5) from metric 63 everywhere; every step's 64 decisions are one ballot
// word.  The reference's decision buffer is cleared per frame and its chainback reads word n + 6
// at step n, so the words past the last step are zeros: the chainback start state never matters.
// The frame is taken from the third copy.  dec: LDS, >= 5 F + 6 words; data: LDS, F bytes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srsran_amd {

__device__ __forceinline__ uint32_t vit_parity32(uint32_t v) { return __builtin_popcount(v) & 1u; }

// All 64 lanes of the workgroup must call it (it synchronises).
__device__ __forceinline__ void viterbi37_tb16(const uint16_t* sym, uint32_t F, uint64_t* dec, uint8_t* data,
                                               int lane)
{
  const int      s     = lane >> 1, b = lane & 1;
  const uint32_t bt0   = vit_parity32((2u * s) & 0x6Du) ? 65535u : 0u;
  const uint32_t bt1   = vit_parity32((2u * s) & 0x4Fu) ? 65535u : 0u;
  const uint32_t bt2   = vit_parity32((2u * s) & 0x57u) ? 65535u : 0u;
  uint32_t       m     = 63;
  const uint32_t steps = 5 * F;
  for (uint32_t t = 0; t < steps; t++) {
    const uint16_t* y  = &sym[3 * (t % F)];
    const uint32_t  a  = ((bt0 ^ y[0]) + (bt1 ^ y[1]) + 1) >> 1;
    const uint32_t  bm = (((bt2 ^ y[2]) + a + 1) >> 1) >> 3;
    const uint32_t  mb = 8191u - bm;
    const uint32_t  o0 = (uint32_t)__shfl((int)m, s, 64);
    const uint32_t  o1 = (uint32_t)__shfl((int)m, s + 32, 64);
    const uint32_t  x0 = (o0 + (b ? mb : bm)) & 0xffffu;
    const uint32_t  x1 = (o1 + (b ? bm : mb)) & 0xffffu;
    const bool      d  = (int16_t)(uint16_t)(x0 - x1) > 0;  // modulo compare of the 16-bit metrics
    m                  = d ? x1 : x0;
    const uint64_t bal = __ballot(d);
    if (lane == 0) {
      dec[t] = bal;
    }
  }
  __syncthreads();
  if (lane == 0) {
    for (int k = 0; k < 6; k++) {
      dec[steps + k] = 0;
    }
    uint32_t st = 0;
    for (int n = (int)steps - 1; n >= 0; n--) {
      const uint32_t k = (uint32_t)(dec[n + 6] >> st) & 1u;
      st               = (st >> 1) | (k << 5);
      if (n >= (int)(2 * F) && n < (int)(3 * F)) {
        data[n - 2 * F] = (uint8_t)k;
      }
    }
  }
  __syncthreads();
}

}  // namespace srsran_amd
