// srsran_4g_amd/csrc/crc24_dev.h -- CRC-24 device helpers shared by the turbo and DL-SCH kernels.
//
// Semantics of srsran_crc_checksum_byte (crc.c:145-163, put_byte crc.h:57-76): MSB-first
// polynomial division, zero initial value, no final XOR.  A long message is split into
// contiguous chunks; each chunk's CRC (computed from zero) is moved to its place by
// multiplying with x^(8*bytes_after) mod P, and the parts XOR together (CRC linearity).
#ifndef SRSRAN_AMD_CRC24_DEV_H
#define SRSRAN_AMD_CRC24_DEV_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srsran_amd {

// one byte into a 24-bit CRC register (table-free)
__device__ __forceinline__ uint32_t crc24_byte(uint32_t crc, uint32_t byte, uint32_t poly)
{
  crc ^= byte << 16;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    crc = (crc & 0x800000u) ? ((crc << 1) ^ poly) : (crc << 1);
  }
  return crc & 0xFFFFFFu;
}

// a * b mod P over GF(2) for 24-bit a, b (P of degree 24, given with its x^24 bit).
// Horner over the bits of b, MSB first, reducing every step: 32-bit ops only.
__device__ __forceinline__ uint32_t clmul_mod24(uint32_t a, uint32_t b, uint32_t poly)
{
  uint32_t r = 0;
#pragma unroll 1
  for (int i = 23; i >= 0; i--) {
    r = (r << 1) ^ (((b >> i) & 1u) ? a : 0u);
    r ^= (r & 0x1000000u) ? poly : 0u;
  }
  return r;
}

// same, fully unrolled (for kernels with registers to spare)
__device__ __forceinline__ uint32_t clmul24(uint32_t a, uint32_t b, uint32_t poly)
{
  uint32_t r = 0;
#pragma unroll
  for (int i = 23; i >= 0; i--) {
    r = (r << 1) ^ (((b >> i) & 1u) ? a : 0u);
    r ^= (r & 0x1000000u) ? poly : 0u;
  }
  return r;
}

}  // namespace srsran_amd
#endif
