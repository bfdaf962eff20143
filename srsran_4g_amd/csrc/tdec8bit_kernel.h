// srsran_4g_amd/csrc/tdec8bit_kernel.h -- launch interface of the 8-bit LLR turbo decoder
// (tdec8bit_kernel.hip): the reference's SSE / AVX2 8-bit window decoders, 16 or 32 sub-blocks.
#ifndef SRSRAN_AMD_TDEC8BIT_KERNEL_H
#define SRSRAN_AMD_TDEC8BIT_KERNEL_H
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace srsran_amd {

struct Tdec8Args {
  const int8_t* in;         // ncb code blocks of int8 LLRs, in_stride bytes apart (device)
  uint32_t      in_stride;
  int           layout_sb;  // 0: natural 3K+12, 1: sub-block layout (3 (K + 32) + 12, rm_turbo)
  uint32_t      K;
  uint32_t      ncb;
  int           n_end;      // half-iterations to run (>= 1)
  uint8_t*      out;        // ncb * K/8 hard-decision bytes (device)
  uint2*        beta;       // scratch, tdec8bit_beta_bytes (device)
  const uint16_t* qpp;      // the interleaver in the SB layout: qpp[j] = SB index of the QPP image of SB index j
  // ---- DL-SCH mode (decode_tb_cb with llr_is_8bit, sch.c:391-456): enabled when cbs != nullptr.  Block i reads
  // (const int8_t*)cbs[i].in (SB layout), skips it when *cbs[i].skip, and stops at the first half-iteration
  // >= min_iters whose decision passes the block's CRC; decisions to out + slot * out_stride ----
  const struct TdecCb* cbs;
  uint32_t        out_stride;
  uint8_t*        noi_out;   // per slot: half-iterations run (0 = skipped)
  uint8_t*        crc_ok;    // per slot
  const uint32_t* xpow_a;    // x^(8m) mod CRC24A / CRC24B (crc24_dev.h combine)
  const uint32_t* xpow_b;
  int             min_iters;
};

size_t     tdec8bit_lds_bytes(int nsb, uint32_t K);
size_t     tdec8bit_beta_bytes(int nsb, uint32_t K, uint32_t ncb);
hipError_t tdec8bit_launch(int nsb, const Tdec8Args& a, hipStream_t stream);
// int8 -> int16 copy of ncb rows (in_stride bytes apart) of len LLRs into a dense int16 array
hipError_t tdec8bit_widen(const int8_t* in, uint32_t in_stride, short* out, uint32_t len, uint32_t ncb,
                          hipStream_t stream);

// 8-bit rate de-matching (srsran_rm_turbo_rx_lut_8bit): sb[p] += sum of e[k], k = inv[p] + j N < E, int8
// wrap-around; positions with inv[p] = 0xFFFF (layout padding) untouched
hipError_t rm8_rx_launch(const int8_t* e, int8_t* sb, const uint16_t* inv, uint32_t E, uint32_t len, uint32_t N,
                         hipStream_t stream);
// the DL-SCH batch's de-matching in the 8-bit form: every RmSlot with e / sb read as int8 (the soft buffer row as
// buffer_f[cb] cast to int8_t*, sch.c:409-414); skip / overwrite as rm_rx_launch
hipError_t rm8_rx_slots_launch(const struct RmSlot* d_slots, uint32_t nslots, uint32_t max_len, hipStream_t stream);
// int8 -> int16 widening of n soft buffer rows (src[i] -> dst[i], len values), for the 16-bit decoders of K <= 800
struct Widen8 {
  const int8_t* src;
  short*        dst;
  uint32_t      len;
};
hipError_t widen8_launch(const Widen8* d_items, uint32_t n, uint32_t max_len, hipStream_t stream);

}  // namespace srsran_amd
#endif
