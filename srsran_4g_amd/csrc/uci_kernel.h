// srsran_4g_amd/csrc/uci_kernel.h -- launch interface of the UCI-on-PUSCH receive kernels
// (HARQ-ACK / RI / CQI multiplexed on the UL-SCH, 36.212 5.2.2.6-5.2.2.8; uci.c, sch.c:1023-1193).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srsran_amd {

static constexpr uint32_t UCI_MAX_CQI_BITS = 64;  // SRSRAN_CQI_MAX_BITS

struct UciOut {
  uint8_t  ack[16];  // decoded HARQ-ACK bits (srsran_uci_value_ack_t::ack_value)
  uint8_t  ri[4];    // decoded RI bits (the reference keeps bit 0 in srsran_uci_value_t::ri)
  uint8_t  cqi[UCI_MAX_CQI_BITS];  // cqi_buff of srsran_ulsch_decode (zeros when the CRC8 fails)
  int32_t  ack_corr;
  int32_t  ack_thr;
  uint32_t ack_valid;
  uint32_t cqi_crc;  // data_crc
};

// One TB's UCI.  The positions of the ACK / RI soft bits follow uci_ulsch_interleave_{ack,ri}_gen
// (uci.c:364-412) from (rows = H' / N_symb, cols = N_symb, Qm).
struct UciDesc {
  int16_t*       q;      // device, PUSCH-order LLRs (ACK positions are zeroed in place, sch.c:1084)
  const uint8_t* c;      // device, unpacked scrambling sequence (1-bit ACK / RI repetitions only)
  const int16_t* g;      // device, de-interleaved LLRs (CQI at the front)
  UciOut*        out;    // device
  uint32_t       Qm, rows, cols;
  uint32_t       ack_bits, ack_Qp;  // O_ACK, Q'_ACK (0: none)
  uint32_t       ri_bits, ri_Qp;    // O_RI, Q'_RI
  uint32_t       cqi_bits, cqi_Qp;  // O_CQI, Q'_CQI (0: none)
};

// HARQ-ACK decode, zeroing of its positions, then RI decode (sch.c:1023-1120): one wave per TB.
hipError_t uci_ack_ri_launch(const UciDesc* d_desc, uint32_t ntb, hipStream_t stream);
// CQI decode from the de-interleaved LLRs (uci.c:202-300): block code ML (<= 11 bits) or
// rate de-matching + tail-biting Viterbi + CRC8.  One wave per TB.
hipError_t uci_cqi_launch(const UciDesc* d_desc, uint32_t ntb, hipStream_t stream);

}  // namespace srsran_amd
