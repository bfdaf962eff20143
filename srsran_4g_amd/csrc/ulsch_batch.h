// srsran_4g_amd/csrc/ulsch_batch.h -- the batched UL-SCH receive behind srsran_pusch_gpu_decode_batch:
// srsran_ulsch_decode (sch.c:994-1193) for many UEs at once, UCI included, with every stage one launch
// over the batch (ACK/RI decode, de-interleaver, CQI decode, decode_tb).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/srsran_sch.h"

namespace srsran_amd {

struct UlschBatchUe {
  srsran_pusch_cfg_t* cfg;
  int16_t*            d_q;       // device: the UE's PUSCH-order LLRs (nof_bits; ACK positions zeroed in place)
  const uint8_t*      d_c;       // device: its unpacked scrambling sequence (1-bit ACK / RI), or null
  int16_t*            d_g;       // device scratch: nof_bits de-interleaved LLRs
  uint8_t*            d_data;    // device scratch inside [d_data_base, + data_bytes): tbs / 8 bytes
  bool                new_data;  // a new transmission: the soft buffer is reset first
  uint8_t*            data;      // host out: the TB (tbs / 8 bytes), or null
  srsran_uci_value_t* uci;       // host out (required when the UE carries UCI)
  int                 ret;       // out: srsran_ulsch_decode's return for this UE
  float               avg;       // out: avg_iterations of this UE's TB (the previous TB's without one)
};

// Enqueues the whole batch on `st` (the UL-SCH object's stream), waits for it (one host sync, two
// when a higher-layer subband CQI report's size depends on a decoded RI) and fills the outputs.
// Returns SRSRAN_SUCCESS when the batch ran (per-UE errors are in ret), an error otherwise.
int ulsch_decode_batch_dev(srsran_sch_t* q, uint32_t n, UlschBatchUe* ues, const uint8_t* d_data_base,
                           size_t data_bytes, hipStream_t st);

}  // namespace srsran_amd
