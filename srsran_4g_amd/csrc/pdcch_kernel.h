// srsran_4g_amd/csrc/pdcch_kernel.h -- launch interface of the PCFICH / PDCCH kernels.
#ifndef SRSRAN_AMD_PDCCH_KERNEL_H
#define SRSRAN_AMD_PDCCH_KERNEL_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srsran_amd {

static constexpr uint32_t PDCCH_MAX_BITS = 128;  // SRSRAN_DCI_MAX_BITS

struct PdcchCand {
  uint32_t L;         // aggregation level (log2)
  uint32_t ncce;      // first CCE
  uint32_t nof_bits;  // DCI payload bits (srsran_dci_format_sizeof)
};

struct PdcchCandOut {
  uint8_t  payload[PDCCH_MAX_BITS];
  uint32_t nof_bits;  // 0: skipped by the |LLR| mean gate
  uint16_t crc_rem;   // CRC remainder = the RNTI of a message for it
  float    corr;      // srsran_pdcch_msg_corr
};

// 2-port TX-diversity predecoding of n control REs gathered through idx (grid indices); the
// equalised symbols in codeword order to d (srsran_predecoding_diversity_multi + layer demap)
struct CtrlEqArgs {
  const float2*   y[2];     // [rx] grids (device)
  const float2*   h[2][2];  // [port][rx] estimates on the same indices
  const uint32_t* idx;      // n grid indices
  float2*         d;        // n equalised symbols
  uint32_t        n;
  uint32_t        sse_symbols;  // leading symbols computed as the reference's SSE body (4 * (n / 4) if n > 32)
  int             nrx;
};
hipError_t ctrl_diversity_launch(const CtrlEqArgs& a, hipStream_t stream);

// x: 16 equalised PCFICH symbols; seq: the subframe's 32 sequence bits (one word); d_data_f: 32
// descrambled LLRs; d_cfi / d_corr: decision and its correlation
hipError_t pcfich_launch(const float2* d_x, const uint32_t* d_seq, float* d_data_f, uint32_t* d_cfi, float* d_corr,
                         hipStream_t stream);
// nbits LLRs of nbits / 2 equalised symbols descrambled by the packed sequence bits
hipError_t pdcch_llr_launch(const float2* d_x, uint32_t nbits, const uint32_t* d_seq, float* d_llr, hipStream_t stream);
hipError_t pdcch_cand_launch(const float* d_llr, const PdcchCand* d_cands, uint32_t n, PdcchCandOut* d_outs,
                             hipStream_t stream);

}  // namespace srsran_amd
#endif
