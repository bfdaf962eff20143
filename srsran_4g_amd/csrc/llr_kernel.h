// srsran_4g_amd/csrc/llr_kernel.h -- PDSCH LLR stages: soft demapping + descrambling.
#ifndef SRSRAN_AMD_LLR_KERNEL_H
#define SRSRAN_AMD_LLR_KERNEL_H
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "eq_kernel.h"

namespace srsran_amd {

// Upload the Gold-sequence jump tables (once per process; idempotent).
hipError_t gold_tables_init();

// Soft demap nsym symbols (interleaved re/im float) of modulation `mod` (0 BPSK .. 4 256QAM) into
// int16 LLRs; when `scramble`, LLR i is negated where the Gold sequence c(bit0 + i) of `seed` is 1;
// when d_csi is set, the PDSCH CSI correction follows with the max CSI read from *d_csi_max.
hipError_t llr_launch(int mod, const float* d_sym, uint32_t nsym, int scramble, uint32_t seed, uint32_t bit0,
                      const float* d_csi, const float* d_csi_max, int16_t* d_llr, hipStream_t stream);

// One demap + descramble + CSI job of a batch (PDSCH codeword of one subframe).
struct LlrItem {
  const float*  sym;      // interleaved re/im symbols
  const float*  csi;      // optional CSI per symbol
  const float*  csi_max;  // max CSI (device), required with csi
  int16_t*      llr;
  uint32_t      n;        // symbols
  uint32_t      seed;
  uint32_t      bit0;
  int           scramble;
  // srsran_evm_run_s (modem/evm.h:175-212) on the first evm_n symbols (0: off): per LLR block the sum of
  // |sym - mod(hard(pre-scrambling LLRs))|^2 into evm_part[block]; evm_finalize_launch turns them into the RMS
  float*        evm_part;
  uint32_t      evm_n;
  // q->llr_is_8bit (pdsch.c:691-737): int8 LLRs here instead of llr (demod_b, sequence_apply_c, the 8-bit CSI
  // correction, srsran_evm_run_b); the launch's llr8 flag selects the form
  int8_t*       llr8;
};
// one EVM result: sqrtf(sum of nparts block sums (in block order) / nsym) into *out
struct EvmItem {
  const float* part;
  uint32_t     nparts;
  uint32_t     nsym;
  float*       out;
};
hipError_t evm_finalize_launch(const EvmItem* d_items, uint32_t nitems, hipStream_t stream);
#ifndef LLR_SPT_CFG
#define LLR_SPT_CFG 8  // symbols per thread of the LLR kernel (build parameter; 8: 1248 workgroups for C3, r04p)
#endif
constexpr uint32_t LLR_BLOCK_SYMBOLS = 256 * LLR_SPT_CFG;  // symbols of one LLR block (evm_part entries = ceil(n / this))
// nitems items of one modulation (device array); max_n = largest n
hipError_t llr_batch_launch(int mod, const LlrItem* d_items, uint32_t nitems, uint32_t max_n, int any_scramble,
                            hipStream_t stream, bool llr8 = false);

// The fused predecode + LLR path (PORT0, or SM / CDD with two codewords of one modulation on two layers; int16
// LLRs, no EVM): every RE of the subframe whose predecoder descriptor is *pa is equalised in the kernel (eq_dev.h)
// and each layer's symbol demapped, descrambled and CSI-corrected as llr_batch_launch does, with no equalised-symbol
// / CSI buffers in between; the CSI maxima come from csi_max_batch_launch.
struct FusedItem {
  const PredArgs* pa;
  int16_t*        llr[2];   // [layer] = codeword on that layer
  uint32_t        seed[2];  // [layer] scrambling seed (bit 0 of the sequence at symbol 0)
  const float*    csi_max;  // [layer] max CSI (device); nullptr: CSI correction off
  uint32_t        n;        // REs (= symbols a layer)
};
// nitems items of one modulation and one predecoder scheme (0: one layer; 2, 3: two); max_n = largest n
hipError_t fused_llr_batch_launch(int mod, int scheme, const FusedItem* d_items, uint32_t nitems, uint32_t max_n,
                                  hipStream_t stream);

// out[i] = c(i) ? -in[i] : in[i] (int16 wrap) for the Gold sequence of `seed`.
hipError_t seq_apply_launch(const int16_t* d_in, int16_t* d_out, uint32_t len, uint32_t seed, hipStream_t stream);
// out[i] = c(i) (one byte per bit) for the Gold sequence of `seed`.
hipError_t seq_unpack_launch(uint8_t* d_out, uint32_t len, uint32_t seed, hipStream_t stream);

// ---- transmitter: PDSCH scrambling + modulation + precoding + RE mapping of one subframe ----
struct PdschTx {
  const uint8_t*  e[2];     // packed e bits per codeword (device)
  uint32_t        seed[2];  // scrambling seeds (pdsch_seed)
  int             mod[2];   // srsran_mod_t
  const uint32_t* idx;      // RE table (srsran_pdsch_re_table order; bit 31 ignored)
  float2*         grid[4];  // per-port subframe grids (2 nsymb x 12 nof_prb)
  uint32_t        nre;      // PDSCH REs
  int             scheme;   // 0: one port; 1: transmit diversity (2 ports, 1 codeword); 3: CDD 2x2 (2 codewords);
                            // 4: transmit diversity on 4 ports (SFBC + FSTD, 1 codeword)
  float           scaling;  // rho_a scaling of the precoder (1)
  float           div_scale;// (float)(scaling * M_SQRT1_2) for 2-port, (float)(scaling / M_SQRT2) for 4-port diversity
};
hipError_t pdsch_tx_launch(const PdschTx* d_items, uint32_t nitems, uint32_t max_nre, hipStream_t stream);
// CRS of ports 0..nports-1 (1, 2 or 4) into grids [nsf][nports][2 nsymb][12 nof_prb] (nsymb = 7 normal CP, 6
// extended); d_sf_idx[sf] = tti % 10
hipError_t crs_put_launch(float2* d_grids, uint32_t nof_prb, uint32_t cell_id, uint32_t nports, uint32_t nsymb,
                          const uint32_t* d_sf_idx, uint32_t nsf, hipStream_t stream);

// One control-channel transmission of one subframe (enb_dl.c:333-420): bits -> scrambling -> QPSK ->
// transmit-diversity precoding -> REs, or a sequence copied as it is onto every port (PSS / SSS).
struct CtrlTxJob {
  float2*         grid[4];   // the subframe's port grids (2 nsymb x 12 nof_prb)
  const uint32_t* re;        // RE (k + l * 12 nof_prb) of each symbol; null: re0 + symbol index
  const float2*   seq;       // kind 2: the symbols (device)
  uint32_t        re0;
  uint32_t        nsym;      // symbols written (a multiple of nports for kinds 0 / 1)
  uint32_t        kind;      // 0: CRC16 + tail-biting convolutional code + rate matching (DCI, BCH);
                             // 1: the CFI codeword of cfi = nof_bits; 2: sequence
  uint32_t        nports;
  uint32_t        nof_bits;  // kind 0: payload bits before the CRC; kind 1: the CFI
  uint32_t        E;         // kind 0: rate-matched length
  uint32_t        bit0;      // kind 0: first rate-matched bit transmitted
  uint32_t        seed;      // scrambling: c_init
  uint32_t        seq_off;   // scrambling: sequence offset of the first transmitted bit
  uint32_t        crc_mask;  // kind 0: 16-bit CRC mask (RNTI, or the BCH antenna-port mask)
  uint32_t        skip;      // kind 0 (DCI): bit c set = CCE c of the message is not written (a later one
                             // takes it, as the reference's sequential puts overwrite)
  uint8_t         payload[128];  // kind 0: payload bits, one a byte
};
hipError_t ctrl_tx_launch(const CtrlTxJob* d_jobs, uint32_t njobs, hipStream_t stream);

}  // namespace srsran_amd
#endif
