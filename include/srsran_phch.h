/*
 * include/srsran_phch.h -- PDSCH LLR stages of the MI355X DL receive path.
 *
 * Drop-in for:
 *   lib/include/srsran/phy/modem/demod_soft.h:30-36   srsran_demod_soft_demodulate_s
 *   lib/include/srsran/phy/common/sequence.h:82        srsran_sequence_apply_s
 *   lib/include/srsran/phy/phch/sequences.h            srsran_sequence_pdsch_apply_s
 * Host pointers, host-synchronous, executed by the HIP kernels of llr_kernel.hip; results are
 * bit-exact with the reference's x86 SSE/AVX2 build ("PDSCH LLR stages").
 * The added srsran_pdsch_gpu_llr() fuses demapping and descrambling over device buffers.
 */
#ifndef SRSRAN_AMD_PHCH_H
#define SRSRAN_AMD_PHCH_H

#include <stdint.h>

#include "srsran_sch.h"

#ifdef __cplusplus
#include <complex>
typedef std::complex<float> cf_t;
extern "C" {
#else
#include <complex.h>
typedef _Complex float cf_t;
#endif

/* demod_soft.c:871-894: int16 soft demapping, LLR > 0 <=> bit 1 after the sign convention of the
 * reference (-scale * y) */
int srsran_demod_soft_demodulate_s(srsran_mod_t modulation, const cf_t* symbols, short* llr, int nsymbols);

/* sequence.c:507-561: out[i] = c(i) ? -in[i] : in[i] for the LTE Gold sequence of `seed` */
void srsran_sequence_apply_s(const int16_t* in, int16_t* out, uint32_t length, uint32_t seed);

/* sequences.c:95-103: seed = rnti*2^14 + q*2^13 + (nslot/2)*2^9 + cell_id (36.211 6.3.1) */
void srsran_sequence_pdsch_apply_s(const int16_t* in,
                                   int16_t*       out,
                                   uint16_t       rnti,
                                   int            q,
                                   uint32_t       nslot,
                                   uint32_t       cell_id,
                                   uint32_t       len);

/* added: fused demap + descramble (+ CSI correction, pdsch.c:523-618) on device buffers,
 * asynchronous on `stream` (a hipStream_t; NULL = default stream).  d_symbols: nsymbols cf_t;
 * d_llr: nsymbols * Qm int16.  scramble = 0 skips the descrambling; d_csi (per symbol) with
 * d_csi_max (one float, e.g. from srsran_predecoding_gpu) enables the CSI correction. */
int srsran_pdsch_gpu_llr(srsran_mod_t modulation,
                         const cf_t*  d_symbols,
                         uint32_t     nsymbols,
                         int          scramble,
                         uint32_t     seed,
                         const float* d_csi,
                         const float* d_csi_max,
                         int16_t*     d_llr,
                         void*        stream);

/* ---- MIMO predecoding (precoding.c:1866-1930 srsran_predecoding_type), MMSE with CSI ----
 * Host pointers, host-synchronous.  Supported: PORT0 (1 port, 1..4 rx), CDD and SPATIALMUX
 * (2 ports, 2 rx, 2 layers; codebooks 0..2).  csi may be NULL. */
int srsran_predecoding_type(cf_t*              y[4],
                            cf_t*              h[4][4],
                            cf_t*              x[4],
                            float*             csi[2],
                            int                nof_rxant,
                            int                nof_ports,
                            int                nof_layers,
                            int                codebook_idx,
                            int                nof_symbols,
                            srsran_tx_scheme_t type,
                            float              scaling,
                            float              noise_estimate);

/* added: the same on device buffers; d_csi_max (2 floats, or NULL) receives the per-layer CSI
 * maximum (the caller zeroes it first). */
int srsran_predecoding_gpu(const cf_t* const d_y[4],
                           const cf_t* const d_h[4][4],
                           cf_t* const       d_x[4],
                           float* const      d_csi[2],
                           float*            d_csi_max,
                           int               nof_rxant,
                           int               nof_ports,
                           int               nof_layers,
                           int               codebook_idx,
                           int               nof_symbols,
                           srsran_tx_scheme_t type,
                           float              scaling,
                           float              noise_estimate,
                           void*              stream);

#ifdef __cplusplus
}
#endif
#endif
