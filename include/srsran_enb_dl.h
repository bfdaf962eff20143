/*
 * include/srsran_enb_dl.h -- MI355X eNB downlink transmit for PDSCH subframes (SURVEY §8f rank 4:
 * the TX side that makes C3 / C4 generation device-resident).
 *
 * Replaces, for subframes carrying CRS + PDSCH:
 *   srsran_enb_dl_put_base's CRS (enb_dl.c:300-330 -> srsran_refsignal_cs_put_sf),
 *   srsran_enb_dl_put_pdsch (enb_dl.c:436-439 -> srsran_pdsch_encode, pdsch.c:1015-1120:
 *     srsran_dlsch_encode2, srsran_sequence_pdsch_apply_pack, srsran_mod_modulate_bytes,
 *     srsran_layermap_type / srsran_precoding_type, srsran_pdsch_put),
 *   srsran_enb_dl_gen_signal (enb_dl.c:446-470: amplitude 0.05 / sqrt(N_RB), srsran_ofdm_tx_sf).
 * Transmission schemes: PORT0 (1 port), TX diversity (2 or 4 ports, 1 TB), CDD (2 ports, 2 TBs); normal or
 * extended CP;
 * rho_a = 1.  Not generated here (their REs stay empty): PSS / SSS, PBCH, PCFICH, PHICH, PDCCH.
 */
#ifndef SRSRAN_AMD_ENB_DL_H
#define SRSRAN_AMD_ENB_DL_H

#include "srsran_ue_dl.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  srsran_cell_t cell;
  void*         gpu; /* added: encoder (srsran_sch_t), modulator (srsran_ofdm_t), grids, tables */
} srsran_enb_dl_gpu_t;

typedef struct {
  uint32_t            tti;
  uint32_t            cfi;
  srsran_pdsch_cfg_t* cfg;                          /* grant: tx_scheme, nof_layers, prb_idx, tb[], rnti */
  const uint8_t*      d_data[SRSRAN_MAX_CODEWORDS]; /* device payloads of the enabled TBs (tbs / 8 bytes) */
} srsran_enb_dl_gpu_sf_t;

int  srsran_enb_dl_gpu_init(srsran_enb_dl_gpu_t* q, srsran_cell_t cell);
void srsran_enb_dl_gpu_free(srsran_enb_dl_gpu_t* q);
/* nof_sf subframes -> d_samples [nof_sf][cell.nof_ports][SRSRAN_SF_LEN(symbol_sz)] (device), the grid
 * scaled by `scale` before the modulator (scale <= 0: the reference's 0.05 / sqrt(N_RB)); every TB's
 * nof_bits must equal the grant's PDSCH REs x Qm (x 2 for transmit diversity's codeword).
 * Asynchronous on `stream` after the host has built the RE tables. */
int srsran_enb_dl_gpu_tx_batch(srsran_enb_dl_gpu_t*          q,
                               uint32_t                      nof_sf,
                               const srsran_enb_dl_gpu_sf_t* sfs,
                               cf_t*                         d_samples,
                               float                         scale,
                               void*                         stream);

#ifdef __cplusplus
}
#endif
#endif
