/*
 * include/srsran_enb_dl.h -- MI355X eNB downlink transmit (the TX side that makes
 * C3 / C4 generation device-resident).
 *
 * Replaces, per subframe:
 *   srsran_enb_dl_put_base (enb_dl.c:333-382): PSS / SSS in subframes 0 and 5 (pss.c:341-379,
 *     sss.c:105-119, gen_sss.c), the CRS (refsignal_cs_put_sf), the PBCH with the MIB of SFN tti / 10
 *     in subframe 0 (pbch.c srsran_pbch_mib_pack / srsran_pbch_encode), the PCFICH (pcfich.c:185-235),
 *   srsran_enb_dl_put_pdcch_dl / _ul (enb_dl.c:392-428 -> srsran_pdcch_encode, pdcch.c:528-660) of
 *     messages packed with srsran_dci_msg_pack_pdsch / _pusch,
 *   srsran_enb_dl_put_pdsch (enb_dl.c:436-439 -> srsran_pdsch_encode, pdsch.c:1015-1120:
 *     srsran_dlsch_encode2, srsran_sequence_pdsch_apply_pack, srsran_mod_modulate_bytes,
 *     srsran_layermap_type / srsran_precoding_type, srsran_pdsch_put),
 *   srsran_enb_dl_gen_signal (enb_dl.c:446-470: amplitude 0.05 / sqrt(N_RB), srsran_ofdm_tx_sf).
 * Transmission schemes: PORT0 (1 port), TX diversity (2 or 4 ports, 1 TB), CDD (2 ports, 2 TBs); normal or
 * extended CP;
 * rho_a = 1.  Not generated here (their REs stay empty): PHICH, MBSFN subframes.
 */
#ifndef SRSRAN_AMD_ENB_DL_H
#define SRSRAN_AMD_ENB_DL_H

#include "srsran_pdcch.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  srsran_cell_t cell;
  void*         gpu; /* added: encoder (srsran_sch_t), modulator (srsran_ofdm_t), grids, tables */
} srsran_enb_dl_gpu_t;

/* Control channels of one subframe. */
typedef struct {
  uint32_t                put_base; /* 1: PSS / SSS / PBCH / PCFICH as srsran_enb_dl_put_base adds them */
  uint32_t                nof_dci;
  const srsran_dci_msg_t* dci;      /* host: packed DCI messages (payload, nof_bits, location, rnti), put in
                                       order as srsran_enb_dl_put_pdcch_dl / _ul would (a later message
                                       overwrites the CCEs it shares with an earlier one) */
} srsran_enb_dl_gpu_ctrl_t;

typedef struct {
  uint32_t                        tti;
  uint32_t                        cfi;
  srsran_pdsch_cfg_t*             cfg;  /* grant: tx_scheme, nof_layers, prb_idx, tb[], rnti; NULL: no PDSCH */
  const uint8_t*                  d_data[SRSRAN_MAX_CODEWORDS]; /* device payloads of the enabled TBs (tbs / 8 bytes) */
  const srsran_enb_dl_gpu_ctrl_t* ctrl; /* added: control channels, NULL: none */
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

/* Device grids of the last batch, [nof_sf][cell.nof_ports][2 nsymb][12 nof_prb] cf_t (the reference's
 * q->sf_symbols, before srsran_enb_dl_gen_signal's scaling); valid until the next batch. */
const cf_t* srsran_enb_dl_gpu_sf_symbols(srsran_enb_dl_gpu_t* q);

/* The 24 MIB bits of SFN sfn (pbch.c srsran_pbch_mib_pack): bandwidth, PHICH duration and resources,
 * the 8 most significant SFN bits, 10 spare bits. */
void srsran_pbch_mib_pack(srsran_cell_t* cell, uint32_t sfn, uint8_t* payload);

#ifdef __cplusplus
}
#endif
#endif
