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
  float                           pdsch_scaling; /* the precoder's scaling (srsran_pdsch_encode's rho_a, pdsch.c:492,
                                                    1066-1070); <= 0: 1 */
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

/* ---------------- enb/enb_dl.h (enb_dl.h:101-124): the reference's per-subframe eNB DL object ----------------
 * A srsENB caller's sequence per subframe, as lib/test/phy/phy_dl_test.c:152-196 and srsenb's cc_worker use it:
 *   srsran_enb_dl_put_base -> srsran_enb_dl_put_pdcch_dl / _ul (each DCI packed with srsran_dci_msg_pack_pdsch /
 *   _pusch at once, as enb_dl.c:392-428) -> srsran_enb_dl_put_pdsch -> srsran_enb_dl_gen_signal.
 * The puts record the subframe (the payloads copied to the device at once, so the caller may reuse its buffers);
 * srsran_enb_dl_gen_signal runs it through srsran_enb_dl_gpu_tx_batch (one subframe) and returns with the time
 * samples of every port in out_buffer[port] (host, SRSRAN_SF_LEN(symbol_sz) samples, the reference's amplitude
 * 0.05 / sqrt(N_RB)) and the grids in sf_symbols[port] (host, before that scaling).  PDSCH scaling rho_a =
 * 10^(p_a / 20) x (sqrt 2 with more than one port) as srsran_pdsch_encode applies it (pdsch.c:492, 1066-1070).
 * Every subframe starts from srsran_enb_dl_put_base (the reference clears the grid there, enb_dl.c:376); a
 * subframe without it carries nothing of the previous one.  Not provided (their REs stay empty, an error message):
 * srsran_enb_dl_put_phich, srsran_enb_dl_put_pmch and MBSFN subframes. */
typedef struct {
  srsran_cell_t         cell;
  srsran_dl_sf_cfg_t    dl_sf;
  cf_t*                 sf_symbols[SRSRAN_MAX_PORTS];  /* host: the last generated subframe's grids */
  cf_t*                 out_buffer[SRSRAN_MAX_PORTS];  /* host: the caller's time-sample buffers (srsran_enb_dl_init) */
  srsran_regs_t         regs;
  srsran_pdcch_t        pdcch;  /* cell, nof_regs / nof_cce a CFI: srsran_pdcch_ue_locations(&q->pdcch, ...) */
  uint32_t              nof_common_locations[3];
  srsran_dci_location_t common_locations[3][SRSRAN_MAX_CANDIDATES_COM];
  void*                 gpu; /* added: the batched transmitter, the recorded subframe, device buffers */
} srsran_enb_dl_t;

int  srsran_enb_dl_init(srsran_enb_dl_t* q, cf_t* out_buffer[SRSRAN_MAX_PORTS], uint32_t max_prb); /* enb_dl.c:33-117 */
void srsran_enb_dl_free(srsran_enb_dl_t* q);                                                          /* enb_dl.c:119-140 */
int  srsran_enb_dl_set_cell(srsran_enb_dl_t* q, srsran_cell_t cell);                                  /* enb_dl.c:142-235 */
bool srsran_enb_dl_location_is_common_ncce(srsran_enb_dl_t* q, const srsran_dci_location_t* loc);    /* enb_dl.c:384-390 */
void srsran_enb_dl_put_base(srsran_enb_dl_t* q, srsran_dl_sf_cfg_t* dl_sf);                           /* enb_dl.c:372-382 */
int  srsran_enb_dl_put_pdcch_dl(srsran_enb_dl_t* q, srsran_dci_cfg_t* dci_cfg, srsran_dci_dl_t* dci_dl); /* :392-408 */
int  srsran_enb_dl_put_pdcch_ul(srsran_enb_dl_t* q, srsran_dci_cfg_t* dci_cfg, srsran_dci_ul_t* dci_ul); /* :410-428 */
int  srsran_enb_dl_put_pdsch(srsran_enb_dl_t* q, srsran_pdsch_cfg_t* pdsch, uint8_t* data[SRSRAN_MAX_CODEWORDS]);
void srsran_enb_dl_gen_signal(srsran_enb_dl_t* q);                                                    /* enb_dl.c:446-470 */
float srsran_enb_dl_get_maximum_signal_power_dBfs(uint32_t nof_prb);                                 /* enb_dl.c:472-477 */

#ifdef __cplusplus
}
#endif
#endif
