/*
 * include/srsran_pusch.h -- MI355X PUSCH receive (eNB side): DMRS, UL channel estimation,
 * SC-FDMA transform de-precoding and srsran_pusch_decode, as a C-ABI drop-in.
 *
 * Replaces, with the reference's names, argument meaning and return codes:
 *   srsran_refsignal_dmrs_pusch_cfg_t / srsran_refsignal_dmrs_pusch_gen
 *                                     lib/include/srsran/phy/ch_estimation/refsignal_ul.h:46-51, 114-119
 *   srsran_chest_ul_t / _res_t, srsran_chest_ul_init / free / res_init / res_free / res_set_identity /
 *   set_cell / pregen / estimate_pusch  lib/include/srsran/phy/ch_estimation/chest_ul.h:40-125
 *   srsran_dft_precoding_valid_prb / get_valid_prb   lib/include/srsran/phy/dft/dft_precoding.h:47-49
 *   srsran_pusch_t, srsran_pusch_res_t, srsran_pusch_init_enb / free / set_cell / assert_grant /
 *   decode                            lib/include/srsran/phy/phch/pusch.h:43-110
 *   srsran_ul_sf_cfg_t                lib/include/srsran/phy/common/phy_common.h:255-259
 *
 * Buffers at this boundary are host memory, as in the reference (sf_symbols and the chest result
 * hold the subframe grid of nof_prb * 12 * 2 * N_symb(cp) REs).  Everything per RE runs on the GPU
 * (csrc/pusch_kernel.hip): DMRS least squares, the 3-tap smoothing, noise / CFO / TA / RSRP
 * reductions, the equaliser, the M-point inverse DFT (M = 12 * L_prb, L_prb = 2^a 3^b 5^c), soft
 * demapping, descrambling, then srsran_ulsch_decode's UCI / de-interleaver / decode_tb kernels.
 * srsran_pusch_gpu_decode_batch (added) takes device grids and estimates for many UEs.
 */
#ifndef SRSRAN_AMD_PUSCH_H
#define SRSRAN_AMD_PUSCH_H

#include <stdbool.h>
#include <stdint.h>

#include "srsran_ue_dl.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SRSRAN_NOF_CSHIFT 8        /* refsignal_ul.h:41 */
#define SRSRAN_NOF_DELTA_SS 30     /* refsignal_ul.h:40 */
#define SRSRAN_NOF_SF_X_FRAME 10   /* phy_common.h:51 */
#define SRSRAN_NSLOTS_X_FRAME 20   /* phy_common.h:52 */
#define SRSRAN_CHEST_MAX_SMOOTH_FIL_LEN 64 /* chest_common.h:28 */
/* DMRS symbol of slot ns_idx (refsignal_ul.h:43) */
#define SRSRAN_REFSIGNAL_UL_L(ns_idx, cp) (((ns_idx) + 1) * ((cp) == SRSRAN_CP_NORM ? 7 : 6) - 4)

typedef struct {
  srsran_tdd_config_t tdd_config;
  uint32_t            tti;
  bool                shortened;
} srsran_ul_sf_cfg_t;

/* PUSCH DMRS common configuration (SIB2) */
typedef struct {
  uint32_t cyclic_shift;
  uint32_t delta_ss;
  bool     group_hopping_en;
  bool     sequence_hopping_en;
} srsran_refsignal_dmrs_pusch_cfg_t;

/* Generate the PUSCH DMRS of one subframe (both slots, 2 * 12 * nof_prb values) for cell `cell`,
 * as refsignal_ul.c:338-358 (srsran_refsignal_ul_set_cell's hopping tables computed internally). */
int srsran_refsignal_dmrs_pusch_gen_cell(const srsran_cell_t*               cell,
                                         srsran_refsignal_dmrs_pusch_cfg_t* cfg,
                                         uint32_t                           nof_prb,
                                         uint32_t                           sf_idx,
                                         uint32_t                           cyclic_shift_for_dmrs,
                                         cf_t*                              r_pusch);

bool     srsran_dft_precoding_valid_prb(uint32_t nof_prb);
uint32_t srsran_dft_precoding_get_valid_prb(uint32_t nof_prb);
/* added, device-side srsran_dft_precoding (dft_precoding.c:114-126) of a receiver: the M-point
 * backward DFT (M = 12 nof_prb) normalised by 1 / sqrt(M) of nof_symbols <= 14 consecutive blocks,
 * asynchronous on `stream` (hipStream_t, NULL = default stream).  d_input / d_output: device. */
int srsran_dft_precoding_gpu(const cf_t* d_input, cf_t* d_output, uint32_t nof_prb, uint32_t nof_symbols, void* stream);

typedef struct {
  cf_t*    ce; /* host, nof_re = nof_prb * 12 * 2 * N_symb(cp) */
  uint32_t nof_re;
  float    noise_estimate;
  float    noise_estimate_dbFs;
  float    rsrp;
  float    rsrp_dBfs;
  float    epre;
  float    epre_dBfs;
  float    snr;
  float    snr_db;
  float    cfo_hz;
  float    ta_us;
  void*    gpu; /* added: device copy of ce (written by srsran_chest_ul_estimate_pusch) */
} srsran_chest_ul_res_t;

typedef struct {
  srsran_cell_t                     cell;
  srsran_refsignal_dmrs_pusch_cfg_t dmrs_cfg;
  bool                              dmrs_signal_configured;
  uint32_t                          smooth_filter_len;
  float                             smooth_filter[SRSRAN_CHEST_MAX_SMOOTH_FIL_LEN];
  void*                             gpu; /* added: pregenerated DMRS on the device, scratch, stream */
} srsran_chest_ul_t;

int  srsran_chest_ul_init(srsran_chest_ul_t* q, uint32_t max_prb);
void srsran_chest_ul_free(srsran_chest_ul_t* q);
int  srsran_chest_ul_res_init(srsran_chest_ul_res_t* q, uint32_t max_prb);
void srsran_chest_ul_res_set_identity(srsran_chest_ul_res_t* q);
void srsran_chest_ul_res_free(srsran_chest_ul_res_t* q);
int  srsran_chest_ul_set_cell(srsran_chest_ul_t* q, srsran_cell_t cell);
/* srs_cfg: SRS is not provided; pass NULL (a non-NULL srs_cfg is ignored) */
void srsran_chest_ul_pregen(srsran_chest_ul_t* q, srsran_refsignal_dmrs_pusch_cfg_t* cfg, void* srs_cfg);
/* chest_ul.c:398-433.  cfg->use_cedron_alg with cfg->meas_ta_en is not provided (FFTW-based in the
 * reference): SRSRAN_ERROR. */
int srsran_chest_ul_estimate_pusch(srsran_chest_ul_t*     q,
                                   srsran_ul_sf_cfg_t*    sf,
                                   srsran_pusch_cfg_t*    cfg,
                                   cf_t*                  input,
                                   srsran_chest_ul_res_t* res);

typedef struct {
  uint8_t*           data;
  srsran_uci_value_t uci;
  bool               crc;
  float              avg_iterations_block;
  float              evm;
  float              epre_dbfs;
} srsran_pusch_res_t;

typedef struct {
  srsran_cell_t cell;
  bool          is_ue;
  uint16_t      ue_rnti;
  uint32_t      max_re;
  bool          llr_is_8bit; /* the 8-bit LLR path is not provided: must stay false */
  srsran_sch_t  ul_sch;
  void*         gpu; /* added: device grid / estimate / symbol / LLR / sequence buffers */
} srsran_pusch_t;

int  srsran_pusch_init_enb(srsran_pusch_t* q, uint32_t max_prb);
void srsran_pusch_free(srsran_pusch_t* q);
int  srsran_pusch_set_cell(srsran_pusch_t* q, srsran_cell_t cell);
int  srsran_pusch_assert_grant(const srsran_pusch_grant_t* grant);
/* pusch.c:358-471.  channel: the srsran_chest_ul_estimate_pusch result (its device copy of ce is
 * used when present, else channel->ce is uploaded).  cfg->meas_evm_en is not provided (evm = NAN). */
int srsran_pusch_decode(srsran_pusch_t*        q,
                        srsran_ul_sf_cfg_t*    sf,
                        srsran_pusch_cfg_t*    cfg,
                        srsran_chest_ul_res_t* channel,
                        cf_t*                  sf_symbols,
                        srsran_pusch_res_t*    out);

/* ---- added: many UEs of one or more cells in a few launches ----
 * Per entry: the device subframe grid of its cell, the PUSCH configuration (UCI included) and the
 * cell's chest object (pregenerated DMRS).  Runs chest_ul_estimate_pusch + pusch_decode for all
 * entries: two launches for estimation and de-precoding, one LLR launch, then the UL-SCH decode of
 * each entry.  Results go to res[i] / chest_res[i] (host; chest_res[i].ce may be NULL).  Returns
 * SRSRAN_SUCCESS when every entry ran (per-entry CRC in res[i].crc). */
typedef struct {
  srsran_chest_ul_t*  chest;
  srsran_ul_sf_cfg_t* sf;
  srsran_pusch_cfg_t* cfg;
  const cf_t*         d_sf_symbols; /* device */
  uint32_t            new_data;     /* 1: as if srsran_softbuffer_rx_reset_tbs(softbuffer, tbs) ran first */
} srsran_pusch_gpu_ue_t;

int srsran_pusch_gpu_decode_batch(srsran_pusch_t*              q,
                                  uint32_t                     nof_ue,
                                  const srsran_pusch_gpu_ue_t* ues,
                                  srsran_chest_ul_res_t*       chest_res,
                                  srsran_pusch_res_t*          res);

#ifdef __cplusplus
}
#endif
#endif
