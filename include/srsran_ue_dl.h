/*
 * include/srsran_ue_dl.h -- DL receive front-end of the MI355X PHY: cell / subframe types,
 * CRS channel estimation, OFDM demodulation, PDSCH and UE DL orchestration.
 *
 * Drop-in for (types keep the reference's field order):
 *   lib/include/srsran/phy/common/phy_common.h:197-253     srsran_cell_t, srsran_dl_sf_cfg_t, ...
 *   lib/include/srsran/phy/ch_estimation/chest_dl.h:43-170  srsran_chest_dl_{t,cfg_t,res_t}, srsran_chest_dl_*
 * Channel estimation runs on the GPU (chest_kernel.hip).  Supported configuration: normal
 * subframes, normal CP, FDD, estimator AVERAGE with the Gauss smoothing filter and REFS noise
 * estimation -- srsUE's defaults (srsue/src/phy/phy_common.cc:83-107); other settings return
 * SRSRAN_ERROR.  srsran_chest_dl_t keeps the fields callers read (cell, nof_rx_antennas, rssi,
 * rsrp, noise_estimate, cfo) and hides the device state behind `gpu`.
 */
#ifndef SRSRAN_AMD_UE_DL_H
#define SRSRAN_AMD_UE_DL_H

#include <stdbool.h>
#include <stdint.h>

#include "srsran_phch.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SRSRAN_MAX_PORTS 4
#define SRSRAN_MAX_LAYERS 4
#define SRSRAN_NRE 12
#define SRSRAN_CP_NORM_NSYMB 7

/* ---------------- phy_common.h ---------------- */
typedef enum { SRSRAN_CP_NORM = 0, SRSRAN_CP_EXT } srsran_cp_t;
typedef enum { SRSRAN_PHICH_NORM = 0, SRSRAN_PHICH_EXT } srsran_phich_length_t;
typedef enum { SRSRAN_PHICH_R_1_6 = 0, SRSRAN_PHICH_R_1_2, SRSRAN_PHICH_R_1, SRSRAN_PHICH_R_2 } srsran_phich_r_t;
typedef enum { SRSRAN_FDD = 0, SRSRAN_TDD = 1 } srsran_frame_type_t;
typedef enum { SRSRAN_SF_NORM = 0, SRSRAN_SF_MBSFN } srsran_sf_t;

typedef struct {
  uint32_t              nof_prb;
  uint32_t              nof_ports;
  uint32_t              id;
  srsran_cp_t           cp;
  srsran_phich_length_t phich_length;
  srsran_phich_r_t      phich_resources;
  srsran_frame_type_t   frame_type;
} srsran_cell_t;

typedef struct {
  uint32_t sf_config;
  uint32_t ss_config;
  bool     configured;
} srsran_tdd_config_t;

typedef struct {
  srsran_tdd_config_t tdd_config;
  uint32_t            tti;
  uint32_t            cfi;
  srsran_sf_t         sf_type;
  uint32_t            non_mbsfn_region;
} srsran_dl_sf_cfg_t;

int srsran_symbol_sz(uint32_t nof_prb);              /* phy_common.c:361-385 (standard rates: powers of 2) */
int srsran_symbol_sz_power2(uint32_t nof_prb);       /* phy_common.c:340-359 */
void srsran_use_standard_symbol_size(bool enabled);  /* phy_common.c:322-325 (only `true` is provided) */

/* ---------------- chest_dl.h ---------------- */
typedef enum { SRSRAN_NOISE_ALG_REFS = 0, SRSRAN_NOISE_ALG_PSS, SRSRAN_NOISE_ALG_EMPTY } srsran_chest_dl_noise_alg_t;
typedef enum {
  SRSRAN_ESTIMATOR_ALG_AVERAGE = 0,
  SRSRAN_ESTIMATOR_ALG_INTERPOLATE,
  SRSRAN_ESTIMATOR_ALG_WIENER
} srsran_chest_dl_estimator_alg_t;
typedef enum { SRSRAN_CHEST_FILTER_GAUSS = 0, SRSRAN_CHEST_FILTER_TRIANGLE, SRSRAN_CHEST_FILTER_NONE } srsran_chest_filter_t;

typedef struct {
  srsran_chest_dl_estimator_alg_t estimator_alg;
  srsran_chest_dl_noise_alg_t     noise_alg;
  srsran_chest_filter_t           filter_type;
  float                           filter_coef[2];
  uint16_t                        mbsfn_area_id;
  bool                            rsrp_neighbour;
  bool                            cfo_estimate_enable;
  uint32_t                        cfo_estimate_sf_mask;
  bool                            sync_error_enable;
} srsran_chest_dl_cfg_t;

typedef struct {
  cf_t*    ce[SRSRAN_MAX_PORTS][SRSRAN_MAX_PORTS]; /* [port][rx], 14 * 12 * nof_prb each (host) */
  uint32_t nof_re;
  float    noise_estimate;
  float    noise_estimate_dbm;
  float    snr_db;
  float    snr_ant_port_db[SRSRAN_MAX_PORTS][SRSRAN_MAX_PORTS];
  float    rsrp;
  float    rsrp_dbm;
  float    rsrp_neigh;
  float    rsrp_port_dbm[SRSRAN_MAX_PORTS];
  float    rsrp_ant_port_dbm[SRSRAN_MAX_PORTS][SRSRAN_MAX_PORTS];
  float    rsrq;
  float    rsrq_db;
  float    rsrq_ant_port_db[SRSRAN_MAX_PORTS][SRSRAN_MAX_PORTS];
  float    rssi_dbm;
  float    cfo;
  float    sync_error;
} srsran_chest_dl_res_t;

typedef struct {
  srsran_cell_t cell;
  uint32_t      nof_rx_antennas;
  float         rssi[SRSRAN_MAX_PORTS][SRSRAN_MAX_PORTS];
  float         rsrp[SRSRAN_MAX_PORTS][SRSRAN_MAX_PORTS];
  float         noise_estimate[SRSRAN_MAX_PORTS][SRSRAN_MAX_PORTS];
  float         cfo;
  void*         gpu; /* added: device CRS tables and scratch */
} srsran_chest_dl_t;

int  srsran_chest_dl_init(srsran_chest_dl_t* q, uint32_t max_prb, uint32_t nof_rx_antennas);
void srsran_chest_dl_free(srsran_chest_dl_t* q);
int  srsran_chest_dl_set_cell(srsran_chest_dl_t* q, srsran_cell_t cell);
int  srsran_chest_dl_res_init(srsran_chest_dl_res_t* q, uint32_t max_prb);
void srsran_chest_dl_res_free(srsran_chest_dl_res_t* q);
int  srsran_chest_dl_estimate(srsran_chest_dl_t* q, srsran_dl_sf_cfg_t* sf, cf_t* input[SRSRAN_MAX_PORTS],
                              srsran_chest_dl_res_t* res);
int  srsran_chest_dl_estimate_cfg(srsran_chest_dl_t*     q,
                                  srsran_dl_sf_cfg_t*    sf,
                                  srsran_chest_dl_cfg_t* cfg,
                                  cf_t*                  input[SRSRAN_MAX_PORTS],
                                  srsran_chest_dl_res_t* res);

/* added: device-resident estimate.  d_grid: nof_rx_antennas grids of 14 * 12 * nof_prb cf_t,
 * back to back; d_ce: [port][rx] rows of 12 * nof_prb (full_grid = 0: the AVERAGE estimate is
 * the same for every symbol) or of 14 * 12 * nof_prb (full_grid = 1).  d_res (4 floats:
 * noise_estimate, rsrp, rssi, cfo as srsran_chest_dl_res_t defines them) is written on the
 * device.  Asynchronous on `stream`. */
int srsran_chest_dl_gpu_estimate(srsran_chest_dl_t* q,
                                 uint32_t           tti,
                                 const cf_t*        d_grid,
                                 cf_t*              d_ce,
                                 int                full_grid,
                                 float*             d_res,
                                 void*              stream);

#ifdef __cplusplus
}
#endif
#endif
