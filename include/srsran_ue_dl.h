/*
 * include/srsran_ue_dl.h -- DL receive front-end of the MI355X PHY: cell / subframe types,
 * CRS channel estimation, OFDM demodulation, PDSCH and UE DL orchestration.
 *
 * Drop-in for (types keep the reference's field order):
 *   lib/include/srsran/phy/common/phy_common.h:197-253     srsran_cell_t, srsran_dl_sf_cfg_t, ...
 *   lib/include/srsran/phy/ch_estimation/chest_dl.h:43-170  srsran_chest_dl_{t,cfg_t,res_t}, srsran_chest_dl_*
 * Channel estimation runs on the GPU (chest_kernel.hip).  Supported configuration: normal
 * subframes, normal or extended CP, FDD, 1/2/4 ports, estimator AVERAGE with the Gauss smoothing filter and REFS noise
 * estimation -- srsUE's defaults (srsue/src/phy/phy_common.cc:83-107); other settings return
 * SRSRAN_ERROR.  srsran_chest_dl_t keeps the fields callers read (cell, nof_rx_antennas, rssi,
 * rsrp, noise_estimate, cfo) and hides the device state behind `gpu`.
 */
#ifndef SRSRAN_AMD_UE_DL_H
#define SRSRAN_AMD_UE_DL_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#include "srsran_phch.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SRSRAN_MAX_PORTS 4
#define SRSRAN_MAX_LAYERS 4
#define SRSRAN_NRE 12
#define SRSRAN_CP_NORM_NSYMB 7
#define SRSRAN_CP_EXT_NSYMB 6

/* ---------------- phy_common.h ---------------- */
typedef enum { SRSRAN_CP_NORM = 0, SRSRAN_CP_EXT } srsran_cp_t;
#define SRSRAN_CP_ISNORM(cp) (cp == SRSRAN_CP_NORM)
#define SRSRAN_CP_ISEXT(cp) (cp == SRSRAN_CP_EXT)
#define SRSRAN_CP_NSYMB(cp) (SRSRAN_CP_ISNORM(cp) ? SRSRAN_CP_NORM_NSYMB : SRSRAN_CP_EXT_NSYMB)
#define SRSRAN_SF_LEN_RE(nof_prb, cp) (2 * SRSRAN_CP_NSYMB(cp) * SRSRAN_NRE * (nof_prb))
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

/* TDD frame structure (phy_common.h:200-225, 396-427; phy_common.c:92-182): the 7 uplink-downlink and 10
 * special-subframe configurations of 36.211 Tables 4.2-2 / 4.2-1.  An unconfigured tdd_config makes every
 * subframe a downlink one, as in the reference. */
#define SRSRAN_MAX_TDD_SS_CONFIGS (10u)
#define SRSRAN_MAX_TDD_SF_CONFIGS (7u)
typedef enum { SRSRAN_TDD_SF_D = 0, SRSRAN_TDD_SF_U = 1, SRSRAN_TDD_SF_S = 2 } srsran_tdd_sf_t;
srsran_tdd_sf_t srsran_sfidx_tdd_type(srsran_tdd_config_t tdd_config, uint32_t sf_idx);              /* phy_common.c:111-118 */
uint32_t        srsran_sfidx_tdd_nof_up(srsran_tdd_config_t tdd_config);                           /* phy_common.c:169-176 */
uint32_t        srsran_sfidx_tdd_nof_gp(srsran_tdd_config_t tdd_config);                           /* phy_common.c:160-167 */
uint32_t        srsran_sfidx_tdd_nof_dw(srsran_tdd_config_t tdd_config);                           /* phy_common.c:151-158 */
uint32_t        srsran_tdd_nof_harq(srsran_tdd_config_t tdd_config);                               /* phy_common.c:178-182 */
uint32_t        srsran_sfidx_tdd_nof_dw_slot(srsran_tdd_config_t tdd_config, uint32_t slot, srsran_cp_t cp); /* :120-136 */

typedef struct {
  srsran_tdd_config_t tdd_config;
  uint32_t            tti;
  uint32_t            cfi;
  srsran_sf_t         sf_type;
  uint32_t            non_mbsfn_region;
} srsran_dl_sf_cfg_t;

/* FFT size per bandwidth.  As in the reference (phy_common.c:31-35), the default is the
 * non-standard 3/4 sampling rate (100 PRB -> 1536, 50 -> 768, 25 -> 384); srsUE and the
 * reference tests switch to power-of-two sizes with srsran_use_standard_symbol_size(true).
 * Both settings are implemented (mixed-radix FFT, radix 8/4/3/2). */
int  srsran_symbol_sz(uint32_t nof_prb);              /* phy_common.c:361-385 */
int  srsran_symbol_sz_power2(uint32_t nof_prb);       /* phy_common.c:340-359 */
void srsran_use_standard_symbol_size(bool enabled);  /* phy_common.c:322-325 */
bool srsran_symbol_size_is_standard(void);           /* phy_common.c:327-330 */
int  srsran_sampling_freq_hz(uint32_t nof_prb);      /* phy_common.c:332-338 */
int  srsran_nof_prb(uint32_t symbol_sz);             /* phy_common.c:387-419 */
bool srsran_symbol_sz_isvalid(uint32_t symbol_sz);   /* phy_common.c:421-437 */

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
/* chest_dl.c:263-278: the MBSFN reference signals of area mbsfn_area_id (refsignal_dl.c:382-422), generated once
 * per area with the cell set at that time.  srsran_chest_dl_estimate_cfg then estimates subframes with
 * sf->sf_type = SRSRAN_SF_MBSFN (estimate_port_mbsfn, chest_dl.c:836-865): the CRS of symbol 0 and the MBSFN
 * reference signals of symbols 2 / 6 / 10, INTERPOLATE (the reference requires it, chest_dl.c:719-721), REFS /
 * PSS / EMPTY noise, Gauss / TRIANGLE / NONE filters; rows 0..11 of res->ce are written, RSRP / RSSI / CFO keep
 * their previous values (the reference does not measure them there).  Refused: AVERAGE, ports 2 / 3 (their
 * interpolation reads row 0, which the reference does not write for them), subframes 0 / 5. */
int  srsran_chest_dl_set_mbsfn_area_id(srsran_chest_dl_t* q, uint16_t mbsfn_area_id);

/* added: nof_sf subframes in one launch (srsUE default configuration).  d_sf_idx[b] = tti % 10
 * of subframe b (device array); d_grid + b * grid_sf_stride: nof_rx grids; d_ce + b *
 * ce_sf_stride: [port][rx] rows of 12 * nof_prb (the AVERAGE estimate); d_res + 4 * b: noise_estimate,
 * rsrp, rssi, cfo.  Asynchronous on `stream`. */
int srsran_chest_dl_gpu_estimate_batch(srsran_chest_dl_t* q,
                                       const uint32_t*    d_sf_idx,
                                       uint32_t           nof_sf,
                                       const cf_t*        d_grid,
                                       size_t             grid_sf_stride,
                                       cf_t*              d_ce,
                                       size_t             ce_sf_stride,
                                       float*             d_res,
                                       void*              stream);

/* added: the batch with an estimator configuration (srsran_chest_dl_estimate_cfg's options): AVERAGE or
 * INTERPOLATE (full_grid = 1 required: d_ce rows of 2 * nsymb * 12 * nof_prb), REFS / PSS / EMPTY noise (PSS /
 * EMPTY estimate in subframes 0 and 5, the other subframes keep the last estimate, across calls as the reference's
 * q->noise_estimate does), Gauss filters of order <= 7 or automatic (with PSS / EMPTY noise the batch runs in
 * segments ending at subframes 0 / 5, whose estimate sets the later subframes' filter), and sync_error_enable
 * (correct_sync_error: each subframe's grids are corrected in place before the estimate, as the reference corrects
 * its input).  cfg = NULL: srsUE's defaults. */
int srsran_chest_dl_gpu_estimate_batch_cfg(srsran_chest_dl_t*           q,
                                           const srsran_chest_dl_cfg_t* cfg,
                                           const uint32_t*              d_sf_idx,
                                           uint32_t                     nof_sf,
                                           const cf_t*                  d_grid,
                                           size_t                       grid_sf_stride,
                                           cf_t*                        d_ce,
                                           size_t                       ce_sf_stride,
                                           int                          full_grid,
                                           float*                       d_res,
                                           void*                        stream);

/* added: the TDD frame configuration the batch estimators assume (sf->tdd_config of srsran_chest_dl_estimate_cfg):
 * special subframes of a TDD cell have fewer CRS symbols in their DwPTS (refsignal_dl.c:169-226).  Ignored for FDD
 * cells.  srsran_ue_dl_gpu_decode_batch sets it from its subframes. */
int srsran_chest_dl_gpu_set_tdd_config(srsran_chest_dl_t* q, srsran_tdd_config_t tdd_config);

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

/* ---------------- OFDM receiver (dft/ofdm.h:49-151, ofdm.c) ----------------
 * GPU FFT (mixed radix 8/4/3/2: 128..2048 points incl. 1536/768/384), no FFTW.  Normal or extended CP and every
 * srsran_ofdm_cfg_t option of the receiver and the modulator: normalize, keep_dc, freq_shift_f (the samples times
 * shift_buffer: the receiver's input, in place as ofdm.c:553-555 / 569-571, the modulator's output; DC then kept),
 * rx_window_offset (clamped to [0, 100] and written back as ofdm.c:151-157; window_offset_n = round(cp x offset)
 * samples into each symbol's cyclic prefix, its phase ramp removed per bin -- an offset whose window leaves the cyclic
 * prefix, i.e. above 1, returns SRSRAN_ERROR where the reference reads before its buffer), phase_compensation_hz
 * (per-symbol phasors, ofdm.c:357-406; set_prb turns it off as ofdm_init_mbsfn_ does).  No CFR (cfr_tx_cfg is not
 * part of this struct: srsran_enb_dl does not enable it).
 * in_buffer / out_buffer are host pointers as in the reference.  sf_type = SRSRAN_SF_MBSFN (with extended CP, as
 * srsran_ue_dl's fft_mbsfn): slot 0 holds the non-MBSFN region's normal-CP symbols, the guard, then extended-CP
 * symbols (ofdm_rx_slot_mbsfn, ofdm.c:522-535); like the reference, such an object transforms its configured
 * buffers even when srsran_ofdm_rx_sf_ng names others (ofdm.c:576-578). */
typedef struct {
  uint32_t    nof_prb;
  cf_t*       in_buffer;
  cf_t*       out_buffer;
  srsran_cp_t cp;
  srsran_sf_t sf_type;
  bool        normalize;
  float       freq_shift_f;
  float       rx_window_offset;
  uint32_t    symbol_sz;
  bool        keep_dc;
  double      phase_compensation_hz;
} srsran_ofdm_cfg_t;

typedef struct {
  srsran_ofdm_cfg_t cfg;
  uint32_t          max_prb;
  uint32_t          nof_symbols;
  uint32_t          nof_re;
  uint32_t          slot_sz;
  uint32_t          sf_sz;
  void*             gpu; /* added: device plan, twiddles and staging */
} srsran_ofdm_t;

int  srsran_ofdm_rx_init_cfg(srsran_ofdm_t* q, srsran_ofdm_cfg_t* cfg);
int  srsran_ofdm_rx_set_prb(srsran_ofdm_t* q, srsran_cp_t cp, uint32_t nof_prb);
void srsran_ofdm_rx_free(srsran_ofdm_t* q);
void srsran_ofdm_rx_sf(srsran_ofdm_t* q);
void srsran_ofdm_rx_sf_ng(srsran_ofdm_t* q, cf_t* input, cf_t* output);
void srsran_ofdm_set_normalize(srsran_ofdm_t* q, bool normalize_enable);
int  srsran_ofdm_rx_init_mbsfn(srsran_ofdm_t* q, srsran_cp_t cp, cf_t* in_buffer, cf_t* out_buffer, uint32_t max_prb);
void srsran_ofdm_set_non_mbsfn_region(srsran_ofdm_t* q, uint8_t non_mbsfn_region); /* ofdm.c:241-244 */
int  srsran_ofdm_set_freq_shift(srsran_ofdm_t* q, float freq_shift);               /* ofdm.c:421-449 */
int  srsran_ofdm_set_phase_compensation(srsran_ofdm_t* q, double center_freq_hz);  /* ofdm.c:357-410 */

/* added: nof_sf subframes x nof_rx antennas on device buffers (d_in: [sf][rx][sf_sz] samples,
 * d_out: [sf][rx][14 * nof_re]); `cfo` rotates the samples as srsran_cfo_correct(.., cfo) would
 * (0 = none).  Asynchronous on `stream`. */
int srsran_ofdm_rx_gpu(srsran_ofdm_t* q, const cf_t* d_in, cf_t* d_out, uint32_t nof_rx, uint32_t nof_sf, float cfo,
                       void* stream);
/* added: the same from the radio's int16 I/Q samples (d_in: [sf][rx][sf_sz][2] int16 on the device), each converted
 * as the host would convert them, (float)i * scale and (float)q * scale, inside the transform's sample load: half
 * the bytes of cf_t samples to move from a host buffer (the result equals srsran_ofdm_rx_gpu on the converted
 * samples).  Asynchronous on `stream`. */
int srsran_ofdm_rx_gpu_sc16(srsran_ofdm_t* q, const int16_t* d_in, float scale, cf_t* d_out, uint32_t nof_rx,
                            uint32_t nof_sf, float cfo, void* stream);

/* Modulator (ofdm.c:585-690): the receiver's options above (srsran_enb_dl's configuration: normalize = false, DC
 * subcarrier left empty, no frequency shift; no MBSFN subframes).  srsran_ofdm_tx_sf: cfg.in_buffer (one
 * port's 2 nsymb x 12 nof_prb grid, host) -> cfg.out_buffer (SRSRAN_SF_LEN samples, host).  Added:
 * srsran_ofdm_tx_gpu on device grids [nof_sf][nof_ports][2 nsymb][12 nof_prb] -> samples
 * [nof_sf][nof_ports][sf_len], the grid scaled by `scale` first (srsran_enb_dl_gen_signal's
 * 0.05 / sqrt(nof_prb)); asynchronous on `stream`. */
int  srsran_ofdm_tx_init_cfg(srsran_ofdm_t* q, srsran_ofdm_cfg_t* cfg);
void srsran_ofdm_tx_free(srsran_ofdm_t* q);
void srsran_ofdm_tx_sf(srsran_ofdm_t* q);
int  srsran_ofdm_tx_gpu(srsran_ofdm_t* q, const cf_t* d_in, cf_t* d_out, uint32_t nof_ports, uint32_t nof_sf, float scale,
                        void* stream);

/* ---------------- PDSCH RE map (added; srsran_pdsch_cp pdsch.c:136-220 as a table) ----------------
 * Number of PDSCH REs of `grant`; writes up to max_len grid indices (l * 12 * nof_prb + k) in
 * srsran_pdsch_get order; bit 31 marks REs of CRS-bearing symbols. */
int srsran_pdsch_re_table(const srsran_cell_t*        cell,
                          const srsran_pdsch_grant_t* grant,
                          uint32_t                    lstart,
                          uint32_t                    sf_idx,
                          uint32_t*                   idx,
                          uint32_t                    max_len);

/* ---------------- PDSCH (phch/pdsch.h:48-111, pdsch.c:788-958) ----------------
 * srsran_pdsch_decode runs on the GPU: RE extraction fused into the MMSE predecoder (gather
 * through the srsran_pdsch_re_table order), rho_b scaling of CRS symbols fused there too,
 * demapping + descrambling + CSI correction fused into one LLR kernel, then DL-SCH decode.
 * Provided: PORT0 (1 port), TX diversity (2 or 4 ports, 1 codeword; layer demap fused), CDD and
 * SPATIALMUX (2 ports x 2 rx, 1 or 2 codewords on 2 layers), MMSE (ZF = MMSE with noise 0, as
 * pdsch.c:811 passes it), 16- and 8-bit LLRs (llr_is_8bit), EVM (meas_evm_en), normal and extended CP, FDD and
 * TDD cells (DwPTS grants of special subframes).
 * Not provided (SRSRAN_ERROR): 4-port CDD / SM (refused by the reference too), MBSFN subframes (the PMCH).
 * The host-side working buffers of the reference struct (ce, symbols, x, d, e, csi) do not
 * exist; the coworker thread is unnecessary (both codewords decode in one GPU pass). */
typedef struct {
  srsran_cell_t cell;
  uint32_t      nof_rx_antennas;
  uint32_t      max_re;
  bool          is_ue;
  bool          llr_is_8bit;
  float         avg_evm;
  srsran_sch_t  dl_sch;
  void*         coworker_ptr;
  void*         gpu; /* added: stream, RE tables, scratch */
} srsran_pdsch_t;

typedef struct {
  uint8_t* payload;
  bool     crc;
  float    avg_iterations_block;
  float    evm;
} srsran_pdsch_res_t;

int  srsran_pdsch_init_ue(srsran_pdsch_t* q, uint32_t max_prb, uint32_t nof_rx_antennas);
/* eNB side (pdsch.c:302-310, 1015-1120): srsran_pdsch_encode writes the PDSCH REs of the ports'
 * host grids (the rest is left as the caller put it: CRS, control channels).  PORT0 (1 port), TX
 * diversity (2 ports, 1 TB), CDD (2 ports, 2 TBs); rho_a scaling (power_scale with p_a != 0) is not
 * provided.  Runs on the GPU: DL-SCH encoding, scrambling, modulation, precoding, RE mapping. */
int  srsran_pdsch_init_enb(srsran_pdsch_t* q, uint32_t max_prb);
int  srsran_pdsch_encode(srsran_pdsch_t*     q,
                         srsran_dl_sf_cfg_t* sf,
                         srsran_pdsch_cfg_t* cfg,
                         uint8_t*            data[SRSRAN_MAX_CODEWORDS],
                         cf_t*               sf_symbols[SRSRAN_MAX_PORTS]);
void srsran_pdsch_free(srsran_pdsch_t* q);
int  srsran_pdsch_enable_coworker(srsran_pdsch_t* q); /* accepted, no effect */
int  srsran_pdsch_set_cell(srsran_pdsch_t* q, srsran_cell_t cell);
/* sf_symbols: nof_rx host grids; channel->ce: the full (14-symbol) host estimates */
int srsran_pdsch_decode(srsran_pdsch_t*        q,
                        srsran_dl_sf_cfg_t*    sf,
                        srsran_pdsch_cfg_t*    cfg,
                        srsran_chest_dl_res_t* channel,
                        cf_t*                  sf_symbols[SRSRAN_MAX_PORTS],
                        srsran_pdsch_res_t     data[SRSRAN_MAX_CODEWORDS]);

/* added: one subframe of a device-resident PDSCH batch */
typedef struct {
  srsran_pdsch_cfg_t* cfg;        /* grant, rnti, softbuffers, csi_enable, power_scale, ... */
  uint32_t            tti;
  uint32_t            cfi;
  const cf_t*         d_grid;     /* nof_rx grids of 14 * 12 * nof_prb */
  const cf_t*         d_ce;       /* [port][rx] estimates */
  uint32_t            ce_full;    /* 1: 14 * 12 * nof_prb per (port, rx); 0: one 12 * nof_prb row */
  const float*        d_noise;    /* device noise estimate (NULL: use `noise`) */
  float               noise;
  uint8_t*            d_payload[SRSRAN_MAX_CODEWORDS]; /* device, >= tbs/8 + 6 bytes */
  uint32_t            new_data[SRSRAN_MAX_CODEWORDS];  /* 1: reset the soft buffer (new transmission) */
} srsran_pdsch_gpu_sf_t;

/* added: decodes every enabled TB of nof_sf subframes in one pass; asynchronous on `stream`.
 * d_result / d_avg_noi receive decode_tb's return / avg iterations per decoded TB, in subframe
 * order then codeword order (enabled TBs only).  Returns the number of TBs enqueued or < 0. */
int srsran_pdsch_gpu_decode_batch(srsran_pdsch_t*              q,
                                  uint32_t                     nof_sf,
                                  const srsran_pdsch_gpu_sf_t* sfs,
                                  int32_t*                     d_result,
                                  float*                       d_avg_noi,
                                  void*                        stream);

/* added (tests / diagnostics): the descrambled, CSI-corrected int16 LLRs (int8 when q->llr_is_8bit; the e bits
 * srsran_dlsch_decode2 receives, pdsch.c:693-733) of subframe `sf` (index into the last srsran_pdsch_gpu_decode_batch /
 * srsran_ue_dl_gpu_decode_batch on q) and transport block `tb`: a device pointer, valid until the next batch on
 * q and complete once that batch's stream has reached it, and their number.  SRSRAN_ERROR if the TB was not in
 * the batch. */
int srsran_pdsch_gpu_last_llr(srsran_pdsch_t* q, uint32_t sf, uint32_t tb, const int16_t** d_llr, uint32_t* nof_llr);
/* added: the RMS EVM (srsran_pdsch_res_t.evm, pdsch.c:698-713) of subframe `sf` / transport block `tb` of the last
 * batch on q, for subframes whose cfg->meas_evm_en was set: a device float (NAN where no symbol was measured),
 * valid until the next batch on q.  SRSRAN_ERROR if it was not measured.  (srsran_pdsch_decode fills data[].evm
 * and q->avg_evm itself.) */
int srsran_pdsch_gpu_last_evm(srsran_pdsch_t* q, uint32_t sf, uint32_t tb, const float** d_evm);

/* ---------------- UE DL (ue/ue_dl.h:77-207, ue_dl.c) ----------------
 * decode_fft_estimate: OFDM, CRS estimation, PCFICH (sets sf->cfi) and the PDCCH LLRs, all on the
 * GPU, for cells of 1, 2 or 4 ports with normal PHICH duration (other cells: the CFI is the caller's
 * sf->cfi).  MBSFN subframes (sf->sf_type, srsran_ue_dl_set_non_mbsfn_region, srsran_ue_dl_set_mbsfn_area_id):
 * fft_mbsfn transforms antenna 0's input buffer into sf_symbols[0] and the other antennas' grids keep the
 * previous subframe, as in the reference (ue_dl.c:104-111, 353-356, 373-376); then the MBSFN estimator and the
 * PCFICH / PDCCH of the non-MBSFN region.  srsran_ue_dl_find_dl_dci / srsran_ue_dl_dci_to_pdsch_grant are in
 * srsran_pdcch.h.  PHICH / PMCH are not provided.  srsran_dl_cfg_t omits the reference's leading cqi_report. */
typedef enum { SRSRAN_TM1 = 0, SRSRAN_TM2, SRSRAN_TM3, SRSRAN_TM4, SRSRAN_TM5, SRSRAN_TM6, SRSRAN_TM7, SRSRAN_TM8,
               SRSRAN_TMINV } srsran_tm_t;

/* phch/dci.h:52-59 (DCI size options) */
typedef struct {
  bool multiple_csi_request_enabled;
  bool cif_enabled;
  bool cif_present;
  bool srs_request_enabled;
  bool ra_format_enabled;
  bool is_not_ue_ss;
} srsran_dci_cfg_t;

typedef struct {
  srsran_pdsch_cfg_t pdsch;
  srsran_dci_cfg_t   dci;
  srsran_tm_t        tm;
  bool               dci_common_ss;
} srsran_dl_cfg_t;

typedef struct {
  srsran_dl_cfg_t       cfg;
  srsran_chest_dl_cfg_t chest_cfg;
  uint32_t              last_ri;
  float                 snr_to_cqi_offset;
} srsran_ue_dl_cfg_t;

typedef struct {
  srsran_cell_t         cell;
  uint32_t              nof_rx_antennas;
  uint16_t              current_mbsfn_area_id;
  srsran_pdsch_t        pdsch;
  srsran_chest_dl_t     chest;
  srsran_chest_dl_res_t chest_res;
  srsran_ofdm_t         fft[SRSRAN_MAX_PORTS];
  srsran_ofdm_t         fft_mbsfn; /* MBSFN subframes: antenna 0's input only, as ue_dl.c:104-111 configures it */
  cf_t*                 sf_symbols[SRSRAN_MAX_PORTS];
  void*                 gpu; /* added: batch pipeline buffers */
} srsran_ue_dl_t;

int  srsran_ue_dl_init(srsran_ue_dl_t* q, cf_t* input[SRSRAN_MAX_PORTS], uint32_t max_prb, uint32_t nof_rx_antennas);
void srsran_ue_dl_free(srsran_ue_dl_t* q);
int  srsran_ue_dl_set_cell(srsran_ue_dl_t* q, srsran_cell_t cell);
int  srsran_ue_dl_decode_fft_estimate(srsran_ue_dl_t* q, srsran_dl_sf_cfg_t* sf, srsran_ue_dl_cfg_t* cfg);
int  srsran_ue_dl_decode_fft_estimate_noguru(srsran_ue_dl_t*     q,
                                             srsran_dl_sf_cfg_t* sf,
                                             srsran_ue_dl_cfg_t* cfg,
                                             cf_t*               input[SRSRAN_MAX_PORTS]);
int  srsran_ue_dl_decode_pdsch(srsran_ue_dl_t*     q,
                               srsran_dl_sf_cfg_t* sf,
                               srsran_pdsch_cfg_t* pdsch_cfg,
                               srsran_pdsch_res_t  data[SRSRAN_MAX_CODEWORDS]);

/* added: one subframe of a UE DL batch (time-domain samples already on the device) */
typedef struct {
  uint32_t            tti;
  uint32_t            cfi;
  srsran_pdsch_cfg_t* pdsch_cfg;
  uint8_t*            d_payload[SRSRAN_MAX_CODEWORDS];
  uint32_t            new_data[SRSRAN_MAX_CODEWORDS];
  srsran_tdd_config_t tdd_config;  /* sf->tdd_config of the reference's calls (TDD cells; the same for every
                                      subframe of a batch); zero = unconfigured (every subframe downlink) */
} srsran_ue_dl_gpu_sf_t;

/* added: OFDM demodulation (with CFO correction by `cfo`, as srsran_cfo_correct(.., cfo)),
 * channel estimation (cfg->chest_cfg: srsUE defaults) and PDSCH decode of nof_sf subframes.
 * d_samples: [sf][rx][sf_len] cf_t on the device.  Results as srsran_pdsch_gpu_decode_batch.
 * Asynchronous on `stream`; returns the number of TBs enqueued or < 0. */
int srsran_ue_dl_gpu_decode_batch(srsran_ue_dl_t*              q,
                                  srsran_ue_dl_cfg_t*          cfg,
                                  uint32_t                     nof_sf,
                                  const srsran_ue_dl_gpu_sf_t* sfs,
                                  const cf_t*                  d_samples,
                                  float                        cfo,
                                  int32_t*                     d_result,
                                  float*                       d_avg_noi,
                                  void*                        stream);
/* added: the same batch from int16 I/Q samples (d_samples: [sf][rx][sf_len][2] int16 on the device, converted as
 * (float)x * scale in the OFDM stage's sample load, srsran_ofdm_rx_gpu_sc16): for callers whose samples come from
 * the radio as sc16 and cross PCIe at half the bytes. */
int srsran_ue_dl_gpu_decode_batch_sc16(srsran_ue_dl_t*              q,
                                       srsran_ue_dl_cfg_t*          cfg,
                                       uint32_t                     nof_sf,
                                       const srsran_ue_dl_gpu_sf_t* sfs,
                                       const int16_t*               d_samples,
                                       float                        scale,
                                       float                        cfo,
                                       int32_t*                     d_result,
                                       float*                       d_avg_noi,
                                       void*                        stream);
/* added: a stream for one PHY worker's batches (srsUE / srsENB decode subframes on several workers at once,
 * srsue/src/main.cc:313-314): a HIP stream on a hardware queue of its own, so that two workers' batches are not
 * queued one behind the other on one of the runtime's shared hardware queues (which streams share a queue depends
 * on every stream created and freed before).  Blocking with respect to the legacy NULL stream.  *stream is a
 * hipStream_t; free it with srsran_gpu_worker_stream_free.  (srsran_pusch_init_enb gives each PUSCH object one.) */
int  srsran_gpu_worker_stream_create(void** stream);
void srsran_gpu_worker_stream_free(void* stream);

/* ---------------- CFO correction (sync/cfo.h:41-63, cfo.c:96-107) ---------------- */
typedef struct {
  float    last_freq;
  float    tol;
  uint32_t nsamples;
  uint32_t max_samples;
  void*    gpu;
} srsran_cfo_t;

int  srsran_cfo_init(srsran_cfo_t* h, uint32_t nsamples);
void srsran_cfo_free(srsran_cfo_t* h);
int  srsran_cfo_resize(srsran_cfo_t* h, uint32_t samples);
void srsran_cfo_set_tol(srsran_cfo_t* h, float tol);
/* output[n] = input[n] * exp(j 2 pi freq n), n = 0..nsamples-1 */
void srsran_cfo_correct(srsran_cfo_t* h, const cf_t* input, cf_t* output, float freq);

#ifdef __cplusplus
}
#endif
#endif
