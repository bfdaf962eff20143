/*
 * include/srsran_sch_nr.h -- NR shared-channel (DL-SCH / UL-SCH) receive boundary of the MI355X decoder.
 *
 * Drop-in for the reference's NR SCH decode surface (paths relative to /root/reference/lib):
 *   include/srsran/phy/common/phy_common_nr.h:264-318, 384-395  srsran_mcs_table_t, srsran_xoverhead_t,
 *                                                               srsran_carrier_nr_t
 *   include/srsran/phy/phch/sch_cfg_nr.h:27-57                  srsran_sch_cfg_t, srsran_sch_tb_t
 *   include/srsran/phy/phch/sch_nr.h:33-164                     srsran_sch_tb_res_nr_t, srsran_sch_nr_args_t,
 *                                                               srsran_sch_nr_tb_info_t, srsran_sch_nr_*,
 *                                                               srsran_{dl,ul}sch_nr_decode
 *   include/srsran/phy/fec/cbsegm.h:75-79                       srsran_cbsegm_ldpc_bg1 / _bg2
 * Semantics of sch_nr.c:114-189, 283-360, 554-750 (incl. its quirks: a code block whose CRC already
 * passed keeps the LLR read pointer where it is), LDPC rate de-matching of ldpc_rm.c and the
 * decoders of srsran_ldpc.h; results are bit-identical to the reference.
 *
 * Differences a caller must know:
 *   - srsran_sch_nr_t keeps `carrier`; the reference's per-lifting-size encoder / decoder tables and
 *     CPU buffers are replaced by an opaque `gpu` pointer.  Only the receive side is provided
 *     (srsran_sch_nr_init_tx / encode: not provided).
 *   - soft buffers are the device-resident srsran_softbuffer_rx_t of srsran_sch.h (init_guru with
 *     max_cb_size >= 25344); cb_crc[] is a host mirror refreshed by every synchronous call.
 *   - TBs needing more than SRSRAN_SCH_NR_MAX_NOF_CB_LDPC code blocks are rejected (the reference
 *     writes past its mask[] array, sch_nr.c:166-168).
 *   - srsran_sch_nr_gpu_decode_batch() is an added, asynchronous entry point over device buffers.
 */
#ifndef SRSRAN_AMD_SCH_NR_H
#define SRSRAN_AMD_SCH_NR_H

#include <stdbool.h>
#include <stdint.h>

#include "srsran_ldpc.h"
#include "srsran_sch.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SRSRAN_MAX_NRE_NR 156                                                           /* phy_common_nr.h:117 */
#define SRSRAN_MAX_PRB_NR 275                                                           /* phy_common_nr.h:84 */
#define SRSRAN_SLOT_MAX_NOF_BITS_NR (SRSRAN_MAX_NRE_NR * SRSRAN_MAX_PRB_NR * 8)         /* phy_common_nr.h:128 */
#define SRSRAN_LDPC_MAX_LEN_ENCODED_CB (MAX_LIFTSIZE * 66)                              /* base_graph.h:64 */
#define SRSRAN_SCH_NR_MAX_NOF_CB_LDPC                                                                                  \
  ((SRSRAN_SLOT_MAX_NOF_BITS_NR + (SRSRAN_LDPC_MAX_LEN_CB - 1)) / SRSRAN_LDPC_MAX_LEN_CB) /* sch_nr.h:28 */

typedef enum {
  srsran_subcarrier_spacing_15kHz = 0,
  srsran_subcarrier_spacing_30kHz,
  srsran_subcarrier_spacing_60kHz,
  srsran_subcarrier_spacing_120kHz,
  srsran_subcarrier_spacing_240kHz,
  srsran_subcarrier_spacing_invalid
} srsran_subcarrier_spacing_t;

typedef enum {
  srsran_mcs_table_64qam = 0,
  srsran_mcs_table_256qam,
  srsran_mcs_table_qam64LowSE,
  srsran_mcs_table_N
} srsran_mcs_table_t;

typedef enum { srsran_xoverhead_0 = 0, srsran_xoverhead_6, srsran_xoverhead_12, srsran_xoverhead_18 } srsran_xoverhead_t;

typedef struct {
  uint32_t                    pci;
  double                      dl_center_frequency_hz;
  double                      ul_center_frequency_hz;
  double                      ssb_center_freq_hz;
  uint32_t                    offset_to_carrier;
  srsran_subcarrier_spacing_t scs;
  uint32_t                    nof_prb;
  uint32_t                    start;
  uint32_t                    max_mimo_layers;
} srsran_carrier_nr_t;

typedef struct {
  srsran_mcs_table_t mcs_table;
  srsran_xoverhead_t xoverhead;
  bool               limited_buffer_rm;
} srsran_sch_cfg_t;

typedef struct {
  srsran_mod_t mod;
  uint32_t     N_L;
  uint32_t     mcs;
  int          tbs;
  double       R;
  double       R_prime;
  int          rv;
  int          ndi;
  uint32_t     nof_re;
  uint32_t     nof_bits;
  uint32_t     cw_idx;
  bool         enabled;
  union {
    void*                   tx;
    srsran_softbuffer_rx_t* rx;
  } softbuffer;
} srsran_sch_tb_t;

typedef struct {
  uint8_t* payload;
  bool     crc;
  float    avg_iter;
} srsran_sch_tb_res_nr_t;

typedef struct {
  bool     disable_simd;           /* true: SRSRAN_LDPC_DECODER_C arithmetic, else the AVX2/AVX512 one */
  bool     decoder_use_flooded;    /* flooded schedule: not provided (init fails) */
  float    decoder_scaling_factor; /* not normal -> 0.8 (sch_nr.c:307) */
  uint32_t max_nof_iter;           /* 0 -> 10 */
} srsran_sch_nr_args_t;

typedef struct {
  srsran_basegraph_t bg;
  uint32_t           Qm;
  uint32_t           G;
  uint32_t           A;
  uint32_t           L_tb;
  uint32_t           L_cb;
  uint32_t           B;
  uint32_t           Bp;
  uint32_t           Kp;
  uint32_t           Kr;
  uint32_t           F;
  uint32_t           Nref;
  uint32_t           Z;
  uint32_t           Nl;
  bool               mask[SRSRAN_SCH_NR_MAX_NOF_CB_LDPC];
  uint32_t           C;
  uint32_t           Cp;
} srsran_sch_nr_tb_info_t;

typedef struct {
  srsran_carrier_nr_t carrier;
  void*               gpu; /* opaque: HIP stream, LDPC decoders per (BG, Z), device staging */
} srsran_sch_nr_t;

int                srsran_cbsegm_ldpc_bg1(srsran_cbsegm_t* s, uint32_t tbs); /* cbsegm.c:269 */
int                srsran_cbsegm_ldpc_bg2(srsran_cbsegm_t* s, uint32_t tbs); /* cbsegm.c:274 */
srsran_basegraph_t srsran_sch_nr_select_basegraph(uint32_t tbs, double R);   /* sch_nr.c:33 */
int                srsran_sch_nr_fill_tb_info(const srsran_carrier_nr_t* carrier,
                                              const srsran_sch_cfg_t*    sch_cfg,
                                              const srsran_sch_tb_t*     tb,
                                              srsran_sch_nr_tb_info_t*   cfg); /* sch_nr.c:114 */
int                srsran_sch_nr_init_rx(srsran_sch_nr_t* q, const srsran_sch_nr_args_t* args);         /* :283 */
int                srsran_sch_nr_set_carrier(srsran_sch_nr_t* q, const srsran_carrier_nr_t* carrier); /* :362 */
void               srsran_sch_nr_free(srsran_sch_nr_t* q);                                            /* :373 */
int                srsran_dlsch_nr_decode(srsran_sch_nr_t*        q,
                                          const srsran_sch_cfg_t* sch_cfg,
                                          const srsran_sch_tb_t*  tb,
                                          int8_t*                 e_bits,
                                          srsran_sch_tb_res_nr_t* res); /* sch_nr.c:761 */
int                srsran_ulsch_nr_decode(srsran_sch_nr_t*        q,
                                          const srsran_sch_cfg_t* sch_cfg,
                                          const srsran_sch_tb_t*  tb,
                                          int8_t*                 e_bits,
                                          srsran_sch_tb_res_nr_t* res); /* sch_nr.c:779 */

/*
 * Added batch entry point: every TB's rate de-matching, LDPC decoding (one launch per (BG, Z)) and TB
 * assembly, asynchronous on `stream` (a hipStream_t).  Per TB: the configuration as for
 * srsran_dlsch_nr_decode, d_e_bits (tb.nof_bits int8 LLRs, device), d_payload (tbs / 8 bytes,
 * device, written only when every code block passed), new_data (1: the TB's code blocks start from an
 * empty soft buffer -- CRC flags, soft bits and saved payloads cleared as srsran_softbuffer_rx_reset_cb
 * would, done inside the rate de-matching launch).  Per TB outputs (device): d_crc[i] (1 = TB CRC ok),
 * d_avg_iter[i].  Soft-buffer flags stay on the device (srsran_softbuffer_rx_sync()).
 */
typedef struct {
  const srsran_sch_cfg_t* sch_cfg;
  const srsran_sch_tb_t*  tb;
  const int8_t*           d_e_bits;
  uint8_t*                d_payload;
  uint32_t                new_data;
} srsran_sch_nr_gpu_tb_t;

int srsran_sch_nr_gpu_decode_batch(srsran_sch_nr_t*              q,
                                   uint32_t                      nof_tb,
                                   const srsran_sch_nr_gpu_tb_t* tbs,
                                   uint8_t*                      d_crc,
                                   float*                        d_avg_iter,
                                   void*                         stream);

#ifdef __cplusplus
}
#endif
#endif
