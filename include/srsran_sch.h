/*
 * include/srsran_sch.h -- DL-SCH receive boundary of the MI355X decoder.
 *
 * Drop-in for the reference's DL-SCH decode surface:
 *   lib/include/srsran/phy/fec/cbsegm.h:32-81          srsran_cbsegm_t, srsran_cbsegm*
 *   lib/include/srsran/phy/fec/crc.h:39-87             srsran_crc_t, srsran_crc_*
 *   lib/include/srsran/phy/fec/turbo/rm_turbo.h:54-87  srsran_rm_turbo_{gentables,free_tables,rx_lut,rx_lut_}
 *   lib/include/srsran/phy/fec/softbuffer.h:41-95      srsran_softbuffer_rx_t, srsran_softbuffer_rx_*
 *   lib/include/srsran/phy/phch/ra.h:43-53             srsran_ra_tb_t
 *   lib/include/srsran/phy/phch/pdsch_cfg.h:37-71      srsran_pdsch_grant_t, srsran_pdsch_cfg_t
 *   lib/include/srsran/phy/phch/sch.h:52-100           srsran_sch_t, srsran_sch_*, srsran_dlsch_decode{,2}
 *
 * Differences a caller must know:
 *   - srsran_softbuffer_rx_t keeps its field layout, but buffer_f[i] and data[i] point into DEVICE
 *     memory (HBM).  cb_crc[] / tb_crc stay host-readable mirrors, refreshed by every synchronous call.
 *   - srsran_sch_t keeps the fields callers touch (max_iterations, avg_iterations, llr_is_8bit,
 *     decoder); the CPU-only scratch buffers are replaced by an opaque `gpu` pointer.
 *   - llr_is_8bit (sch.c:409-428) is provided: e bits are then int8 (passed through the int16_t* parameters,
 *     as the reference casts them), the soft buffer rows hold int8 LLRs in the 8-bit decoder's layout, and the
 *     blocks decode on the 8-bit window decoders (K > 800) or the 16-bit ones on the widened row (K <= 800).
 *   - srsran_dlsch_gpu_decode_batch() is an added, asynchronous entry point over device buffers.
 */
#ifndef SRSRAN_AMD_SCH_H
#define SRSRAN_AMD_SCH_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#include "srsran_tdec.h"

#ifdef __cplusplus
extern "C" {
#endif

#ifndef SRSRAN_ERROR_OUT_OF_BOUNDS
#define SRSRAN_ERROR_OUT_OF_BOUNDS -5
#endif

#define SRSRAN_MAX_PRB 110         /* phy_common.h:106 */
#define SRSRAN_MAX_CODEWORDS 2     /* phy_common.h:60 */
#define SRSRAN_MAX_CODEBLOCKS 32   /* phy_common.h:64 */
#define SRSRAN_LTE_CRC24A 0x1864CFB /* phy_common.h:72 */
#define SRSRAN_LTE_CRC24B 0x1800063 /* phy_common.h:73 */
#define SOFTBUFFER_SIZE 18600      /* softbuffer.h:58 */

/* ---------------- code block segmentation (cbsegm.h:32-81, cbsegm.c:62-140) ---------------- */
typedef struct {
  uint32_t F;
  uint32_t C;
  uint32_t K1;
  uint32_t K2;
  uint32_t K1_idx;
  uint32_t K2_idx;
  uint32_t C1;
  uint32_t C2;
  uint32_t tbs;
  uint32_t L_tb;
  uint32_t L_cb;
  uint32_t Z;
} srsran_cbsegm_t;

int  srsran_cbsegm(srsran_cbsegm_t* s, uint32_t tbs);  /* cbsegm.c:62-117 */
int  srsran_cbsegm_cbsize(uint32_t index);              /* cbsegm.c:133-140 */
bool srsran_cbsegm_cbsize_isvalid(uint32_t size);       /* cbsegm.c:142-151 */
int  srsran_cbsegm_cbindex(uint32_t long_cb);           /* cbsegm.c:119-131 */

/* ---------------- CRC (crc.h:39-87, crc.c:117-195) -- host utility ---------------- */
typedef struct {
  uint64_t table[256];
  int      polynom;
  int      order;
  uint64_t crcinit;
  uint64_t crcmask;
  uint64_t crchighbit;
  uint32_t srsran_crc_out;
} srsran_crc_t;

int      srsran_crc_init(srsran_crc_t* h, uint32_t srsran_crc_poly, int srsran_crc_order); /* crc.c:69-93 */
int      srsran_crc_set_init(srsran_crc_t* h, uint64_t init_value);                        /* crc.c:95-103 */
uint32_t srsran_crc_checksum_byte(srsran_crc_t* h, const uint8_t* data, int len);          /* crc.c:145-163 */
bool     srsran_crc_match_byte(srsran_crc_t* h, uint8_t* data, int len);                   /* crc.c:179-185 */
uint32_t srsran_crc_attach_byte(srsran_crc_t* h, uint8_t* data, int len);                  /* crc.c:165-177 */

/* ---------------- turbo rate de-matching RX (rm_turbo.h:54-87, rm_turbo.c:390-483) ----------------
 * Host pointers, host-synchronous: output[deinter[i % (3K+12)]] += input[i] (int16 wrap), executed by
 * the HIP de-matching kernel.  enable_input_tdec selects the decoder's sub-block (SB) layout for
 * K >= 408 exactly like rm_turbo.c:403-418; the output buffer must then hold 3*(K+32)+12 values. */
void srsran_rm_turbo_gentables(void);
void srsran_rm_turbo_free_tables(void);
int  srsran_rm_turbo_rx_lut(int16_t* input, int16_t* output, uint32_t in_len, uint32_t cb_idx, uint32_t rv_idx);
int  srsran_rm_turbo_rx_lut_(int16_t* input,
                             int16_t* output,
                             uint32_t in_len,
                             uint32_t cb_idx,
                             uint32_t rv_idx,
                             bool     enable_input_tdec);
int  srsran_rm_turbo_rx_lut_8bit(int8_t* input, int8_t* output, uint32_t in_len, uint32_t cb_idx, uint32_t rv_idx);

/* ---------------- turbo encoder and rate matching TX (turbocoder.h:45-59, rm_turbo.h:58-65) ----------------
 * Host pointers, host-synchronous, executed by HIP kernels (enc_kernel.hip: the DL-SCH encoder's PCCC and a
 * rate-matching read-out over the reference's interleaver tables).
 * srsran_tcod_encode: long_cb unpacked input bits (SRSRAN_TX_NULL marks a filler bit) -> 3 long_cb + 12 unpacked
 *   bits, x_k z_k z'_k then the tails, as turbocoder.c:77-185.
 * srsran_rm_turbo_tx_lut: the packed systematic (K + 4 bits, the tails in the byte after K) and parity (2 (K + 4)
 *   bits) streams of srsran_tcod_encode_lut; for rv_idx 0 the circular buffer is built into w_buff (3 K + 12 bits,
 *   packed), otherwise read from it; out_len bits from k0 of rv_idx into output (packed) at bit w_offset
 *   (rm_turbo.c:345-388). */
#ifndef SRSRAN_TX_NULL
#define SRSRAN_TX_NULL 100
#endif
typedef struct {
  uint32_t max_long_cb;
  uint8_t* temp;
  void*    gpu; /* added: device buffers */
} srsran_tcod_t;
int  srsran_tcod_init(srsran_tcod_t* h, uint32_t max_long_cb);                            /* turbocoder.c:44-62 */
void srsran_tcod_free(srsran_tcod_t* h);                                                   /* turbocoder.c:64-75 */
int  srsran_tcod_encode(srsran_tcod_t* h, uint8_t* input, uint8_t* output, uint32_t long_cb); /* turbocoder.c:77-185 */
int  srsran_rm_turbo_tx_lut(uint8_t* w_buff, uint8_t* systematic, uint8_t* parity, uint8_t* output, uint32_t cb_idx,
                            uint32_t out_len, uint32_t w_offset, uint32_t rv_idx);      /* rm_turbo.c:345-388 */

/* ---------------- HARQ soft buffer (softbuffer.h:41-95, softbuffer.c:36-178) ---------------- */
typedef struct {
  uint32_t  max_cb;
  uint32_t  max_cb_size;
  int16_t** buffer_f; /* DEVICE pointers, one per code block (max_cb_size int16 each) */
  uint8_t** data;     /* DEVICE pointers, saved CB payload (max_cb_size/8 bytes each) */
  bool*     cb_crc;   /* host mirror */
  bool      tb_crc;   /* host mirror */
  void*     gpu;      /* added: device arena + device flags */
} srsran_softbuffer_rx_t;

int  srsran_softbuffer_rx_init(srsran_softbuffer_rx_t* q, uint32_t nof_prb);
int  srsran_softbuffer_rx_init_guru(srsran_softbuffer_rx_t* q, uint32_t max_cb, uint32_t max_cb_size);
void srsran_softbuffer_rx_reset(srsran_softbuffer_rx_t* p);
void srsran_softbuffer_rx_reset_tbs(srsran_softbuffer_rx_t* q, uint32_t tbs);
void srsran_softbuffer_rx_reset_cb(srsran_softbuffer_rx_t* q, uint32_t nof_cb);
void srsran_softbuffer_rx_reset_cb_crc(srsran_softbuffer_rx_t* q, uint32_t nof_cb);
void srsran_softbuffer_rx_free(srsran_softbuffer_rx_t* p);
/* added: copy the device cb_crc / tb_crc flags into the host mirror (after asynchronous batches) */
int srsran_softbuffer_rx_sync(srsran_softbuffer_rx_t* q);
/* added: soft-buffer device arena of the soft buffers initialised from now on: enable = 0 gives
   every soft buffer its own hipMalloc; bytes (> 0) = capacity of per-device arenas not created yet
   (default 1 GiB).  Decoding results and decoder choice do not depend on it. */
int srsran_softbuffer_rx_gpu_arena(int enable, size_t bytes);
/* added: device address of the soft buffer's first code block (diagnostics) */
const void* srsran_softbuffer_rx_gpu_ptr(const srsran_softbuffer_rx_t* q);

/* ---------------- grant / PDSCH configuration (ra.h:43-53, pdsch_cfg.h:37-71) ---------------- */
typedef enum {
  SRSRAN_MOD_BPSK = 0,
  SRSRAN_MOD_QPSK,
  SRSRAN_MOD_16QAM,
  SRSRAN_MOD_64QAM,
  SRSRAN_MOD_256QAM,
  SRSRAN_MOD_NITEMS
} srsran_mod_t; /* phy_common.h:285-292 */

typedef enum {
  SRSRAN_TXSCHEME_PORT0,
  SRSRAN_TXSCHEME_DIVERSITY,
  SRSRAN_TXSCHEME_SPATIALMUX,
  SRSRAN_TXSCHEME_CDD
} srsran_tx_scheme_t; /* phy_common.h:273-278 */

typedef enum { SRSRAN_MIMO_DECODER_ZF, SRSRAN_MIMO_DECODER_MMSE } srsran_mimo_decoder_t; /* phy_common.h:280 */

uint32_t srsran_mod_bits_x_symbol(srsran_mod_t mod); /* phy_common.c */

typedef struct {
  srsran_mod_t mod;
  int          tbs;
  int          rv;
  uint32_t     nof_bits;
  uint32_t     cw_idx;
  bool         enabled;
  uint32_t     mcs_idx;
} srsran_ra_tb_t;

typedef struct {
  srsran_tx_scheme_t tx_scheme;
  uint32_t           pmi;
  bool               prb_idx[2][SRSRAN_MAX_PRB];
  uint32_t           nof_prb;
  uint32_t           nof_re;
  uint32_t           nof_symb_slot[2];
  srsran_ra_tb_t     tb[SRSRAN_MAX_CODEWORDS];
  int                last_tbs[SRSRAN_MAX_CODEWORDS];
  uint32_t           nof_tb;
  uint32_t           nof_layers;
} srsran_pdsch_grant_t;

typedef struct {
  srsran_pdsch_grant_t grant;

  uint16_t              rnti;
  uint32_t              max_nof_iterations;
  srsran_mimo_decoder_t decoder_type;
  float                 p_a;
  uint32_t              p_b;
  float                 rs_power;
  bool                  power_scale;
  bool                  csi_enable;
  bool                  use_tbs_index_alt;

  union {
    void*                   tx[SRSRAN_MAX_CODEWORDS];
    srsran_softbuffer_rx_t* rx[SRSRAN_MAX_CODEWORDS];
  } softbuffers;

  bool     meas_evm_en;
  bool     meas_time_en;
  uint32_t meas_time_value;
} srsran_pdsch_cfg_t;

/* ---------------- shared channel decoder (sch.h:52-100, sch.c:140-609) ---------------- */
typedef struct {
  uint32_t      max_iterations; /* half-iterations, default 10 (sch.c:36,165) */
  float         avg_iterations;
  bool          llr_is_8bit;
  srsran_tdec_t decoder;
  void*         gpu; /* added: stream, staging and scratch of the DL-SCH GPU path */
} srsran_sch_t;

int   srsran_sch_init(srsran_sch_t* q);
void  srsran_sch_free(srsran_sch_t* q);
void  srsran_sch_set_max_noi(srsran_sch_t* q, uint32_t max_iterations);
float srsran_sch_last_noi(srsran_sch_t* q);

/* e_bits: host int16 LLRs (grant.tb[tb_idx].nof_bits); data: host payload buffer, receives every byte
 * the reference's decode_tb writes (tbs/8 + 3 bytes for one CB, up to tbs/8 + 6 for several). */
int srsran_dlsch_decode(srsran_sch_t* q, srsran_pdsch_cfg_t* cfg, int16_t* e_bits, uint8_t* data);
int srsran_dlsch_decode2(srsran_sch_t*       q,
                         srsran_pdsch_cfg_t* cfg,
                         int16_t*            e_bits,
                         uint8_t*            data,
                         int                 tb_idx,
                         uint32_t            nof_layers);

/* added: srsran_dlsch_decode2 whose LLRs are already in device memory (written before the call
 * returns control to the host, e.g. by a synchronised stream). */
int srsran_dlsch_decode2_dev(srsran_sch_t*       q,
                             srsran_pdsch_cfg_t* cfg,
                             const int16_t*      d_e_bits,
                             uint8_t*            data,
                             int                 tb_idx,
                             uint32_t            nof_layers);

/* ---------------- added: batched, asynchronous DL-SCH decode over device buffers ----------------
 * One entry per transport block; every entry is decoded with exactly the semantics of
 * decode_tb (sch.c:509-573) against its own soft buffer.  Results land in device memory:
 *   d_result[i]  = SRSRAN_SUCCESS / SRSRAN_ERROR / SRSRAN_ERROR_INVALID_INPUTS (decode_tb's return)
 *   d_avg_noi[i] = avg_iterations of that TB (sch.c:489)
 * Soft buffer flags are updated on the device; call srsran_softbuffer_rx_sync() to read them on
 * the host.  `stream` is a hipStream_t (NULL = the default stream).  q->max_iterations
 * applies to every TB.  Returns SRSRAN_SUCCESS once the work is enqueued. */
typedef struct {
  uint32_t                tbs;
  uint32_t                Qm; /* bits per symbol x layers, as decode_tb receives it */
  uint32_t                rv;
  uint32_t                nof_e_bits;
  const int16_t*          d_e_bits; /* device; int8_t LLRs when the srsran_sch_t has llr_is_8bit */
  uint8_t*                d_data;   /* device, >= tbs/8 + 6 bytes */
  srsran_softbuffer_rx_t* softbuffer;
  uint32_t                new_data; /* 1: as if srsran_softbuffer_rx_reset_tbs(softbuffer, tbs) ran first */
} srsran_dlsch_gpu_tb_t;

int srsran_dlsch_gpu_decode_batch(srsran_sch_t*                q,
                                  uint32_t                     nof_tb,
                                  const srsran_dlsch_gpu_tb_t* tbs,
                                  int32_t*                     d_result,
                                  float*                       d_avg_noi,
                                  void*                        stream);

/* ---- DL-SCH transmit (sch.c:240-359, 621-652; turbocoder.c; rm_turbo.c:345-388) ----
 * TB CRC24A, code block segmentation with CRC24B, turbo encoding and rate matching, all on the GPU.
 * e_bits: packed, MSB first, cfg->grant.tb[tb_idx].nof_bits bits (ceil(nof_bits / 8) bytes written).
 * data must be given: the reference's retransmission from the soft buffer (data == NULL) is not
 * provided; the soft buffer argument is not used (every call encodes from the payload).  Filler
 * bits are refused as in the reference. */
int srsran_dlsch_encode(srsran_sch_t* q, srsran_pdsch_cfg_t* cfg, uint8_t* data, uint8_t* e_bits);
int srsran_dlsch_encode2(srsran_sch_t*       q,
                         srsran_pdsch_cfg_t* cfg,
                         uint8_t*            data,
                         uint8_t*            e_bits,
                         int                 tb_idx,
                         uint32_t            nof_layers);

/* Added batch entry point: many TBs in three launches, asynchronous on `stream`. */
typedef struct {
  uint32_t       tbs;
  uint32_t       Qm; /* bits per symbol x layers, as encode_tb receives it */
  uint32_t       rv;
  uint32_t       nof_e_bits;
  const uint8_t* d_data;   /* device, tbs / 8 bytes */
  uint8_t*       d_e_bits; /* device, ceil(nof_e_bits / 8) bytes, packed MSB first */
} srsran_dlsch_gpu_enc_t;

int srsran_dlsch_gpu_encode_batch(srsran_sch_t* q, uint32_t nof_tb, const srsran_dlsch_gpu_enc_t* tbs, void* stream);

/* ---- UL-SCH receive with UCI multiplexed (sch.c:994-1193, uci.c, cqi.c) ----
 * Mirrors of pusch_cfg.h:29-87, uci_cfg.h:31-59 and cqi.h:74-143 keep the reference's field names
 * and layout so callers compile unchanged. */
#define SRSRAN_MAX_CARRIERS 5      /* phy_common.h:56 */
#ifndef SRSRAN_NRE
#define SRSRAN_NRE 12
#endif
#define SRSRAN_CQI_MAX_BITS 64     /* cqi.h:38 */
#define SRSRAN_UCI_MAX_ACK_BITS 10 /* uci_cfg.h:27 */
#define SRSRAN_UCI_MAX_M 9         /* uci_cfg.h:29 */

typedef struct {
  bool     pending_tb[SRSRAN_MAX_CODEWORDS];
  uint32_t nof_acks;
  uint32_t ncce[SRSRAN_UCI_MAX_M];
  uint32_t N_bundle;
  uint32_t tdd_ack_M;
  uint32_t tdd_ack_m;
  bool     tdd_is_multiplex;
  uint32_t tpc_for_pucch;
  uint32_t grant_cc_idx;
} srsran_uci_cfg_ack_t;

typedef enum {
  SRSRAN_CQI_TYPE_WIDEBAND = 0,
  SRSRAN_CQI_TYPE_SUBBAND_UE,
  SRSRAN_CQI_TYPE_SUBBAND_UE_DIFF,
  SRSRAN_CQI_TYPE_SUBBAND_HL
} srsran_cqi_type_t;

typedef struct {
  bool              data_enable;
  bool              pmi_present;
  bool              four_antenna_ports;
  bool              rank_is_not_one;
  bool              subband_label_2_bits;
  uint32_t          scell_index;
  uint32_t          L;
  uint32_t          N;
  uint32_t          sb_idx;
  srsran_cqi_type_t type;
  uint32_t          ri_len;
} srsran_cqi_cfg_t;

typedef struct {
  srsran_uci_cfg_ack_t ack[SRSRAN_MAX_CARRIERS];
  srsran_cqi_cfg_t     cqi;
  bool                 is_scheduling_request_tti;
} srsran_uci_cfg_t;

typedef struct {
  uint8_t  wideband_cqi_cw0;
  uint32_t subband_diff_cqi_cw0;
  uint8_t  wideband_cqi_cw1;
  uint32_t subband_diff_cqi_cw1;
  uint32_t pmi;
} srsran_cqi_hl_subband_t;
typedef struct {
  uint8_t  wideband_cqi;
  uint8_t  subband_diff_cqi;
  uint32_t position_subband;
} srsran_cqi_ue_diff_subband_t;
typedef struct {
  uint8_t wideband_cqi;
  uint8_t spatial_diff_cqi;
  uint8_t pmi;
} srsran_cqi_format2_wideband_t;
typedef struct {
  uint8_t subband_cqi;
  uint8_t subband_label;
} srsran_cqi_ue_subband_t;
typedef struct {
  union {
    srsran_cqi_format2_wideband_t wideband;
    srsran_cqi_ue_subband_t       subband_ue;
    srsran_cqi_ue_diff_subband_t  subband_ue_diff;
    srsran_cqi_hl_subband_t       subband_hl;
  };
  bool data_crc;
} srsran_cqi_value_t;

typedef struct {
  uint8_t ack_value[SRSRAN_UCI_MAX_ACK_BITS];
  bool    valid;
} srsran_uci_value_ack_t;

typedef struct {
  bool                   scheduling_request;
  srsran_cqi_value_t     cqi;
  srsran_uci_value_ack_t ack;
  uint8_t                ri;
} srsran_uci_value_t;

typedef struct {
  uint32_t I_offset_cqi;
  uint32_t I_offset_ri;
  uint32_t I_offset_ack;
} srsran_uci_offset_cfg_t;

typedef struct {
  uint32_t       L_prb;
  uint32_t       n_prb[2];
  uint32_t       n_prb_tilde[2];
  uint32_t       freq_hopping;
  uint32_t       nof_re;
  uint32_t       nof_symb;
  srsran_ra_tb_t tb;
  srsran_ra_tb_t last_tb;
  uint32_t       n_dmrs;
  bool           is_rar;
} srsran_pusch_grant_t;

typedef struct {
  uint16_t                rnti;
  srsran_uci_cfg_t        uci_cfg;
  srsran_uci_offset_cfg_t uci_offset;
  srsran_pusch_grant_t    grant;
  uint32_t                max_nof_iterations;
  uint32_t                last_O_cqi;
  uint32_t                K_segm;
  uint32_t                current_tx_nb;
  bool                    csi_enable;
  bool                    enable_64qam;
  union {
    void*                   tx;
    srsran_softbuffer_rx_t* rx;
  } softbuffers;
  bool     meas_time_en;
  uint32_t meas_time_value;
  bool     meas_epre_en;
  bool     meas_ta_en;
  bool     use_cedron_alg;
  bool     meas_evm_en;
} srsran_pusch_cfg_t;

/* sch.c:1122: decode the HARQ-ACK and RI bits (zeroing the ACK positions of q_bits), de-interleave
 * q_bits (nof_bits LLRs in PUSCH order, RI cells skipped) into g_bits, decode the CQI at its front
 * and decode_tb the rest.  c_seq: the unpacked PUSCH scrambling sequence (needed for 1-bit ACK / RI).
 * Returns decode_tb's value (SRSRAN_SUCCESS when the TB CRC matched) or, without a TB, Q'_CQI
 * (Q'_RI without CQI) as the reference does; sets cfg->K_segm and, for subband-HL CQI with RI,
 * cfg->uci_cfg.cqi.rank_is_not_one.  All LLR work runs on the GPU (uci_kernel.hip, sch_kernel.hip). */
int srsran_ulsch_decode(srsran_sch_t*       q,
                        srsran_pusch_cfg_t* cfg,
                        int16_t*            q_bits,
                        int16_t*            g_bits,
                        uint8_t*            c_seq,
                        uint8_t*            data,
                        srsran_uci_value_t* uci_data);

/* UCI helpers (sch.h:117-125, uci.h:129-144, cqi.h:145-151) */
float    srsran_sch_beta_cqi(uint32_t I_cqi);
float    srsran_sch_beta_ack(uint32_t I_harq);
uint32_t srsran_sch_find_Ioffset_ack(float beta);
uint32_t srsran_sch_find_Ioffset_cqi(float beta);
uint32_t srsran_sch_find_Ioffset_ri(float beta);
uint32_t srsran_qprime_cqi_ext(uint32_t L_prb, uint32_t nof_symbols, uint32_t tbs, float beta);
uint32_t srsran_qprime_ack_ext(uint32_t L_prb, uint32_t nof_symbols, uint32_t tbs, uint32_t nof_ack, float beta);
uint32_t srsran_uci_cfg_total_ack(const srsran_uci_cfg_t* uci_cfg);
int      srsran_cqi_size(srsran_cqi_cfg_t* cfg);
int      srsran_cqi_value_pack(srsran_cqi_cfg_t* cfg, srsran_cqi_value_t* value, uint8_t buff[SRSRAN_CQI_MAX_BITS]);
int      srsran_cqi_value_unpack(srsran_cqi_cfg_t* cfg, uint8_t buff[SRSRAN_CQI_MAX_BITS], srsran_cqi_value_t* value);

/* Added batch entry point: per TB the de-interleaver (device scratch d_g_bits) and decode_tb, all
 * asynchronous on `stream`; d_result / d_avg_noi as srsran_dlsch_gpu_decode_batch. */
typedef struct {
  uint32_t                tbs;
  uint32_t                Qm;
  uint32_t                rv;
  uint32_t                nof_e_bits; /* H'_total Qm */
  uint32_t                nof_symb;   /* N_symb^PUSCH */
  const int16_t*          d_q_bits;   /* device, PUSCH order */
  int16_t*                d_g_bits;   /* device scratch, nof_e_bits */
  uint8_t*                d_data;     /* device, >= tbs/8 + 6 bytes */
  srsran_softbuffer_rx_t* softbuffer;
  uint32_t                new_data;
} srsran_ulsch_gpu_tb_t;

int srsran_ulsch_gpu_decode_batch(srsran_sch_t*                q,
                                  uint32_t                     nof_tb,
                                  const srsran_ulsch_gpu_tb_t* tbs,
                                  int32_t*                     d_result,
                                  float*                       d_avg_noi,
                                  void*                        stream);

#ifdef __cplusplus
}
#endif
#endif
