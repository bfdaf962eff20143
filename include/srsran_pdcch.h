/*
 * include/srsran_pdcch.h -- downlink control channels of the MI355X PHY: REG mapping, PCFICH,
 * PDCCH (blind decoding on the GPU), DCI sizes / unpacking and the DL resource allocation that turns
 * a DCI into a PDSCH grant.
 *
 * Drop-in for (types keep the reference's field order):
 *   lib/include/srsran/phy/phch/regs.h:42-99      srsran_regs_t (REG tables held as RE index lists)
 *   lib/include/srsran/phy/phch/pcfich.h:41-86    srsran_pcfich_t, srsran_pcfich_*
 *   lib/include/srsran/phy/phch/pdcch.h:49-142    srsran_pdcch_t, srsran_pdcch_*
 *   lib/include/srsran/phy/phch/dci.h:36-200      srsran_dci_*_t, srsran_dci_format_sizeof, srsran_dci_msg_unpack_pdsch
 *   lib/include/srsran/phy/phch/ra.h:43-106, ra_dl.h:37-60   srsran_ra_*, srsran_ra_dl_dci_to_grant
 *
 * GPU work (pdcch_kernel.hip): PCFICH and PDCCH RE extraction + TX-diversity / MMSE predecoding
 * (the PDSCH predecoder, eq_kernel.hip), float QPSK demodulation and descrambling, CFI correlation,
 * and one wave per PDCCH candidate for rate de-matching, quantisation, the 16-bit tail-biting
 * Viterbi decoder (64 lanes = 64 trellis states), CRC16 / RNTI and the re-encoding correlation.
 * Bit-exact with the reference's AVX2 build for the LLRs, decoded payloads and CRC remainders.
 * Provided: FDD, normal CP, 1, 2 or 4 ports, PHICH normal duration; DCI formats 0, 1, 1A, 1C
 * (size), 2, 2A; resource allocation types 0, 1 and 2 (localized).  Others return SRSRAN_ERROR.
 */
#ifndef SRSRAN_AMD_PDCCH_H
#define SRSRAN_AMD_PDCCH_H

#include <stdbool.h>
#include <stdint.h>

#include "srsran_ue_dl.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- ra.h ---------------- */
#define SRSRAN_RA_NOF_TBS_IDX 34
typedef enum { SRSRAN_RA_ALLOC_TYPE0 = 0, SRSRAN_RA_ALLOC_TYPE1 = 1, SRSRAN_RA_ALLOC_TYPE2 = 2 } srsran_ra_type_t;
typedef struct {
  uint32_t rbg_bitmask;
} srsran_ra_type0_t;
typedef struct {
  uint32_t vrb_bitmask;
  uint32_t rbg_subset;
  bool     shift;
} srsran_ra_type1_t;
typedef struct {
  uint32_t riv;
  enum { SRSRAN_RA_TYPE2_NPRB1A_2 = 0, SRSRAN_RA_TYPE2_NPRB1A_3 = 1 } n_prb1a;
  enum { SRSRAN_RA_TYPE2_NG1 = 0, SRSRAN_RA_TYPE2_NG2 = 1 } n_gap;
  enum { SRSRAN_RA_TYPE2_LOC = 0, SRSRAN_RA_TYPE2_DIST = 1 } mode;
} srsran_ra_type2_t;

uint32_t     srsran_ra_type0_P(uint32_t nof_prb);                                          /* ra.c:60-72 */
uint32_t     srsran_ra_type1_N_rb(uint32_t nof_prb);                                       /* ra.c:74-79 */
void         srsran_ra_type2_from_riv(uint32_t riv, uint32_t* L_crb, uint32_t* RB_start, uint32_t nof_prb,
                                      uint32_t nof_vrb);                                   /* ra.c:49-58 */
uint32_t     srsran_ra_type2_to_riv(uint32_t L_crb, uint32_t RB_start, uint32_t nof_prb); /* ra.c:37-47 */
int          srsran_ra_tbs_idx_from_mcs(uint32_t mcs, bool use_tbs_index_alt, bool is_ul); /* ra.c:146-149 */
srsran_mod_t srsran_ra_dl_mod_from_mcs(uint32_t mcs, bool use_tbs_index_alt);              /* ra.c:151-174 */
int          srsran_ra_tbs_from_idx(uint32_t tbs_idx, uint32_t n_prb);                     /* ra.c:225-232 */

/* ---------------- dci.h / phy_common.h ---------------- */
#define SRSRAN_DCI_MAX_BITS 128
#define SRSRAN_MAX_DCI_MSG 5
#define SRSRAN_MAX_CANDIDATES_UE 16
#define SRSRAN_MAX_CANDIDATES_COM 6
#define SRSRAN_MAX_CANDIDATES (SRSRAN_MAX_CANDIDATES_UE + SRSRAN_MAX_CANDIDATES_COM)
#define SRSRAN_SIRNTI 0xFFFF
#define SRSRAN_PRNTI 0xFFFE
#define SRSRAN_MRNTI 0xFFFD
#define SRSRAN_CRNTI_START 0x000B
#define SRSRAN_CRNTI_END 0xFFF3
#define SRSRAN_RARNTI_START 0x0001
#define SRSRAN_RARNTI_END 0x000A
#define SRSRAN_RNTI_ISRAR(rnti) (rnti >= SRSRAN_RARNTI_START && rnti <= SRSRAN_RARNTI_END)
#define SRSRAN_RNTI_ISUSER(rnti) (rnti >= SRSRAN_CRNTI_START && rnti <= SRSRAN_CRNTI_END)
#define SRSRAN_DCI_IS_TB_EN(tb) (!(tb.mcs_idx == 0 && tb.rv == 1))

typedef enum {
  SRSRAN_DCI_FORMAT0 = 0,
  SRSRAN_DCI_FORMAT1,
  SRSRAN_DCI_FORMAT1A,
  SRSRAN_DCI_FORMAT1B,
  SRSRAN_DCI_FORMAT1C,
  SRSRAN_DCI_FORMAT1D,
  SRSRAN_DCI_FORMAT2,
  SRSRAN_DCI_FORMAT2A,
  SRSRAN_DCI_FORMAT2B,
  SRSRAN_DCI_FORMATN0,
  SRSRAN_DCI_FORMATN1,
  SRSRAN_DCI_FORMATN2,
  SRSRAN_DCI_FORMAT_RAR,
  SRSRAN_DCI_NOF_FORMATS
} srsran_dci_format_t;

/* srsran_dci_cfg_t: srsran_ue_dl.h */

typedef struct {
  uint32_t L;    /* aggregation level (log2) */
  uint32_t ncce; /* first CCE */
} srsran_dci_location_t;

typedef struct {
  uint8_t               payload[SRSRAN_DCI_MAX_BITS];
  uint32_t              nof_bits;
  srsran_dci_location_t location;
  srsran_dci_format_t   format;
  uint16_t              rnti;
} srsran_dci_msg_t;

typedef struct {
  uint32_t mcs_idx;
  int      rv;
  bool     ndi;
  uint32_t cw_idx;
} srsran_dci_tb_t;

typedef struct {
  uint16_t              rnti;
  srsran_dci_format_t   format;
  srsran_dci_location_t location;
  uint32_t              ue_cc_idx;
  srsran_ra_type_t      alloc_type;
  union {
    srsran_ra_type0_t type0_alloc;
    srsran_ra_type1_t type1_alloc;
    srsran_ra_type2_t type2_alloc;
  };
  srsran_dci_tb_t tb[SRSRAN_MAX_CODEWORDS];
  bool            tb_cw_swap;
  uint32_t        pinfo;
  bool            pconf;
  bool            power_offset;
  uint8_t         tpc_pucch;
  bool            is_pdcch_order;
  uint32_t        preamble_idx;
  uint32_t        prach_mask_idx;
  uint32_t        cif;
  bool            cif_present;
  bool            srs_request;
  bool            srs_request_present;
  uint32_t        pid;
  uint32_t        dai;
  bool            is_tdd;
  bool            is_dwpts;
  bool            sram_id;
} srsran_dci_dl_t;

/* Unpacked DCI format 0 (dci.h:130-178, without the SRSRAN_DCI_HEXDEBUG members) */
typedef struct {
  uint16_t              rnti;
  srsran_dci_format_t   format;
  srsran_dci_location_t location;
  uint32_t              ue_cc_idx;
  srsran_ra_type2_t     type2_alloc;
  enum {
    SRSRAN_RA_PUSCH_HOP_DISABLED  = -1,
    SRSRAN_RA_PUSCH_HOP_QUART     = 0,
    SRSRAN_RA_PUSCH_HOP_QUART_NEG = 1,
    SRSRAN_RA_PUSCH_HOP_HALF      = 2,
    SRSRAN_RA_PUSCH_HOP_TYPE2     = 3
  } freq_hop_fl;
  srsran_dci_tb_t  tb;
  uint32_t         n_dmrs;
  bool             cqi_request;
  uint32_t         dai;
  uint32_t         ul_idx;
  bool             is_tdd;
  uint8_t          tpc_pusch;
  uint32_t         cif;
  bool             cif_present;
  uint8_t          multiple_csi_request;
  bool             multiple_csi_request_present;
  bool             srs_request;
  bool             srs_request_present;
  srsran_ra_type_t ra_type;
  bool             ra_type_present;
} srsran_dci_ul_t;

uint32_t srsran_dci_format_sizeof(const srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* cfg,
                                  srsran_dci_format_t format);                                 /* dci.c:359-413 */
int      srsran_dci_msg_unpack_pdsch(srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* cfg,
                                     srsran_dci_msg_t* msg, srsran_dci_dl_t* dci);             /* dci.c:1288-1340 */
int      srsran_dci_msg_pack_pdsch(srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* cfg,
                                   srsran_dci_dl_t* dci, srsran_dci_msg_t* msg);               /* dci.c:1243-1286 */
int      srsran_dci_msg_pack_pusch(srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* cfg,
                                   srsran_dci_ul_t* dci, srsran_dci_msg_t* msg);               /* dci.c:1342-1367 */
int      srsran_dci_msg_unpack_pusch(srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* cfg,
                                     srsran_dci_msg_t* msg, srsran_dci_ul_t* dci);             /* dci.c:1369-1395, 492-566 */
bool     srsran_dci_location_isvalid(srsran_dci_location_t* c);                                /* dci.c:1442-1449 */
int      srsran_dci_location_set(srsran_dci_location_t* c, uint32_t L, uint32_t nCCE);          /* dci.c:1425-1440 */
void     srsran_dci_cfg_set_common_ss(srsran_dci_cfg_t* cfg);                                  /* dci.c:1420-1423 */
bool     srsran_location_find_location(const srsran_dci_location_t* locations, uint32_t nof_locations,
                                       const srsran_dci_location_t* location);                /* dci.c:1407-1418 */

/* ---------------- ra_dl.h ---------------- */
int srsran_ra_dl_dci_to_grant(const srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_tm_t tm,
                              bool pdsch_use_tbs_index_alt, const srsran_dci_dl_t* dci,
                              srsran_pdsch_grant_t* grant);                                   /* ra_dl.c:610-647 */
uint32_t srsran_ra_dl_grant_nof_re(const srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf,
                                   srsran_pdsch_grant_t* grant);                              /* ra_dl.c:668-681 */

/* ---------------- regs.h ---------------- */
typedef struct {
  srsran_cell_t         cell;
  uint32_t              max_ctrl_symbols;
  uint32_t              ngroups_phich;
  uint32_t              ngroups_phich_m1;
  srsran_phich_r_t      phich_res;
  srsran_phich_length_t phich_len;
  uint32_t              phich_mi;
  uint32_t              pdcch_nregs[3]; /* usable PDCCH REGs per CFI (multiple of 9) */
  uint32_t              pcfich_re[16];  /* added: grid indices l * 12 * nof_prb + k, srsran_regs_pcfich_get order */
  uint32_t*             pdcch_re[3];    /* added: 4 * pdcch_nregs[c] grid indices per CFI, srsran_regs_pdcch_get order */
} srsran_regs_t;

int      srsran_regs_init(srsran_regs_t* h, srsran_cell_t cell);                                       /* regs.c:706-709 */
int      srsran_regs_init_opts(srsran_regs_t* h, srsran_cell_t cell, uint32_t phich_mi, bool mbsfn_or_sf1_6_tdd); /* regs.c:711-783 */
void     srsran_regs_free(srsran_regs_t* h);
int      srsran_regs_pdcch_nregs(srsran_regs_t* h, uint32_t cfi);
int      srsran_regs_pdcch_ncce(srsran_regs_t* h, uint32_t cfi);
uint32_t srsran_regs_pcfich_nregs(srsran_regs_t* h);
uint32_t srsran_regs_phich_ngroups(srsran_regs_t* h);
uint32_t srsran_regs_phich_ngroups_m1(srsran_regs_t* h);

/* ---------------- pcfich.h ---------------- */
#define PCFICH_CFI_LEN 32
#define PCFICH_RE 16
typedef struct {
  srsran_cell_t  cell;
  uint32_t       nof_rx_antennas;
  uint32_t       nof_symbols;
  srsran_regs_t* regs;
  float          data_f[PCFICH_CFI_LEN]; /* descrambled LLRs of the last decode (host copy) */
  void*          gpu;                    /* added: device tables, scratch and stream */
} srsran_pcfich_t;

int   srsran_pcfich_init(srsran_pcfich_t* q, uint32_t nof_rx_antennas);
void  srsran_pcfich_free(srsran_pcfich_t* q);
int   srsran_pcfich_set_cell(srsran_pcfich_t* q, srsran_regs_t* regs, srsran_cell_t cell);
/* sf_symbols: nof_rx host grids; channel->ce: full-grid host estimates.  Sets sf->cfi. */
int   srsran_pcfich_decode(srsran_pcfich_t* q, srsran_dl_sf_cfg_t* sf, srsran_chest_dl_res_t* channel,
                           cf_t* sf_symbols[SRSRAN_MAX_PORTS], float* corr_result);
float srsran_pcfich_cfi_decode(srsran_pcfich_t* q, uint32_t* cfi); /* on q->data_f (host, pcfich.c:113-134) */

/* ---------------- pdcch.h ---------------- */
typedef struct {
  srsran_cell_t  cell;
  uint32_t       nof_regs[3];
  uint32_t       nof_cce[3];
  uint32_t       max_bits;
  uint32_t       nof_rx_antennas;
  bool           is_ue;
  srsran_regs_t* regs;
  uint32_t       llr_cfi; /* added: CFI of the LLRs last extracted (device-resident) */
  void*          gpu;     /* added: device LLRs, sequences, tables, stream */
} srsran_pdcch_t;

int   srsran_pdcch_init_ue(srsran_pdcch_t* q, uint32_t max_prb, uint32_t nof_rx_antennas);
void  srsran_pdcch_free(srsran_pdcch_t* q);
void  srsran_pdcch_set_regs(srsran_pdcch_t* q, srsran_regs_t* regs);
int   srsran_pdcch_set_cell(srsran_pdcch_t* q, srsran_regs_t* regs, srsran_cell_t cell);
float srsran_pdcch_coderate(uint32_t nof_bits, uint32_t l);
/* Extracts, equalises, demodulates and descrambles the CFI's control region on the GPU; the
 * 72 * nof_cce float LLRs stay on the device for srsran_pdcch_decode_msg. */
int   srsran_pdcch_extract_llr(srsran_pdcch_t* q, srsran_dl_sf_cfg_t* sf, srsran_chest_dl_res_t* channel,
                               cf_t* sf_symbols[SRSRAN_MAX_PORTS]);
int   srsran_pdcch_decode_msg(srsran_pdcch_t* q, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* dci_cfg,
                              srsran_dci_msg_t* msg);
float srsran_pdcch_msg_corr(srsran_pdcch_t* q, srsran_dci_msg_t* msg);
/* Copies the device LLRs of the last extraction (72 * nof_cce floats) to llr; returns the count. */
int   srsran_pdcch_get_llr(srsran_pdcch_t* q, float* llr, uint32_t max);
/* added: loads n = 72 * nof_cce(cfi) host LLRs as the ones the next decodes use. */
int   srsran_pdcch_set_llr(srsran_pdcch_t* q, uint32_t cfi, const float* llr, uint32_t n);
uint32_t srsran_pdcch_ue_locations(srsran_pdcch_t* q, srsran_dl_sf_cfg_t* sf, srsran_dci_location_t* locations,
                                   uint32_t max_locations, uint16_t rnti);
uint32_t srsran_pdcch_ue_locations_ncce(uint32_t nof_cce, srsran_dci_location_t* c, uint32_t max_candidates,
                                        uint32_t sf_idx, uint16_t rnti);
uint32_t srsran_pdcch_ue_locations_ncce_L(uint32_t nof_cce, srsran_dci_location_t* c, uint32_t max_candidates,
                                          uint32_t sf_idx, uint16_t rnti, int Ls);
uint32_t srsran_pdcch_common_locations(srsran_pdcch_t* q, srsran_dci_location_t* locations, uint32_t max_locations,
                                       uint32_t cfi);
uint32_t srsran_pdcch_common_locations_ncce(uint32_t nof_cce, srsran_dci_location_t* c, uint32_t max_candidates);

/* added: nof_msg candidates decoded in one launch (each exactly as srsran_pdcch_decode_msg) with
 * their correlations (srsran_pdcch_msg_corr; 0 for skipped candidates). */
int srsran_pdcch_gpu_decode_msgs(srsran_pdcch_t* q, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* dci_cfg,
                                 srsran_dci_msg_t* msgs, uint32_t nof_msg, float* corr);

/* ---------------- ue_dl.h (control part) ---------------- */
/* Blind search of the DL DCIs of `rnti` (ue_dl.c:416-689) over the LLRs that
 * srsran_ue_dl_decode_fft_estimate extracted; every candidate of the search spaces is decoded in
 * one GPU launch. */
int srsran_ue_dl_find_dl_dci(srsran_ue_dl_t* q, srsran_dl_sf_cfg_t* sf, srsran_ue_dl_cfg_t* dl_cfg, uint16_t rnti,
                             srsran_dci_dl_t dci_dl[SRSRAN_MAX_DCI_MSG]);
int srsran_ue_dl_dci_to_pdsch_grant(srsran_ue_dl_t* q, srsran_dl_sf_cfg_t* sf, srsran_ue_dl_cfg_t* cfg,
                                    srsran_dci_dl_t* dci, srsran_pdsch_grant_t* grant);
/* The format 0 DCIs the last srsran_ue_dl_find_dl_dci call found for its C-RNTI (ue_dl.c:573-611:
 * no search of its own; the pending list is emptied), unpacked into dci_ul.  Returns their number. */
int srsran_ue_dl_find_ul_dci(srsran_ue_dl_t* q, srsran_dl_sf_cfg_t* sf, srsran_ue_dl_cfg_t* dl_cfg, uint16_t rnti,
                             srsran_dci_ul_t dci_ul[SRSRAN_MAX_DCI_MSG]);
/* PHICH m_i of the REG tables the PDCCH search uses (ue_dl.c:263-273, 296-313): auto = the FDD
 * value 1; manual = m_i of mi_idx (0, 1 or 2; srsUE's blind m_i search on unconfigured TDD cells). */
void srsran_ue_dl_set_mi_manual(srsran_ue_dl_t* q, uint32_t mi_idx);
void srsran_ue_dl_set_mi_auto(srsran_ue_dl_t* q);
/* MBSFN area of the PMCH (ue_dl.c:277-294): recorded in current_mbsfn_area_id; the PMCH itself is not
 * provided, so no MBSFN reference signal or scrambling is generated. */
int  srsran_ue_dl_set_mbsfn_area_id(srsran_ue_dl_t* q, uint16_t mbsfn_area_id);
void srsran_ue_dl_set_non_mbsfn_region(srsran_ue_dl_t* q, uint8_t non_mbsfn_region_length);

#ifdef __cplusplus
}
#endif
#endif /* SRSRAN_AMD_PDCCH_H */
