// srsran_4g_amd/csrc/dci_api.cpp -- DCI sizes and unpacking, and the DL resource allocation that
// turns a DCI into a PDSCH grant (include/srsran_pdcch.h).  Host code: a few hundred bit fields per
// subframe, nothing for the GPU.
//
//   DCI sizes      phch/dci.c:93-413 (FDD: 3-bit HARQ process number, no DAI; TDD: 4 bits + DAI)
//   DCI unpack     phch/dci.c:492-566 (format 0), :641-708 (format 1), :797-897 (1A), :1153-1241 (2 / 2A),
//                  :1288-1340, :1369-1395
//   DCI pack       phch/dci.c:415-490 (0), :579-639 (1), :710-795 (1A), :952-988 (1C), :1076-1151 (2/2A/2B),
//                  :1243-1286, :1342-1367
//   RA             phch/ra.c:37-250 (RIV, RBG size P, MCS -> I_TBS / modulation, TBS table)
//                  phch/ra_dl.c:42-681 (PRB allocation types 0 / 1 / 2, TB sizes, RE count, MIMO)
// TDD: 4-bit HARQ process numbers and the DAI / UL index (the reference's packers write no DAI: it stays in the zero
// padding, while its unpackers read it -- restated as is, dci.c:415-1367).
// Not provided (SRSRAN_ERROR): format 1B / 1D / 2B unpacking, 1B / 1D packing.
#include <cmath>
#include <cstdio>
#include <cstring>

#include "../../include/srsran_pdcch.h"

namespace {

#include "tbs_table.inc"

uint32_t riv_nbits(uint32_t nof_prb)
{
  return (uint32_t)ceilf(log2f((float)nof_prb * ((float)nof_prb + 1) / 2));
}

bool is_ambiguous_size(uint32_t n)
{
  static const uint32_t sizes[10] = {12, 14, 16, 20, 24, 26, 32, 40, 44, 56};
  for (uint32_t s : sizes) {
    if (n == s) {
      return true;
    }
  }
  return false;
}

// HARQ process number: 3 bits FDD, 4 bits TDD; TDD adds the 2-bit DAI (UL index with configuration 0) to formats
// 0 / 1 / 1A / 2 / 2A (dci.c:38-40, 142-143, 190-191, 217, 276-277, 313-349)
bool     is_tdd(const srsran_cell_t* cell) { return cell->frame_type == SRSRAN_TDD; }
uint32_t pid_len(const srsran_cell_t* cell) { return is_tdd(cell) ? 4 : 3; }
uint32_t dai_len(const srsran_cell_t* cell) { return is_tdd(cell) ? 2 : 0; }

uint32_t format0_size_(const srsran_cell_t* cell, const srsran_dci_cfg_t* cfg)
{
  return (cfg->cif_enabled ? 3 : 0) + 1 + 1 + riv_nbits(cell->nof_prb) + 5 + 1 + 2 + 3 + dai_len(cell) +
         ((cfg->multiple_csi_request_enabled && !cfg->is_not_ue_ss) ? 2 : 1) +
         ((cfg->srs_request_enabled && !cfg->is_not_ue_ss) ? 1 : 0) + 1;
}

uint32_t format1A_size(const srsran_cell_t* cell, const srsran_dci_cfg_t* cfg)
{
  uint32_t n = (cfg->cif_enabled ? 3 : 0) + 1 + 1 + riv_nbits(cell->nof_prb) + 5 + pid_len(cell) + 1 + 2 + 2 +
               dai_len(cell) + (cfg->srs_request_enabled ? 1 : 0);
  while (n < format0_size_(cell, cfg)) {
    n++;
  }
  if (is_ambiguous_size(n)) {
    n++;
  }
  return n;
}

uint32_t format0_size(const srsran_cell_t* cell, const srsran_dci_cfg_t* cfg)
{
  uint32_t n = format0_size_(cell, cfg);
  while (n < format1A_size(cell, cfg)) {
    n++;
  }
  return n;
}

uint32_t rbg_bits(uint32_t nof_prb) { return (uint32_t)ceilf((float)nof_prb / srsran_ra_type0_P(nof_prb)); }

uint32_t ra_type2_ngap(uint32_t nof_prb, bool ngap_is_1)  // ra.c:81-103
{
  if (nof_prb <= 10) {
    return nof_prb / 2;
  } else if (nof_prb == 11) {
    return 4;
  } else if (nof_prb <= 19) {
    return 8;
  } else if (nof_prb <= 26) {
    return 12;
  } else if (nof_prb <= 44) {
    return 18;
  } else if (nof_prb <= 49) {
    return 27;
  } else if (nof_prb <= 63) {
    return ngap_is_1 ? 27 : 9;
  } else if (nof_prb <= 79) {
    return ngap_is_1 ? 32 : 16;
  }
  return ngap_is_1 ? 48 : 16;
}

uint32_t ra_type2_n_vrb_dl(uint32_t nof_prb, bool ngap_is_1)  // ra.c:115-124
{
  const uint32_t ngap = ra_type2_ngap(nof_prb, ngap_is_1);
  return ngap_is_1 ? 2 * (ngap < nof_prb - ngap ? ngap : nof_prb - ngap) : (nof_prb / ngap) * 2 * ngap;
}

uint32_t format1C_size(const srsran_cell_t* cell)
{
  const uint32_t n_step = cell->nof_prb < 50 ? 2 : 4;
  uint32_t       n      = riv_nbits(ra_type2_n_vrb_dl(cell->nof_prb, true) / n_step) + 5;
  return cell->nof_prb >= 50 ? n + 1 : n;
}

uint32_t format2x_size(const srsran_cell_t* cell, const srsran_dci_cfg_t* cfg, srsran_dci_format_t f)
{
  uint32_t pbits = 0;
  if (f == SRSRAN_DCI_FORMAT2) {
    pbits = cell->nof_ports <= 2 ? 3 : 6;
  } else if (f == SRSRAN_DCI_FORMAT2A) {
    pbits = cell->nof_ports <= 2 ? 0 : 2;
  }
  uint32_t n = rbg_bits(cell->nof_prb) + 2 + pid_len(cell) + 1 + 2 * (5 + 1 + 2) + pbits + (cfg->cif_enabled ? 3 : 0) +
               dai_len(cell);
  if (cell->nof_prb > 10) {
    n++;
  }
  while (is_ambiguous_size(n)) {
    n++;
  }
  return n;
}

uint32_t bit_pack(const uint8_t** y, uint32_t n)
{
  uint32_t v = 0;
  for (uint32_t i = 0; i < n; i++) {
    v = (v << 1) | ((*y)[i] & 1u);
  }
  *y += n;
  return v;
}

// Format 0 (36.212 5.3.3.1.1; dci.c:492-566): after the optional CIF and the 0/1A flag, the fields
// in transmission order.  Width 0 = field absent in this configuration.
struct F0Field {
  enum Id { HOP, HOP_TYPE, RIV, MCS, NDI, TPC, DMRS, UL_IDX, DAI, CSI, CQI, SRS, RA_TYPE } id;
  uint32_t width;
};

int unpack_format0(const srsran_cell_t* cell, const srsran_dl_sf_cfg_t* sf, const srsran_dci_cfg_t* cfg,
                   srsran_dci_msg_t* msg, srsran_dci_ul_t* dci)
{
  const bool cfg0 = is_tdd(cell) && sf && sf->tdd_config.sf_config == 0;  // IS_TDD_CFG0: UL index instead of DAI
  const uint8_t* y = msg->payload;
  if (cfg->cif_enabled) {
    dci->cif         = bit_pack(&y, 3);
    dci->cif_present = true;
  }
  if (bit_pack(&y, 1) != 0) {
    return SRSRAN_ERROR;  // the flag says format 1A
  }
  msg->format = SRSRAN_DCI_FORMAT0;
  // hopping flag, then (if set) 1 or 2 hopping bits that the RIV gives up (36.213 Table 8.4-1)
  const bool     hop      = bit_pack(&y, 1) != 0;
  const uint32_t n_ul_hop = hop ? (cell->nof_prb < 50 ? 1u : 2u) : 0u;
  const bool     ue_ss    = !cfg->is_not_ue_ss;
  const F0Field  fields[] = {
      {F0Field::HOP_TYPE, n_ul_hop},
      {F0Field::RIV, riv_nbits(cell->nof_prb) - n_ul_hop},
      {F0Field::MCS, 5},
      {F0Field::NDI, 1},
      {F0Field::TPC, 2},
      {F0Field::DMRS, 3},
      {F0Field::UL_IDX, cfg0 ? 2u : 0u},
      {F0Field::DAI, is_tdd(cell) && !cfg0 ? 2u : 0u},
      {F0Field::CSI, cfg->multiple_csi_request_enabled && ue_ss ? 2u : 0u},
      {F0Field::CQI, cfg->multiple_csi_request_enabled && ue_ss ? 0u : 1u},
      {F0Field::SRS, cfg->srs_request_enabled && ue_ss ? 1u : 0u},
      {F0Field::RA_TYPE, cfg->ra_format_enabled ? 1u : 0u},
  };
  dci->freq_hop_fl = srsran_dci_ul_t::SRSRAN_RA_PUSCH_HOP_DISABLED;
  for (const F0Field& f : fields) {
    if (f.width == 0) {
      continue;
    }
    const uint32_t v = bit_pack(&y, f.width);
    switch (f.id) {
      case F0Field::HOP_TYPE:
        dci->freq_hop_fl = (decltype(dci->freq_hop_fl))v;
        break;
      case F0Field::RIV:
        dci->type2_alloc.riv = v;
        break;
      case F0Field::MCS:
        dci->tb.mcs_idx = v;
        break;
      case F0Field::NDI:
        dci->tb.ndi = v != 0;
        break;
      case F0Field::TPC:
        dci->tpc_pusch = (uint8_t)v;
        break;
      case F0Field::DMRS:
        dci->n_dmrs = v;
        break;
      case F0Field::UL_IDX:
        dci->ul_idx = v;
        dci->is_tdd = true;
        break;
      case F0Field::DAI:
        dci->dai    = v;
        dci->is_tdd = true;
        break;
      case F0Field::CSI:
        dci->multiple_csi_request_present = true;
        dci->multiple_csi_request         = (uint8_t)v;
        break;
      case F0Field::CQI:
        dci->cqi_request = v != 0;
        break;
      case F0Field::SRS:
        dci->srs_request_present = true;
        dci->srs_request         = v != 0;
        break;
      case F0Field::RA_TYPE:
        dci->ra_type_present = true;
        dci->ra_type         = (srsran_ra_type_t)(v != 0);
        break;
      default:
        break;
    }
  }
  return SRSRAN_SUCCESS;
}

void tb_disable(srsran_dci_tb_t& tb)
{
  tb.mcs_idx = 0;
  tb.rv      = 1;
}

// resource allocation of formats 1 / 2 / 2A: type 0 or type 1 (dci.c:657-680, 1172-1194)
int unpack_type01(const srsran_cell_t* cell, const uint8_t** y, srsran_dci_dl_t* dci)
{
  dci->alloc_type = cell->nof_prb > 10 ? (srsran_ra_type_t) * (*y)++ : SRSRAN_RA_ALLOC_TYPE0;
  const uint32_t P          = srsran_ra_type0_P(cell->nof_prb);
  const uint32_t alloc_size = rbg_bits(cell->nof_prb);
  switch (dci->alloc_type) {
    case SRSRAN_RA_ALLOC_TYPE0:
      dci->type0_alloc.rbg_bitmask = bit_pack(y, alloc_size);
      return SRSRAN_SUCCESS;
    case SRSRAN_RA_ALLOC_TYPE1: {
      const uint32_t lp            = (uint32_t)ceilf(log2f((float)P));
      dci->type1_alloc.rbg_subset  = bit_pack(y, lp);
      dci->type1_alloc.shift       = *(*y)++ ? true : false;
      dci->type1_alloc.vrb_bitmask = bit_pack(y, alloc_size - lp - 1);
      return SRSRAN_SUCCESS;
    }
    default:
      return SRSRAN_ERROR;
  }
}

int unpack_format1(const srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* cfg, srsran_dci_msg_t* msg,
                   srsran_dci_dl_t* dci)
{
  const uint8_t* y = msg->payload;
  if (msg->nof_bits != srsran_dci_format_sizeof(cell, sf, cfg, SRSRAN_DCI_FORMAT1)) {
    return SRSRAN_ERROR;
  }
  if (cfg->cif_enabled) {
    dci->cif         = bit_pack(&y, 3);
    dci->cif_present = true;
  }
  if (unpack_type01(cell, &y, dci)) {
    return SRSRAN_ERROR;
  }
  dci->tb[0].mcs_idx = bit_pack(&y, 5);
  dci->pid           = bit_pack(&y, pid_len(cell));
  dci->tb[0].ndi     = *y++ ? true : false;
  dci->tb[0].rv      = (int)bit_pack(&y, 2);
  dci->tpc_pucch     = (uint8_t)bit_pack(&y, 2);
  if (is_tdd(cell)) {  // dci.c:697-701
    dci->dai    = bit_pack(&y, 2);
    dci->is_tdd = true;
  }
  return SRSRAN_SUCCESS;
}

int unpack_format1A(const srsran_cell_t* cell, srsran_dci_cfg_t* cfg, srsran_dci_msg_t* msg, srsran_dci_dl_t* dci)
{
  const uint8_t* y = msg->payload;
  if (cfg->cif_enabled) {
    dci->cif         = bit_pack(&y, 3);
    dci->cif_present = true;
  }
  if (*y++ != 1) {
    return SRSRAN_ERROR;  // format 0
  }
  msg->format = SRSRAN_DCI_FORMAT1A;
  if (*y == 0) {  // PDCCH order: localized, RIV all ones, remaining bits zero (dci.c:822-843)
    const int nb = (int)riv_nbits(cell->nof_prb);
    int       i  = 0;
    while (i < nb && y[1 + i] == 1) {
      i++;
    }
    if (i == nb) {
      i = 1 + 10 + nb;
      while (i < (int)msg->nof_bits - 1 && y[i] == 0) {
        i++;
      }
      if (i == (int)msg->nof_bits - 1) {
        y += 1 + nb;
        dci->is_pdcch_order = true;
        dci->preamble_idx   = bit_pack(&y, 6);
        dci->prach_mask_idx = bit_pack(&y, 4);
        return SRSRAN_SUCCESS;
      }
    }
  }
  dci->is_pdcch_order    = false;
  dci->alloc_type        = SRSRAN_RA_ALLOC_TYPE2;
  dci->type2_alloc.mode  = *y++ ? srsran_ra_type2_t::SRSRAN_RA_TYPE2_DIST : srsran_ra_type2_t::SRSRAN_RA_TYPE2_LOC;
  dci->type2_alloc.n_gap = srsran_ra_type2_t::SRSRAN_RA_TYPE2_NG1;
  uint32_t nb_gap        = 0;
  const bool user        = SRSRAN_RNTI_ISUSER(msg->rnti);
  if (user && dci->type2_alloc.mode == srsran_ra_type2_t::SRSRAN_RA_TYPE2_DIST && cell->nof_prb >= 50) {
    nb_gap                 = 1;
    dci->type2_alloc.n_gap = *y++ ? srsran_ra_type2_t::SRSRAN_RA_TYPE2_NG2 : srsran_ra_type2_t::SRSRAN_RA_TYPE2_NG1;
  }
  dci->type2_alloc.riv = bit_pack(&y, riv_nbits(cell->nof_prb) - nb_gap);
  dci->tb[0].mcs_idx   = bit_pack(&y, 5);
  dci->pid             = bit_pack(&y, pid_len(cell));
  if (!user) {
    if (cell->nof_prb >= 50 && dci->type2_alloc.mode == srsran_ra_type2_t::SRSRAN_RA_TYPE2_DIST) {
      dci->type2_alloc.n_gap = *y++ ? srsran_ra_type2_t::SRSRAN_RA_TYPE2_NG2 : srsran_ra_type2_t::SRSRAN_RA_TYPE2_NG1;
    } else {
      y++;  // NDI reserved
    }
  } else {
    dci->tb[0].ndi = *y++ ? true : false;
  }
  dci->tb[0].rv = (int)bit_pack(&y, 2);
  if (user) {
    y += 2;  // TPC
  } else {
    y++;
    dci->type2_alloc.n_prb1a =
        *y++ ? srsran_ra_type2_t::SRSRAN_RA_TYPE2_NPRB1A_3 : srsran_ra_type2_t::SRSRAN_RA_TYPE2_NPRB1A_2;
  }
  if (is_tdd(cell)) {  // dci.c:890-894
    dci->dai    = bit_pack(&y, 2);
    dci->is_tdd = true;
  }
  return SRSRAN_SUCCESS;
}

int unpack_format1C(const srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* cfg, srsran_dci_msg_t* msg,
                    srsran_dci_dl_t* dci)  // dci.c:990-1023
{
  if (msg->nof_bits != srsran_dci_format_sizeof(cell, sf, cfg, SRSRAN_DCI_FORMAT1C)) {
    return SRSRAN_ERROR;
  }
  const uint8_t* y       = msg->payload;
  dci->alloc_type        = SRSRAN_RA_ALLOC_TYPE2;
  dci->type2_alloc.mode  = srsran_ra_type2_t::SRSRAN_RA_TYPE2_DIST;
  if (cell->nof_prb >= 50) {
    dci->type2_alloc.n_gap = *y++ ? srsran_ra_type2_t::SRSRAN_RA_TYPE2_NG2 : srsran_ra_type2_t::SRSRAN_RA_TYPE2_NG1;
  }
  const uint32_t n_step   = cell->nof_prb < 50 ? 2 : 4;
  const uint32_t n_vrb_dl =
      ra_type2_n_vrb_dl(cell->nof_prb, dci->type2_alloc.n_gap == srsran_ra_type2_t::SRSRAN_RA_TYPE2_NG1);
  dci->type2_alloc.riv = bit_pack(&y, riv_nbits(n_vrb_dl / n_step));
  dci->tb[0].mcs_idx   = bit_pack(&y, 5);
  dci->tb[0].rv        = -1;  // from the SFN / subframe, by the caller (36.321 5.3.1)
  msg->nof_bits        = (uint32_t)(y - msg->payload);
  return SRSRAN_SUCCESS;
}

int unpack_format2x(const srsran_cell_t* cell, srsran_dci_cfg_t* cfg, srsran_dci_msg_t* msg, srsran_dci_dl_t* dci)
{
  const uint8_t* y = msg->payload;
  if (cfg->cif_enabled) {
    dci->cif         = bit_pack(&y, 3);
    dci->cif_present = true;
  }
  if (unpack_type01(cell, &y, dci)) {
    return SRSRAN_ERROR;
  }
  dci->tpc_pucch  = (uint8_t)bit_pack(&y, 2);
  if (is_tdd(cell)) {  // dci.c:1193-1197: the DAI between the TPC command and the HARQ process
    dci->dai    = bit_pack(&y, 2);
    dci->is_tdd = true;
  }
  dci->pid = bit_pack(&y, pid_len(cell));
  if (msg->format == SRSRAN_DCI_FORMAT2B) {  // dci.c:1203-1207: the scrambling identity in the swap flag's place
    dci->sram_id = *y++ ? true : false;
  } else {
    dci->tb_cw_swap = *y++ ? true : false;
  }
  uint32_t nof_tb = 0;
  for (int i = 0; i < SRSRAN_MAX_CODEWORDS; i++) {
    dci->tb[i].mcs_idx = bit_pack(&y, 5);
    dci->tb[i].ndi     = *y++ ? true : false;
    dci->tb[i].rv      = (int)bit_pack(&y, 2);
    if (SRSRAN_DCI_IS_TB_EN(dci->tb[i])) {
      nof_tb++;
    }
  }
  if (msg->format == SRSRAN_DCI_FORMAT2) {
    dci->pinfo = bit_pack(&y, cell->nof_ports <= 2 ? 3 : 6);
  } else if (msg->format == SRSRAN_DCI_FORMAT2A) {
    dci->pinfo = bit_pack(&y, cell->nof_ports <= 2 ? 0 : 2);
  }
  for (int i = 0; i < SRSRAN_MAX_CODEWORDS; i++) {
    dci->tb[i].cw_idx = nof_tb == 2 ? (uint32_t)(((dci->tb_cw_swap ? 1 : 0) + i) % nof_tb) : 0;
  }
  return SRSRAN_SUCCESS;
}

// ---- DCI packing (the eNB side: srsran_enb_dl_put_pdcch_dl / _ul, dci.c:415-490, 579-639, 710-795,
// 952-988, 1076-1151) ----
void bit_put(uint8_t** y, uint32_t v, uint32_t n)  // MSB first, as srsran_bit_unpack
{
  for (uint32_t i = 0; i < n; i++) {
    *(*y)++ = (uint8_t)((v >> (n - 1 - i)) & 1u);
  }
}

// zero padding up to the format's size; the reference leaves its "reserved" bits as they were in a
// message it zeroed first (enb_dl.c:390), so they are written as zeros here
void pad_to(srsran_dci_msg_t* msg, uint8_t* y, uint32_t n)
{
  while ((uint32_t)(y - msg->payload) < n) {
    *y++ = 0;
  }
  msg->nof_bits = (uint32_t)(y - msg->payload);
}

int pack_format0(const srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, const srsran_dci_cfg_t* cfg, const srsran_dci_ul_t* dci,
                 srsran_dci_msg_t* msg)
{
  uint8_t* y = msg->payload;
  if (dci->cif_present) {
    bit_put(&y, dci->cif, 3);
  }
  *y++                = 0;  // format 0 / 1A flag
  uint32_t n_ul_hop   = 0;
  const bool hop      = dci->freq_hop_fl != srsran_dci_ul_t::SRSRAN_RA_PUSCH_HOP_DISABLED;
  *y++                = hop ? 1 : 0;
  if (hop) {
    n_ul_hop = cell->nof_prb < 50 ? 1 : 2;  // 36.213 Table 8.4-1
    bit_put(&y, (uint32_t)dci->freq_hop_fl, n_ul_hop);
  }
  const bool ue_ss = !cfg->is_not_ue_ss;
  bit_put(&y, dci->type2_alloc.riv, riv_nbits(cell->nof_prb) - n_ul_hop);
  bit_put(&y, dci->tb.mcs_idx, 5);
  *y++ = dci->tb.ndi ? 1 : 0;
  bit_put(&y, dci->tpc_pusch, 2);
  bit_put(&y, dci->n_dmrs, 3);
  *y++ = dci->cqi_request ? 1 : 0;
  if (cfg->multiple_csi_request_enabled && ue_ss) {
    *y++ = 0;
  }
  if (cfg->srs_request_enabled && ue_ss) {
    *y++ = dci->srs_request && dci->srs_request_present ? 1 : 0;
  }
  pad_to(msg, y, srsran_dci_format_sizeof(cell, sf, const_cast<srsran_dci_cfg_t*>(cfg), SRSRAN_DCI_FORMAT0));
  return SRSRAN_SUCCESS;
}

int pack_type01(const srsran_cell_t* cell, uint8_t** y, const srsran_dci_dl_t* dci)
{
  if (cell->nof_prb > 10) {
    *(*y)++ = (uint8_t)dci->alloc_type;
  }
  const uint32_t P = srsran_ra_type0_P(cell->nof_prb), alloc_size = rbg_bits(cell->nof_prb);
  switch (dci->alloc_type) {
    case SRSRAN_RA_ALLOC_TYPE0:
      bit_put(y, dci->type0_alloc.rbg_bitmask, alloc_size);
      return SRSRAN_SUCCESS;
    case SRSRAN_RA_ALLOC_TYPE1: {
      const uint32_t lp = (uint32_t)ceilf(log2f((float)P));
      bit_put(y, dci->type1_alloc.rbg_subset, lp);
      *(*y)++ = dci->type1_alloc.shift ? 1 : 0;
      bit_put(y, dci->type1_alloc.vrb_bitmask, alloc_size - lp - 1);
      return SRSRAN_SUCCESS;
    }
    default:
      fprintf(stderr, "[srsran_dci] formats 1 / 2 take resource allocation type 0 or 1\n");
      return SRSRAN_ERROR;
  }
}

int pack_format1(const srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* cfg, const srsran_dci_dl_t* dci,
                 srsran_dci_msg_t* msg)
{
  uint8_t* y = msg->payload;
  if (dci->cif_present) {
    bit_put(&y, dci->cif, 3);
  }
  if (pack_type01(cell, &y, dci)) {
    return SRSRAN_ERROR;
  }
  bit_put(&y, dci->tb[0].mcs_idx, 5);
  bit_put(&y, dci->pid, pid_len(cell));  // no DAI: the reference packers leave it to the padding
  *y++ = dci->tb[0].ndi ? 1 : 0;
  bit_put(&y, (uint32_t)dci->tb[0].rv, 2);
  bit_put(&y, dci->tpc_pucch, 2);
  pad_to(msg, y, srsran_dci_format_sizeof(cell, sf, cfg, SRSRAN_DCI_FORMAT1));
  return SRSRAN_SUCCESS;
}

int pack_format1A(const srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* cfg, const srsran_dci_dl_t* dci,
                  srsran_dci_msg_t* msg)
{
  uint8_t* y = msg->payload;
  if (dci->cif_present) {
    bit_put(&y, dci->cif, 3);
  }
  *y++ = 1;  // format 0 / 1A flag
  if (dci->is_pdcch_order) {  // localized, RIV all ones, preamble and PRACH mask indices (36.212 5.3.3.1.3)
    *y++ = 0;
    bit_put(&y, 0xffffffffu, riv_nbits(cell->nof_prb));
    bit_put(&y, dci->preamble_idx, 6);
    bit_put(&y, dci->prach_mask_idx, 4);
  } else {
    if (dci->alloc_type != SRSRAN_RA_ALLOC_TYPE2) {
      fprintf(stderr, "[srsran_dci] format 1A takes resource allocation type 2\n");
      return SRSRAN_ERROR;
    }
    const bool user = SRSRAN_RNTI_ISUSER(dci->rnti);
    const bool dist = dci->type2_alloc.mode == srsran_ra_type2_t::SRSRAN_RA_TYPE2_DIST;
    *y++            = dist ? 1 : 0;
    uint32_t nb_gap = 0;
    if (user && dist && cell->nof_prb >= 50) {
      nb_gap = 1;
      *y++   = (uint8_t)dci->type2_alloc.n_gap;
    }
    bit_put(&y, dci->type2_alloc.riv, riv_nbits(cell->nof_prb) - nb_gap);
    bit_put(&y, dci->tb[0].mcs_idx, 5);
    bit_put(&y, dci->pid, pid_len(cell));  // no DAI: the reference packers leave it to the padding
    if (user) {
      *y++ = dci->tb[0].ndi ? 1 : 0;
    } else {
      *y++ = cell->nof_prb >= 50 && dist ? (uint8_t)dci->type2_alloc.n_gap : 0;
    }
    bit_put(&y, (uint32_t)dci->tb[0].rv, 2);
    if (user) {
      bit_put(&y, 0, 2);  // TPC (not provided by the reference either)
    } else {
      *y++ = 0;  // TPC MSB reserved, LSB = N_PRB^1A for the TBS
      *y++ = (uint8_t)dci->type2_alloc.n_prb1a;
    }
  }
  pad_to(msg, y, srsran_dci_format_sizeof(cell, sf, cfg, SRSRAN_DCI_FORMAT1A));
  return SRSRAN_SUCCESS;
}

int pack_format1C(const srsran_cell_t* cell, const srsran_dci_dl_t* dci, srsran_dci_msg_t* msg)
{
  uint8_t* y = msg->payload;
  if (dci->cif_present) {
    bit_put(&y, dci->cif, 3);
  }
  if (dci->alloc_type != SRSRAN_RA_ALLOC_TYPE2 || dci->type2_alloc.mode != srsran_ra_type2_t::SRSRAN_RA_TYPE2_DIST) {
    fprintf(stderr, "[srsran_dci] format 1C takes distributed type 2 resource allocation\n");
    return SRSRAN_ERROR;
  }
  if (cell->nof_prb >= 50) {
    *y++ = (uint8_t)dci->type2_alloc.n_gap;
  }
  const uint32_t n_step   = cell->nof_prb < 50 ? 2 : 4;
  const uint32_t n_vrb_dl = ra_type2_n_vrb_dl(cell->nof_prb, dci->type2_alloc.n_gap == srsran_ra_type2_t::SRSRAN_RA_TYPE2_NG1);
  bit_put(&y, dci->type2_alloc.riv, riv_nbits(n_vrb_dl / n_step));
  bit_put(&y, dci->tb[0].mcs_idx, 5);
  msg->nof_bits = (uint32_t)(y - msg->payload);  // no padding (dci.c:986)
  return SRSRAN_SUCCESS;
}

int pack_format2x(const srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* cfg, const srsran_dci_dl_t* dci,
                  srsran_dci_msg_t* msg)
{
  uint8_t* y = msg->payload;
  if (dci->cif_present) {
    bit_put(&y, dci->cif, 3);
  }
  if (pack_type01(cell, &y, dci)) {
    return SRSRAN_ERROR;
  }
  bit_put(&y, dci->tpc_pucch, 2);
  bit_put(&y, dci->pid, pid_len(cell));  // no DAI: the reference packers leave it to the padding
  *y++ = (msg->format == SRSRAN_DCI_FORMAT2B ? dci->sram_id : dci->tb_cw_swap) ? 1 : 0;
  for (int i = 0; i < 2; i++) {
    bit_put(&y, dci->tb[i].mcs_idx, 5);
    *y++ = dci->tb[i].ndi ? 1 : 0;
    bit_put(&y, (uint32_t)dci->tb[i].rv, 2);
  }
  if (msg->format == SRSRAN_DCI_FORMAT2) {
    bit_put(&y, dci->pinfo, cell->nof_ports <= 2 ? 3 : 6);
  } else if (msg->format == SRSRAN_DCI_FORMAT2A) {
    bit_put(&y, dci->pinfo, cell->nof_ports <= 2 ? 0 : 2);
  }
  pad_to(msg, y, srsran_dci_format_sizeof(cell, sf, cfg, msg->format));
  return SRSRAN_SUCCESS;
}

// ---- ra_dl.c ----
uint32_t ra_re_x_prb(const srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, uint32_t slot, uint32_t prb)
{
  // PDSCH REs of one PRB in one slot (ra_dl.c:42-161): normal subframes of FDD and TDD cells, normal or extended CP.
  // A TDD special subframe counts only its DwPTS symbols in each slot.  Unsigned arithmetic as the reference's.
  const uint32_t sfi    = sf->tti % 10;
  const uint32_t nctrl  = cell->nof_prb <= 10 ? sf->cfi + 1 : sf->cfi;  // SRSRAN_NOF_CTRL_SYMBOLS
  const bool     ext    = cell->cp == SRSRAN_CP_EXT;
  const bool     tdd    = cell->frame_type == SRSRAN_TDD;
  const uint32_t np     = cell->nof_ports;
  uint32_t       nsym   = SRSRAN_CP_NSYMB(cell->cp);
  if (tdd && srsran_sfidx_tdd_type(sf->tdd_config, sfi) == SRSRAN_TDD_SF_S) {
    nsym = srsran_sfidx_tdd_nof_dw_slot(sf->tdd_config, slot, cell->cp);
  }
  uint32_t   re     = slot == 0 ? (nsym - nctrl) * 12 : nsym * 12;
  bool       refs   = true;  // remove the CRS REs below
  const bool centre = prb >= cell->nof_prb / 2 - 3 && prb < cell->nof_prb / 2 + 3 + (cell->nof_prb % 2);
  const bool half   = (cell->nof_prb % 2) && (prb == cell->nof_prb / 2 - 3 || prb == cell->nof_prb / 2 + 3);
  if (!tdd) {  // PSS / SSS at the end of slot 0 of subframes 0 / 5, PBCH in slot 1 of subframe 0
    if ((sfi == 0 || sfi == 5) && centre) {
      if (sfi == 0) {
        if (slot == 0) {
          re = (nsym - nctrl - 2) * 12;
        } else if (ext) {
          re   = (nsym - 4) * 12;  // both CRS symbols of the slot fall under the PBCH
          refs = false;
        } else {
          re = (nsym - 4) * 12 + 2 * np;
        }
      } else if (slot == 0) {
        re = (nsym - nctrl - 2) * 12;
      }
      if (half) {
        if (slot == 0) {
          re += 2 * 12 / 2;
        } else if (sfi == 0) {
          re += 4 * 12 / 2 - np;
          if (ext) {
            re -= np > 2 ? 2 : np;
          }
        }
      }
    }
  } else {  // SSS in the last symbol of subframes 0 / 5 (+ PBCH in subframe 0), PSS in symbol 2 of subframes 1 / 6
    if ((((sfi == 0 || sfi == 5) && slot == 1) || ((sfi == 1 || sfi == 6) && slot == 0)) && centre) {
      if (sfi == 0) {
        if (ext) {
          re   = (nsym - 5) * 12;
          refs = false;
        } else {
          re = (nsym - 5) * 12 + 2 * np;
        }
      } else if (sfi == 5) {
        re = (nsym - 1) * 12;
      } else {
        re = (nsym - nctrl - 1) * 12;
      }
      if (half) {
        re += 12 / 2;
        if (sfi == 0) {
          re += 4 * 12 / 2 - np;
          if (ext) {
            re -= np > 2 ? 2 : np;
          }
        }
      }
    }
  }
  if (refs) {  // CRS of the slot's symbols (a short DwPTS holds fewer of them)
    const bool full = (!ext && nsym >= 5) || (ext && nsym >= 4);
    switch (np) {
      case 1:
      case 2:
        if (full) {
          re -= 2 * (slot + 1) * np;
        } else if (slot == 1 && nsym >= 1) {
          re -= 2 * np;
        }
        break;
      case 4:
        if (slot == 1) {
          if (full) {
            re -= 12;
          } else if (nsym >= 2) {
            re -= 8;
          }
        } else if (full) {
          re -= 4;
          if (nctrl == 1) {
            re -= 4;
          }
        }
        break;
    }
  }
  return re;
}

int prb_allocation(const srsran_dci_dl_t* dci, srsran_pdsch_grant_t* grant, uint32_t nof_prb)
{
  const uint32_t P = srsran_ra_type0_P(nof_prb);
  switch (dci->alloc_type) {
    case SRSRAN_RA_ALLOC_TYPE0: {
      const uint32_t bm = dci->type0_alloc.rbg_bitmask;
      const int      nb = (int)ceilf((float)nof_prb / P);
      for (int i = 0; i < nb; i++) {
        if (bm & (1u << (nb - i - 1))) {
          for (uint32_t j = 0; j < P; j++) {
            if (i * P + j < nof_prb) {
              grant->prb_idx[0][i * P + j] = true;
              grant->nof_prb++;
            }
          }
        }
      }
      break;
    }
    case SRSRAN_RA_ALLOC_TYPE1: {
      if (dci->type1_alloc.rbg_subset >= P) {
        return SRSRAN_ERROR;
      }
      const uint32_t n_rb_type1 = srsran_ra_type1_N_rb(nof_prb);
      const uint32_t temp       = ((nof_prb - 1) / P) % P;
      uint32_t       n_rb_sub;
      if (dci->type1_alloc.rbg_subset < temp) {
        n_rb_sub = ((nof_prb - 1) / (P * P)) * P + P;
      } else if (dci->type1_alloc.rbg_subset == temp) {
        n_rb_sub = ((nof_prb - 1) / (P * P)) * P + ((nof_prb - 1) % P) + 1;
      } else {
        n_rb_sub = ((nof_prb - 1) / (P * P)) * P;
      }
      const int shift = dci->type1_alloc.shift ? (int)(n_rb_sub - n_rb_type1) : 0;
      for (uint32_t i = 0; i < n_rb_type1; i++) {
        if (dci->type1_alloc.vrb_bitmask & (1u << (n_rb_type1 - i - 1))) {
          const uint32_t idx = ((i + shift) / P) * P * P + dci->type1_alloc.rbg_subset * P + (i + shift) % P;
          if (idx >= nof_prb) {
            return SRSRAN_ERROR;
          }
          grant->prb_idx[0][idx] = true;
          grant->nof_prb++;
        }
      }
      break;
    }
    case SRSRAN_RA_ALLOC_TYPE2: {  // ra_dl.c:225-316
      const bool dist = dci->type2_alloc.mode != srsran_ra_type2_t::SRSRAN_RA_TYPE2_LOC;
      const bool ng1  = dci->type2_alloc.n_gap == srsran_ra_type2_t::SRSRAN_RA_TYPE2_NG1;
      uint32_t   nof_vrb = dist ? ra_type2_n_vrb_dl(nof_prb, ng1) : nof_prb, nof_prb_t2 = nof_prb, n_step = 1;
      if (dci->format == SRSRAN_DCI_FORMAT1C) {  // 36.213 7.1.6.3: RIV in units of N_RB^step
        n_step = nof_prb < 50 ? 2 : 4;
        nof_vrb /= n_step;
        nof_prb_t2 = nof_vrb;
      }
      uint32_t L_crb = 0, RB_start = 0;
      srsran_ra_type2_from_riv(dci->type2_alloc.riv, &L_crb, &RB_start, nof_prb_t2, nof_vrb);
      L_crb *= n_step;
      RB_start *= n_step;
      if (!dist) {
        for (uint32_t i = 0; i < L_crb; i++) {
          if (i + RB_start >= SRSRAN_MAX_PRB) {
            return SRSRAN_ERROR;
          }
          grant->prb_idx[0][i + RB_start] = true;
          grant->nof_prb++;
        }
        memcpy(grant->prb_idx[1], grant->prb_idx[0], sizeof(grant->prb_idx[0]));
        return SRSRAN_SUCCESS;
      }
      // distributed VRBs: the interleaver of 36.211 6.2.3.2, even slot (prb_idx[0]) and odd slot (prb_idx[1])
      const int N_vrb = ng1 ? (int)ra_type2_n_vrb_dl(nof_prb, true) : 2 * (int)ra_type2_n_vrb_dl(nof_prb, true);
      const int N_gap = (int)ra_type2_ngap(nof_prb, ng1);
      const int N_row = (int)ceilf((float)N_vrb / (4 * P)) * (int)P;
      const int N_null = 4 * N_row - N_vrb;
      for (int i = 0; i < (int)L_crb; i++) {
        const int n_vrb = i + (int)RB_start, nt_vrb = n_vrb % N_vrb, blk = N_vrb * (n_vrb / N_vrb);
        const int nt_prb  = 2 * N_row * (nt_vrb % 2) + nt_vrb / 2 + blk;
        const int nt2_prb = N_row * (nt_vrb % 4) + nt_vrb / 4 + blk;
        int       odd;
        if (N_null != 0 && nt_vrb >= N_vrb - N_null && nt_vrb % 2 == 1) {
          odd = nt_prb - N_row;
        } else if (N_null != 0 && nt_vrb >= N_vrb - N_null && nt_vrb % 2 == 0) {
          odd = nt_prb - N_row + N_null / 2;
        } else if (N_null != 0 && nt_vrb < N_vrb - N_null && nt_vrb % 4 >= 2) {
          odd = nt2_prb - N_null / 2;
        } else {
          odd = nt2_prb;
        }
        const int even = (odd + N_vrb / 2) % N_vrb + blk;
        const int p0 = odd < N_vrb / 2 ? odd : odd + N_gap - N_vrb / 2;
        const int p1 = even < N_vrb / 2 ? even : even + N_gap - N_vrb / 2;
        if (p0 < 0 || p0 >= (int)nof_prb || p1 < 0 || p1 >= (int)nof_prb) {
          return SRSRAN_ERROR;
        }
        grant->prb_idx[0][p0] = true;
        grant->prb_idx[1][p1] = true;
        grant->nof_prb++;
      }
      return SRSRAN_SUCCESS;
    }
    default:
      return SRSRAN_ERROR;
  }
  memcpy(grant->prb_idx[1], grant->prb_idx[0], sizeof(grant->prb_idx[0]));
  return SRSRAN_SUCCESS;
}

int compute_tb(bool alt, const srsran_dci_dl_t* dci, srsran_pdsch_grant_t* grant)  // ra_dl.c:345-422
{
  for (int i = 0; i < SRSRAN_MAX_CODEWORDS; i++) {
    grant->tb[i].mcs_idx = dci->tb[i].mcs_idx;
    grant->tb[i].rv      = dci->tb[i].rv;
    grant->tb[i].cw_idx  = dci->tb[i].cw_idx;
    if ((SRSRAN_DCI_IS_TB_EN(dci->tb[i]) && dci->format >= SRSRAN_DCI_FORMAT2) ||
        (dci->format < SRSRAN_DCI_FORMAT2 && i == 0)) {
      grant->tb[i].enabled = true;
      grant->nof_tb++;
    } else {
      grant->tb[i].enabled = false;
    }
  }
  if (dci->format == SRSRAN_DCI_FORMAT1A || !SRSRAN_RNTI_ISUSER(dci->rnti)) {
    alt = false;
  }
  if (!SRSRAN_RNTI_ISUSER(dci->rnti) && dci->rnti != SRSRAN_MRNTI) {  // ra_dl.c:374-399
    int tbs = -1;
    if (dci->format == SRSRAN_DCI_FORMAT1A) {
      const uint32_t n_prb = dci->type2_alloc.n_prb1a == srsran_ra_type2_t::SRSRAN_RA_TYPE2_NPRB1A_2 ? 2 : 3;
      tbs                  = srsran_ra_tbs_from_idx(dci->tb[0].mcs_idx, n_prb);
    } else if (dci->format == SRSRAN_DCI_FORMAT1C) {  // 36.213 Table 7.1.7.2.3-1
      static const int kTbs1C[32] = {40,  56,  72,  120, 136, 144, 176, 208,  224,  256,  280,  296,  328,  336,  392,  488,
                                     552, 600, 632, 696, 776, 840, 904, 1000, 1064, 1128, 1224, 1288, 1384, 1480, 1608, 1736};
      if (dci->tb[0].mcs_idx < 32) {
        tbs = kTbs1C[dci->tb[0].mcs_idx];
      }
    } else {
      fprintf(stderr, "[srsran_ra] P/SI/RA-RNTI grants: formats 1A / 1C only\n");
      return SRSRAN_ERROR;
    }
    if (tbs < 0) {
      return SRSRAN_ERROR;
    }
    grant->tb[0].mod = SRSRAN_MOD_QPSK;
    grant->tb[0].tbs = tbs;
    return SRSRAN_SUCCESS;
  }
  // a TDD special subframe scales the PRB count for the TBS look-up (ra_dl.c:401-405, 36.213 7.1.7)
  const double   scaled = 0.75 * grant->nof_prb;
  const uint32_t n_prb  = dci->is_dwpts ? (uint32_t)(scaled > 1 ? scaled : 1) : grant->nof_prb;
  for (int i = 0; i < SRSRAN_MAX_CODEWORDS; i++) {
    if (!grant->tb[i].enabled) {
      grant->tb[i].tbs = 0;
      continue;
    }
    // srsran_dl_fill_ra_mcs (ra_dl.c:323-341): a retransmission MCS (no TBS index) stores last_tbs in the TB, but the
    // function returns 0 and its caller stores that (ra_dl.c:409)
    grant->tb[i].mod = srsran_ra_dl_mod_from_mcs(grant->tb[i].mcs_idx, alt);
    const int i_tbs  = srsran_ra_tbs_idx_from_mcs(grant->tb[i].mcs_idx, alt, false);
    grant->tb[i].tbs = i_tbs >= 0 ? srsran_ra_tbs_from_idx((uint32_t)i_tbs, n_prb) : 0;
    if (grant->tb[i].tbs < 0) {
      return SRSRAN_ERROR;
    }
  }
  return SRSRAN_SUCCESS;
}

int config_mimo(const srsran_cell_t* cell, srsran_tm_t tm, const srsran_dci_dl_t* dci, srsran_pdsch_grant_t* grant)
{
  const uint32_t nof_tb = grant->nof_tb;
  grant->tx_scheme      = SRSRAN_TXSCHEME_PORT0;
  bool valid            = true;
  switch (tm) {  // ra_dl.c:451-507
    case SRSRAN_TM1:
    case SRSRAN_TM2:
      grant->tx_scheme = cell->nof_ports > 1 ? SRSRAN_TXSCHEME_DIVERSITY : SRSRAN_TXSCHEME_PORT0;
      valid            = nof_tb == 1;
      break;
    case SRSRAN_TM3:
      if (nof_tb == 1) {
        grant->tx_scheme = SRSRAN_TXSCHEME_DIVERSITY;
      } else if (nof_tb == 2) {
        grant->tx_scheme = SRSRAN_TXSCHEME_CDD;
      } else {
        valid = false;
      }
      break;
    case SRSRAN_TM4:
      if (nof_tb == 1) {
        grant->tx_scheme = dci->pinfo == 0 ? SRSRAN_TXSCHEME_DIVERSITY : SRSRAN_TXSCHEME_SPATIALMUX;
      } else if (nof_tb == 2) {
        grant->tx_scheme = SRSRAN_TXSCHEME_SPATIALMUX;
      } else {
        valid = false;
      }
      break;
    case SRSRAN_TM5:
    case SRSRAN_TM6:
    case SRSRAN_TM7:
    case SRSRAN_TM8:
      break;
    default:
      valid = false;
  }
  if (!valid) {
    return SRSRAN_ERROR;
  }
  if (grant->tx_scheme == SRSRAN_TXSCHEME_SPATIALMUX) {  // ra_dl.c:509-538
    if (nof_tb == 1) {
      if (dci->pinfo > 0 && dci->pinfo < 5) {
        grant->pmi = dci->pinfo - 1;
      } else {
        return SRSRAN_ERROR;
      }
    } else {
      if (dci->pinfo >= 2) {
        return SRSRAN_ERROR;
      }
      grant->pmi = dci->pinfo % 2;
    }
  }
  switch (grant->tx_scheme) {  // ra_dl.c:540-581
    case SRSRAN_TXSCHEME_PORT0:
      if (nof_tb != 1) {
        return SRSRAN_ERROR;
      }
      grant->nof_layers = 1;
      break;
    case SRSRAN_TXSCHEME_DIVERSITY:
      if (nof_tb != 1) {
        return SRSRAN_ERROR;
      }
      grant->nof_layers = cell->nof_ports;
      break;
    case SRSRAN_TXSCHEME_SPATIALMUX:
      grant->nof_layers = nof_tb;
      break;
    case SRSRAN_TXSCHEME_CDD:
      if (nof_tb != 2) {
        return SRSRAN_ERROR;
      }
      grant->nof_layers = 2;
      break;
  }
  return SRSRAN_SUCCESS;
}

}  // namespace

extern "C" {

uint32_t srsran_ra_type0_P(uint32_t nof_prb)
{
  return nof_prb <= 10 ? 1 : nof_prb <= 26 ? 2 : nof_prb <= 63 ? 3 : 4;
}

uint32_t srsran_ra_type1_N_rb(uint32_t nof_prb)
{
  const uint32_t P = srsran_ra_type0_P(nof_prb);
  return (uint32_t)ceilf((float)nof_prb / P) - (uint32_t)ceilf(log2f((float)P)) - 1;
}

uint32_t srsran_ra_type2_to_riv(uint32_t L_crb, uint32_t RB_start, uint32_t nof_prb)
{
  return (L_crb - 1) <= nof_prb / 2 ? nof_prb * (L_crb - 1) + RB_start
                                    : nof_prb * (nof_prb - L_crb + 1) + nof_prb - 1 - RB_start;
}

void srsran_ra_type2_from_riv(uint32_t riv, uint32_t* L_crb, uint32_t* RB_start, uint32_t nof_prb, uint32_t nof_vrb)
{
  *L_crb    = riv / nof_prb + 1;
  *RB_start = riv % nof_prb;
  if (*L_crb > nof_vrb - *RB_start) {
    *L_crb    = nof_prb - riv / nof_prb + 1;
    *RB_start = nof_prb - riv % nof_prb - 1;
  }
}

int srsran_ra_tbs_idx_from_mcs(uint32_t mcs, bool use_tbs_index_alt, bool is_ul)
{
  if (is_ul) {
    static const int ul[29] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 19, 20, 21,
                               22, 23, 24, 25, 26};  // 36.213 Table 8.6.1-1
    return mcs < 29 ? ul[mcs] : SRSRAN_ERROR;
  }
  if (use_tbs_index_alt) {
    return mcs < 28 ? kDlMcsTbsAlt[mcs] : SRSRAN_ERROR;
  }
  return mcs < 29 ? kDlMcsTbs[mcs] : SRSRAN_ERROR;
}

srsran_mod_t srsran_ra_dl_mod_from_mcs(uint32_t mcs, bool use_tbs_index_alt)
{
  if (use_tbs_index_alt) {
    if (mcs < 5 || mcs == 28) {
      return SRSRAN_MOD_QPSK;
    } else if (mcs < 11 || mcs == 29) {
      return SRSRAN_MOD_16QAM;
    } else if (mcs < 20 || mcs == 30) {
      return SRSRAN_MOD_64QAM;
    }
    return SRSRAN_MOD_256QAM;
  }
  if (mcs < 10 || mcs == 29) {
    return SRSRAN_MOD_QPSK;
  } else if (mcs < 17 || mcs == 30) {
    return SRSRAN_MOD_16QAM;
  }
  return SRSRAN_MOD_64QAM;
}

int srsran_ra_tbs_from_idx(uint32_t tbs_idx, uint32_t n_prb)
{
  if (tbs_idx < SRSRAN_RA_NOF_TBS_IDX && n_prb > 0 && n_prb <= SRSRAN_MAX_PRB) {
    return kTbs[tbs_idx][n_prb - 1];
  }
  return SRSRAN_ERROR;
}

uint32_t srsran_dci_format_sizeof(const srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* cfg,
                                  srsran_dci_format_t format)
{
  (void)sf;
  srsran_dci_cfg_t zero;
  memset(&zero, 0, sizeof(zero));
  const srsran_dci_cfg_t* c = cfg ? cfg : &zero;
  switch (format) {
    case SRSRAN_DCI_FORMAT0:
      return format0_size(cell, c);
    case SRSRAN_DCI_FORMAT1A:
      return format1A_size(cell, c);
    case SRSRAN_DCI_FORMAT1: {
      uint32_t n = rbg_bits(cell->nof_prb) + 5 + pid_len(cell) + 1 + 2 + 2 + (c->cif_enabled ? 3 : 0) + dai_len(cell) +
                   (cell->nof_prb > 10 ? 1 : 0);
      while (n == format0_size(cell, c) || n == format1A_size(cell, c) || is_ambiguous_size(n)) {
        n++;
      }
      return n;
    }
    case SRSRAN_DCI_FORMAT1C:
      return format1C_size(cell);
    case SRSRAN_DCI_FORMAT2:
    case SRSRAN_DCI_FORMAT2A:
    case SRSRAN_DCI_FORMAT2B:
      return format2x_size(cell, c, format);
    default:
      return 0;
  }
}

int srsran_dci_msg_unpack_pusch(srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* cfg,
                                srsran_dci_msg_t* msg, srsran_dci_ul_t* dci)
{
  (void)sf;
  if (!cell || !msg || !dci) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  memset(dci, 0, sizeof(*dci));
  dci->rnti     = msg->rnti;
  dci->location = msg->location;
  dci->format   = msg->format;
  srsran_dci_cfg_t zero;
  memset(&zero, 0, sizeof(zero));
  return unpack_format0(cell, sf, cfg ? cfg : &zero, msg, dci);
}

int srsran_dci_msg_unpack_pdsch(srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* cfg,
                                srsran_dci_msg_t* msg, srsran_dci_dl_t* dci)
{
  if (!cell || !msg || !dci) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  memset(dci, 0, sizeof(*dci));
  for (int i = 1; i < SRSRAN_MAX_CODEWORDS; i++) {
    tb_disable(dci->tb[i]);
  }
  dci->rnti     = msg->rnti;
  dci->location = msg->location;
  dci->format   = msg->format;
  srsran_dci_cfg_t zero;
  memset(&zero, 0, sizeof(zero));
  if (!cfg) {
    cfg = &zero;
  }
  // dci.c:1317-1319
  dci->is_dwpts = cell->frame_type == SRSRAN_TDD && sf && srsran_sfidx_tdd_type(sf->tdd_config, sf->tti % 10) == SRSRAN_TDD_SF_S;
  switch (msg->format) {
    case SRSRAN_DCI_FORMAT1:
      return unpack_format1(cell, sf, cfg, msg, dci);
    case SRSRAN_DCI_FORMAT1A:
      return unpack_format1A(cell, cfg, msg, dci);
    case SRSRAN_DCI_FORMAT1C:
      return unpack_format1C(cell, sf, cfg, msg, dci);
    case SRSRAN_DCI_FORMAT2:
    case SRSRAN_DCI_FORMAT2A:
    case SRSRAN_DCI_FORMAT2B:
      return unpack_format2x(cell, cfg, msg, dci);
    default:
      fprintf(stderr, "[srsran_dci] unpacking of DCI format %d is not provided\n", (int)msg->format);
      return SRSRAN_ERROR;
  }
}

int srsran_dci_msg_pack_pdsch(srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* cfg, srsran_dci_dl_t* dci,
                              srsran_dci_msg_t* msg)
{
  if (!cell || !dci || !msg) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  msg->rnti     = dci->rnti;
  msg->location = dci->location;
  msg->format   = dci->format;
  srsran_dci_cfg_t zero;
  memset(&zero, 0, sizeof(zero));
  if (!cfg) {
    cfg = &zero;
  }
  switch (msg->format) {
    case SRSRAN_DCI_FORMAT1:
      return pack_format1(cell, sf, cfg, dci, msg);
    case SRSRAN_DCI_FORMAT1A:
      return pack_format1A(cell, sf, cfg, dci, msg);
    case SRSRAN_DCI_FORMAT1C:
      return pack_format1C(cell, dci, msg);
    case SRSRAN_DCI_FORMAT2:
    case SRSRAN_DCI_FORMAT2A:
    case SRSRAN_DCI_FORMAT2B:
      return pack_format2x(cell, sf, cfg, dci, msg);
    default:
      fprintf(stderr, "[srsran_dci] packing of DCI format %d is not provided\n", (int)msg->format);
      return SRSRAN_ERROR;
  }
}

int srsran_dci_msg_pack_pusch(srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* cfg, srsran_dci_ul_t* dci,
                              srsran_dci_msg_t* msg)
{
  if (!cell || !dci || !msg) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  msg->rnti     = dci->rnti;
  msg->location = dci->location;
  msg->format   = dci->format;
  srsran_dci_cfg_t zero;
  memset(&zero, 0, sizeof(zero));
  return pack_format0(cell, sf, cfg ? cfg : &zero, dci, msg);
}

bool srsran_dci_location_isvalid(srsran_dci_location_t* c)
{
  return c && c->L <= 3 && c->ncce <= 87;
}

int srsran_dci_location_set(srsran_dci_location_t* c, uint32_t L, uint32_t nCCE)
{
  if (L <= 3 && nCCE <= 87) {
    c->L    = L;
    c->ncce = nCCE;
    return SRSRAN_SUCCESS;
  }
  return SRSRAN_ERROR;
}

void srsran_dci_cfg_set_common_ss(srsran_dci_cfg_t* cfg)
{
  cfg->is_not_ue_ss = true;
}

bool srsran_location_find_location(const srsran_dci_location_t* locations, uint32_t nof_locations,
                                   const srsran_dci_location_t* location)
{
  for (uint32_t i = 0; i < nof_locations; i++) {
    if (locations[i].L == location->L && locations[i].ncce == location->ncce) {
      return true;
    }
  }
  return false;
}

uint32_t srsran_ra_dl_grant_nof_re(const srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_pdsch_grant_t* grant)
{
  uint32_t n = 0;
  for (uint32_t s = 0; s < 2; s++) {
    for (uint32_t j = 0; j < cell->nof_prb; j++) {
      if (grant->prb_idx[s][j]) {
        n += ra_re_x_prb(cell, sf, s, j);
      }
    }
  }
  return n;
}

int srsran_ra_dl_dci_to_grant(const srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_tm_t tm,
                              bool pdsch_use_tbs_index_alt, const srsran_dci_dl_t* dci, srsran_pdsch_grant_t* grant)
{
  if (!cell || !sf || !dci || !grant) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (sf->sf_type != SRSRAN_SF_NORM) {
    fprintf(stderr, "[srsran_ra] PDSCH grants of normal subframes only (MBSFN subframes carry the PMCH)\n");
    return SRSRAN_ERROR;
  }
  if (cell->frame_type == SRSRAN_TDD && srsran_sfidx_tdd_type(sf->tdd_config, sf->tti % 10) == SRSRAN_TDD_SF_U) {
    fprintf(stderr, "[srsran_ra] subframe %u is an uplink subframe of TDD configuration %u\n", sf->tti % 10,
            sf->tdd_config.sf_config);
    return SRSRAN_ERROR;
  }
  memset(grant, 0, sizeof(*grant));
  if (prb_allocation(dci, grant, cell->nof_prb) || compute_tb(pdsch_use_tbs_index_alt, dci, grant)) {
    return SRSRAN_ERROR;
  }
  grant->nof_re = srsran_ra_dl_grant_nof_re(cell, sf, grant);
  // ra_dl.c:428-440: a TDD special subframe carries the PDSCH in its DwPTS symbols only
  const bool special = cell->frame_type == SRSRAN_TDD &&
                       srsran_sfidx_tdd_type(sf->tdd_config, sf->tti % 10) == SRSRAN_TDD_SF_S;
  grant->nof_symb_slot[0] = special ? srsran_sfidx_tdd_nof_dw_slot(sf->tdd_config, 0, cell->cp) : SRSRAN_CP_NSYMB(cell->cp);
  grant->nof_symb_slot[1] = special ? srsran_sfidx_tdd_nof_dw_slot(sf->tdd_config, 1, cell->cp) : SRSRAN_CP_NSYMB(cell->cp);
  for (int i = 0; i < SRSRAN_MAX_CODEWORDS; i++) {
    if (grant->tb[i].enabled) {
      grant->tb[i].nof_bits = grant->nof_re * srsran_mod_bits_x_symbol(grant->tb[i].mod);
    }
  }
  return config_mimo(cell, tm, dci, grant);
}

}  // extern "C"
