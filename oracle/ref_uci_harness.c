/*
 * oracle/ref_uci_harness.c -- TEST INFRASTRUCTURE ONLY (linked into oracle/_ref/libsrsref.so).
 *
 * Drives the reference's own UCI-on-PUSCH code, compiled from /root/reference:
 *   phch/uci.c (srsran_uci_encode_ack_ri / srsran_uci_decode_ack_ri, srsran_uci_encode_cqi_pusch /
 *   srsran_uci_decode_cqi_pusch, Q' formulas), fec/block/block.c, and the convolutional / rate
 *   matching / CRC sources already in the library,
 * as the checker of srsran_ulsch_decode with UCI (tests/test_uci_*.py).
 *
 * phch/sch.c and phch/cqi.c include the CMake-generated srsran/srsran.h and are not buildable
 * here, so the UL-SCH orchestration around uci.c is restated below, step for step:
 *   ref_ulsch_uci_rx  sch.c:994-1021 (de-interleaver with RI, srsran_vec_lut_sis), sch.c:1023-1120
 *                     (uci_decode_ri_ack), sch.c:1122-1183 (srsran_ulsch_decode up to decode_tb)
 *   ref_ulsch_uci_tx  sch.c:1195-1337 (srsran_ulsch_encode with the TB's e bits given, on unpacked
 *                     bits) and the placeholder / repetition marking of pusch.c:315-331
 *   cqi sizes / packing from cqi.c:41-384.
 */
#include <math.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "srsran/phy/fec/block/block.h"
#include "srsran/phy/fec/cbsegm.h"
#include "srsran/phy/phch/cqi.h"
#include "srsran/phy/phch/pusch_cfg.h"
#include "srsran/phy/phch/uci.h"

/* ---------------- cqi.c restatement ---------------- */
static uint32_t hl_pmi_bits(const srsran_cqi_cfg_t* c)
{
  return c->four_antenna_ports ? 4 : (c->rank_is_not_one ? 1 : 2);
}

int ref_cqi_size(srsran_cqi_cfg_t* c)
{
  if (!c->data_enable) {
    return (int)c->ri_len;
  }
  switch (c->type) {
    case SRSRAN_CQI_TYPE_WIDEBAND:
      if (!c->pmi_present) {
        return 4;
      }
      return 4 + (c->rank_is_not_one ? 3 : 0) + (c->four_antenna_ports ? 4 : (c->rank_is_not_one ? 1 : 2));
    case SRSRAN_CQI_TYPE_SUBBAND_UE:
      return c->subband_label_2_bits ? 6 : 5;
    case SRSRAN_CQI_TYPE_SUBBAND_UE_DIFF:
      return 6 + (int)c->L;
    case SRSRAN_CQI_TYPE_SUBBAND_HL:
      return (int)((4 + 2 * c->N) * ((c->rank_is_not_one && c->pmi_present) ? 2 : 1) +
                   (c->pmi_present ? hl_pmi_bits(c) : 0));
  }
  return -1;
}

/* field list of a report: (value pointer, width) in transmission order */
typedef struct {
  uint32_t* v[8];
  uint32_t  w[8];
  int       n;
} fields_t;

static void add(fields_t* f, uint32_t* v, uint32_t w)
{
  f->v[f->n] = v;
  f->w[f->n] = w;
  f->n++;
}

/* the report's fields as 32-bit scratch values t[] (copied from / to the union by the callers) */
static void cqi_fields(const srsran_cqi_cfg_t* c, uint32_t* t, fields_t* f)
{
  f->n = 0;
  switch (c->type) {
    case SRSRAN_CQI_TYPE_WIDEBAND: /* t: wideband, spatial diff, pmi */
      add(f, &t[0], 4);
      if (c->pmi_present) {
        if (c->rank_is_not_one) {
          add(f, &t[1], 3);
        }
        add(f, &t[2], c->four_antenna_ports ? 4 : (c->rank_is_not_one ? 1 : 2));
      }
      break;
    case SRSRAN_CQI_TYPE_SUBBAND_UE: /* t: subband cqi, label */
      add(f, &t[0], 4);
      add(f, &t[1], c->subband_label_2_bits ? 2 : 1);
      break;
    case SRSRAN_CQI_TYPE_SUBBAND_UE_DIFF: /* t: wideband, diff (written twice: cqi.c:77-85) */
      add(f, &t[0], 4);
      add(f, &t[1], 2);
      add(f, &t[1], c->L);
      break;
    case SRSRAN_CQI_TYPE_SUBBAND_HL: /* t: wb0, sb0, wb1, sb1, pmi */
      add(f, &t[0], 4);
      add(f, &t[1], 2 * c->N);
      if (c->rank_is_not_one) {
        add(f, &t[2], 4);
        add(f, &t[3], 2 * c->N);
      }
      if (c->pmi_present) {
        add(f, &t[4], hl_pmi_bits(c));
      }
      break;
  }
}

static void value_to_t(const srsran_cqi_cfg_t* c, const srsran_cqi_value_t* v, uint32_t* t)
{
  memset(t, 0, 5 * sizeof(uint32_t));
  switch (c->type) {
    case SRSRAN_CQI_TYPE_WIDEBAND:
      t[0] = v->wideband.wideband_cqi, t[1] = v->wideband.spatial_diff_cqi, t[2] = v->wideband.pmi;
      break;
    case SRSRAN_CQI_TYPE_SUBBAND_UE:
      t[0] = v->subband_ue.subband_cqi, t[1] = v->subband_ue.subband_label;
      break;
    case SRSRAN_CQI_TYPE_SUBBAND_UE_DIFF:
      t[0] = v->subband_ue_diff.wideband_cqi, t[1] = v->subband_ue_diff.subband_diff_cqi;
      break;
    case SRSRAN_CQI_TYPE_SUBBAND_HL:
      t[0] = v->subband_hl.wideband_cqi_cw0, t[1] = v->subband_hl.subband_diff_cqi_cw0;
      t[2] = v->subband_hl.wideband_cqi_cw1, t[3] = v->subband_hl.subband_diff_cqi_cw1;
      t[4] = v->subband_hl.pmi;
      break;
  }
}

int ref_cqi_pack(srsran_cqi_cfg_t* c, srsran_cqi_value_t* v, uint8_t* buff)
{
  uint32_t t[5];
  fields_t f;
  value_to_t(c, v, t);
  cqi_fields(c, t, &f);
  int n = 0;
  for (int i = 0; i < f.n; i++) {
    for (uint32_t b = 0; b < f.w[i]; b++) {
      buff[n++] = (uint8_t)((*f.v[i] >> (f.w[i] - 1 - b)) & 1u);
    }
  }
  return n;
}

/* unpack into the union fields the reference writes (untouched fields keep their value) */
int ref_cqi_unpack(srsran_cqi_cfg_t* c, const uint8_t* buff, srsran_cqi_value_t* v)
{
  uint32_t t[5];
  fields_t f;
  value_to_t(c, v, t);
  cqi_fields(c, t, &f);
  int n = 0;
  for (int i = 0; i < f.n; i++) {
    uint32_t x = 0;
    for (uint32_t b = 0; b < f.w[i]; b++) {
      x = (x << 1) | (buff[n++] & 1u);
    }
    *f.v[i] = x;
  }
  switch (c->type) {
    case SRSRAN_CQI_TYPE_WIDEBAND:
      v->wideband.wideband_cqi = (uint8_t)t[0];
      if (c->pmi_present) {
        if (c->rank_is_not_one) {
          v->wideband.spatial_diff_cqi = (uint8_t)t[1];
        }
        v->wideband.pmi = (uint8_t)t[2];
      }
      break;
    case SRSRAN_CQI_TYPE_SUBBAND_UE:
      v->subband_ue.subband_cqi = (uint8_t)t[0], v->subband_ue.subband_label = (uint8_t)t[1];
      break;
    case SRSRAN_CQI_TYPE_SUBBAND_UE_DIFF:
      v->subband_ue_diff.wideband_cqi = (uint8_t)t[0], v->subband_ue_diff.subband_diff_cqi = (uint8_t)t[1];
      break;
    case SRSRAN_CQI_TYPE_SUBBAND_HL:
      v->subband_hl.wideband_cqi_cw0 = (uint8_t)t[0], v->subband_hl.subband_diff_cqi_cw0 = t[1];
      if (c->rank_is_not_one) {
        v->subband_hl.wideband_cqi_cw1 = (uint8_t)t[2], v->subband_hl.subband_diff_cqi_cw1 = t[3];
      }
      if (c->pmi_present) {
        v->subband_hl.pmi = (uint8_t)t[4];
      }
      break;
  }
  return n;
}

/* ---------------- sch.c restatement ---------------- */
static float beta_harq(uint32_t i)
{
  const float t[16] = {2.0, 2.5, 3.125, 4.0, 5.0, 6.250, 8.0, 10.0, 12.625, 15.875, 20.0, 31.0, 50.0, 80.0, 126.0, -1.0};
  return i < 15 ? t[i] : t[0];
}
static float beta_ri(uint32_t i)
{
  const float t[16] = {1.25, 1.625, 2.0, 2.5, 3.125, 4.0, 5.0, 6.25, 8.0, 10.0, 12.625, 15.875, 20.0, -1.0, -1.0, -1.0};
  return i < 13 ? t[i] : t[0];
}
static float beta_cqi(uint32_t i)
{
  const float t[16] = {-1.0, -1.0, 1.125, 1.25, 1.375, 1.625, 1.750, 2.0, 2.25, 2.5, 2.875, 3.125, 3.5, 4.0, 5.0, 6.25};
  return (i > 1 && i < 16) ? t[i] : t[2];
}

static srsran_uci_cqi_pusch_t g_cqi;
static bool                   g_cqi_ready;
static srsran_uci_bit_t       g_bits[2 * 4 * 1200 * 8 + 64]; /* RI then ACK, 4 M_sc Qm each */

static srsran_uci_bit_t* g_bits_tab(void) { return g_bits; }

/* get_beta_cqi_offset through srsran_sch_beta_cqi (sch.c:88-96) */
static float srsran_sch_beta_cqi_ref(uint32_t i) { return i < 16 ? beta_cqi(i) : 0.0f; }

static srsran_uci_cqi_pusch_t* cqi_obj(void)
{
  if (!g_cqi_ready) {
    srsran_uci_cqi_init(&g_cqi);
    g_cqi_ready = true;
  }
  return &g_cqi;
}

uint32_t ref_sizeof_pusch_cfg(void) { return (uint32_t)sizeof(srsran_pusch_cfg_t); }
uint32_t ref_sizeof_uci_value(void) { return (uint32_t)sizeof(srsran_uci_value_t); }

static uint32_t qm_of(const srsran_pusch_cfg_t* cfg) { return srsran_mod_bits_x_symbol(cfg->grant.tb.mod); }

static uint32_t cbsegm_K(uint32_t tbs)
{
  srsran_cbsegm_t s;
  if (srsran_cbsegm(&s, tbs)) {
    return 0;
  }
  return s.C1 * s.K1 + s.C2 * s.K2;
}

/* out[0..3] = Q'_RI, Q'_CQI, G (the TB's LLRs are G Qm from g_bits[Q'_CQI Qm]), Q'_ACK;
 * returns what srsran_ulsch_decode would hold in ret before decode_tb (< 0: error) */
int ref_ulsch_uci_rx(srsran_pusch_cfg_t* cfg,
                     int16_t*            q_bits,
                     int16_t*            g_bits,
                     uint8_t*            c_seq,
                     srsran_uci_value_t* uci,
                     uint32_t*           out)
{
  const uint32_t nb_q = cfg->grant.tb.nof_bits, Qm = qm_of(cfg);
  cfg->K_segm         = cbsegm_K((uint32_t)cfg->grant.tb.tbs);
  const uint32_t nack = srsran_uci_cfg_total_ack(&cfg->uci_cfg);
  srsran_cqi_cfg_t* cq = &cfg->uci_cfg.cqi;
  const bool        hl = cq->data_enable && cq->type == SRSRAN_CQI_TYPE_SUBBAND_HL && cq->ri_len;

  /* uci_decode_ri_ack (sch.c:1023-1120) */
  if (hl) {
    cq->rank_is_not_one = false;
  }
  uint32_t cqi_len = (uint32_t)ref_cqi_size(cq);
  uint32_t Qp_ack = 0, Qp_ri = 0;
  int      ret    = 0;
  if (nack > 0) {
    float beta = beta_harq(cfg->uci_offset.I_offset_ack);
    if (cfg->grant.tb.tbs == 0) {
      beta /= beta_cqi(cfg->uci_offset.I_offset_cqi);
    }
    ret = srsran_uci_decode_ack_ri(cfg, q_bits, c_seq, beta, nb_q / Qm, cqi_len, g_bits_tab(), uci->ack.ack_value,
                                   &uci->ack.valid, nack, false);
    if (ret < 0) {
      return ret;
    }
    Qp_ack = (uint32_t)ret;
    for (uint32_t i = 0; i < Qp_ack * Qm; i++) {
      q_bits[g_bits_tab()[i].position] = 0;
    }
  }
  if (cq->ri_len > 0) {
    float beta = beta_ri(cfg->uci_offset.I_offset_ri);
    if (cfg->grant.tb.tbs == 0) {
      beta /= beta_cqi(cfg->uci_offset.I_offset_cqi);
    }
    ret = srsran_uci_decode_ack_ri(cfg, q_bits, c_seq, beta, nb_q / Qm, cqi_len, g_bits_tab(), &uci->ri, NULL,
                                   cq->ri_len, true);
    if (ret < 0) {
      return ret;
    }
    Qp_ri = (uint32_t)ret;
  } else {
    ret = 0;
  }
  if (cq->data_enable && cq->type == SRSRAN_CQI_TYPE_SUBBAND_HL && cq->ri_len) {
    cq->rank_is_not_one = uci->ri > 0;
  }
  ret = (int)Qp_ri;

  /* ulsch_deinterleave (sch.c:661-682, 994-1021) */
  const uint32_t H = nb_q / Qm, rows = H / cfg->grant.nof_symb, cols = cfg->grant.nof_symb;
  uint8_t*       ri_present = calloc(H * Qm, 1);
  uint32_t*      lut        = malloc(sizeof(uint32_t) * H * Qm);
  for (uint32_t i = 0; i < Qp_ri * Qm; i++) {
    ri_present[g_bits_tab()[i].position] = 1;
  }
  uint32_t idx = 0;
  for (uint32_t j = 0; j < rows; j++) {
    for (uint32_t i = 0; i < cols; i++) {
      for (uint32_t k = 0; k < Qm; k++) {
        const uint32_t p = j * Qm + i * rows * Qm + k;
        if (ri_present[p]) {
          lut[p] = 0;
        } else {
          lut[p] = idx++;
        }
      }
    }
  }
  for (uint32_t i = 0; i < H * Qm; i++) { /* srsran_vec_lut_sis */
    g_bits[lut[i]] = q_bits[i];
  }
  free(ri_present);
  free(lut);

  /* CQI (sch.c:1160-1183) */
  uint32_t Qp_cqi = 0;
  if (cq->data_enable) {
    uint8_t cqi_buff[SRSRAN_CQI_MAX_BITS];
    memset(cqi_buff, 0, sizeof(cqi_buff));
    cqi_len = (uint32_t)ref_cqi_size(cq);
    ret     = srsran_uci_decode_cqi_pusch(cqi_obj(), cfg, g_bits, srsran_sch_beta_cqi_ref(cfg->uci_offset.I_offset_cqi),
                                      Qp_ri, cqi_len, cqi_buff, &uci->cqi.data_crc);
    if (ret < 0) {
      return ret;
    }
    ref_cqi_unpack(cq, cqi_buff, &uci->cqi);
    Qp_cqi = (uint32_t)ret;
  }
  out[0] = Qp_ri;
  out[1] = Qp_cqi;
  out[2] = H - Qp_ri - Qp_cqi;
  out[3] = Qp_ack;
  return ret;
}

/* srsran_ulsch_encode (sch.c:1195-1337) on unpacked bits with the TB's rate-matched e bits given
 * (G Qm of them, G = H' - Q'_RI - Q'_CQI: call once with e_data = NULL to learn G in out[2]).
 * q_types[p]: 0 / 1 = bit value, 2 = placeholder "x", 3 = repetition "y" (pusch.c:315-331). */
int ref_ulsch_uci_tx(srsran_pusch_cfg_t* cfg, srsran_uci_value_t* uci, const uint8_t* e_data, uint8_t* q_types,
                     uint32_t* out)
{
  const uint32_t nb_q = cfg->grant.tb.nof_bits, Qm = qm_of(cfg);
  cfg->K_segm         = cbsegm_K((uint32_t)cfg->grant.tb.tbs);
  srsran_cqi_cfg_t* cq = &cfg->uci_cfg.cqi;
  const uint32_t    H  = nb_q / Qm, rows = H / cfg->grant.nof_symb, cols = cfg->grant.nof_symb;
  uint8_t           cqi_buff[SRSRAN_CQI_MAX_BITS];
  memset(cqi_buff, 0, sizeof(cqi_buff));
  int cqi_len = 0;
  if (cq->data_enable) {
    cqi_len = ref_cqi_pack(cq, &uci->cqi, cqi_buff);
  }
  srsran_uci_bit_t* bits = g_bits_tab();
  uint32_t          Qp_ri = 0, Qp_cqi = 0, Qp_ack = 0;
  if (cq->ri_len > 0) {
    float beta = beta_ri(cfg->uci_offset.I_offset_ri);
    if (cfg->grant.tb.tbs == 0) {
      beta /= beta_cqi(cfg->uci_offset.I_offset_cqi);
    }
    uint8_t ri[2] = {uci->ri, 0};
    int     r = srsran_uci_encode_ack_ri(cfg, ri, cq->ri_len, (uint32_t)cqi_len, beta, H, true, 0, bits);
    if (r < 0) {
      return r;
    }
    Qp_ri = (uint32_t)r;
  }
  uint8_t* g = calloc(H * Qm, 1);
  if (cqi_len > 0) {
    int r = srsran_uci_encode_cqi_pusch(cqi_obj(), cfg, cqi_buff, (uint32_t)cqi_len,
                                        srsran_sch_beta_cqi_ref(cfg->uci_offset.I_offset_cqi), Qp_ri, g);
    if (r < 0) {
      free(g);
      return r;
    }
    Qp_cqi = (uint32_t)r;
  }
  const uint32_t G = H - Qp_ri - Qp_cqi;
  out[0]           = Qp_ri;
  out[1]           = Qp_cqi;
  out[2]           = G;
  if (!e_data) {
    free(g);
    return 0;
  }
  if (cfg->grant.tb.tbs > 0) {
    memcpy(g + Qp_cqi * Qm, e_data, G * Qm);
  }
  /* ulsch_interleave (sch.c:949-990 and the qm2/4/6 bodies): rows outer, columns inner, RI cells skipped */
  uint8_t* ri_present = calloc(H * Qm, 1);
  for (uint32_t i = 0; i < Qp_ri * Qm; i++) {
    ri_present[bits[i].position] = 1;
  }
  uint32_t rd = 0;
  for (uint32_t j = 0; j < rows; j++) {
    for (uint32_t i = 0; i < cols; i++) {
      const uint32_t k = (i * rows + j) * Qm;
      if (ri_present[k]) {
        continue;
      }
      for (uint32_t b = 0; b < Qm; b++) {
        q_types[k + b] = g[rd++];
      }
    }
  }
  free(ri_present);
  free(g);
  /* ACK (sch.c:1300-1318), then the RI / ACK bit types at their positions */
  const uint32_t nack = srsran_uci_cfg_total_ack(&cfg->uci_cfg);
  if (nack > 0) {
    float beta = beta_harq(cfg->uci_offset.I_offset_ack);
    if (cfg->grant.tb.tbs == 0) {
      beta /= beta_cqi(cfg->uci_offset.I_offset_cqi);
    }
    int r = srsran_uci_encode_ack_ri(cfg, uci->ack.ack_value, nack, (uint32_t)cqi_len, beta, H, false, 0,
                                     &bits[Qp_ri * Qm]);
    if (r < 0) {
      return r;
    }
    Qp_ack = (uint32_t)r;
  }
  out[3] = Qp_ack;
  for (uint32_t i = 0; i < (Qp_ack + Qp_ri) * Qm; i++) {
    const uint32_t p = bits[i].position;
    if (p < nb_q) {
      q_types[p] = bits[i].type == UCI_BIT_1           ? 1
                   : bits[i].type == UCI_BIT_PLACEHOLDER ? 2
                   : bits[i].type == UCI_BIT_REPETITION  ? 3
                                                         : 0;
    }
  }
  return 0;
}
