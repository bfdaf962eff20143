/*
 * oracle/ref_enb_ctrl_harness.c -- TEST INFRASTRUCTURE ONLY (linked into oracle/_ref/libsrsref.so).
 *
 * The eNB control channels of one subframe as srsran_enb_dl_put_base + srsran_enb_dl_put_pdcch_dl do them
 * (enb_dl.c:333-420), built from the reference's own code compiled from /root/reference:
 *   PSS / SSS    sync/gen_sss.c srsran_sss_generate; pss.c's srsran_pss_generate / _put_slot and sss.c's
 *                srsran_sss_put_slot are restated (pss.c / sss.c pull in the DFT and cannot be linked
 *                without FFTW): pss.c:341-379, sss.c:105-119
 *   PBCH         fec/crc.c, convolutional/convcoder.c, turbo/rm_conv.c, phch/sequences.c srsran_sequence_pbch,
 *                scrambling/scrambling.c, modem/mod.c, mimo/layermap.c + precoding.c, phch/prb_dl.c
 *                prb_cp_ref / prb_cp; the orchestration of pbch.c srsran_pbch_encode, srsran_pbch_mib_pack,
 *                srsran_pbch_cp and the CRC mask table are restated (pbch.c includes the CMake-generated
 *                srsran/version.h through srsran/srsran.h)
 *   PCFICH       phch/pcfich.c srsran_pcfich_encode
 *   PDCCH        phch/pdcch.c srsran_pdcch_encode (one call per message, in order)
 * as the checker of the GPU control transmitter (tests/test_enb_ctrl_gpu.py).
 */
#include <complex.h>
#include <math.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "prb_dl.h" /* $(REF)/src/phy/phch */
#include "srsran/phy/common/phy_common.h"
#include "srsran/phy/common/sequence.h"
#include "srsran/phy/fec/convolutional/convcoder.h"
#include "srsran/phy/fec/convolutional/rm_conv.h"
#include "srsran/phy/fec/crc.h"
#include "srsran/phy/mimo/layermap.h"
#include "srsran/phy/mimo/precoding.h"
#include "srsran/phy/modem/mod.h"
#include "srsran/phy/phch/pcfich.h"
#include "srsran/phy/phch/pdcch.h"
#include "srsran/phy/phch/regs.h"
#include "srsran/phy/scrambling/scrambling.h"
#include "srsran/phy/sync/sss.h"

int srsran_sequence_pbch(srsran_sequence_t* seq, srsran_cp_t cp, uint32_t cell_id); /* phch/sequences.c */

static srsran_cell_t enb_cell(uint32_t nof_prb, uint32_t nof_ports, uint32_t id, int cp, int phich_len, int phich_res)
{
  srsran_cell_t c;
  memset(&c, 0, sizeof(c));
  c.nof_prb         = nof_prb;
  c.nof_ports       = nof_ports;
  c.id              = id;
  c.cp              = cp ? SRSRAN_CP_EXT : SRSRAN_CP_NORM;
  c.phich_length    = (srsran_phich_length_t)phich_len;
  c.phich_resources = (srsran_phich_r_t)phich_res;
  c.frame_type      = SRSRAN_FDD;
  return c;
}

/* pss.c:341-370 */
static void pss_generate(cf_t* signal, uint32_t N_id_2)
{
  const float root_value[] = {25.0, 29.0, 34.0};
  int         sign         = -1;
  for (int i = 0; i < 31; i++) {
    float arg = (float)sign * M_PI * root_value[N_id_2] * ((float)i * ((float)i + 1.0)) / 63.0;
    signal[i] = cosf(arg) + I * sinf(arg);
  }
  for (int i = 31; i < 62; i++) {
    float arg = (float)sign * M_PI * root_value[N_id_2] * (((float)i + 2.0) * ((float)i + 1.0)) / 63.0;
    signal[i] = cosf(arg) + I * sinf(arg);
  }
}

/* srsran_pbch_mib_pack (pbch.c) */
static void mib_pack(const srsran_cell_t* cell, uint32_t sfn, uint8_t* msg)
{
  int bw = cell->nof_prb <= 6 ? 0 : cell->nof_prb <= 15 ? 1 : 1 + (int)cell->nof_prb / 25;
  int res = 0;
  switch (cell->phich_resources) {
    case SRSRAN_PHICH_R_1_6:
      res = 0;
      break;
    case SRSRAN_PHICH_R_1_2:
      res = 1;
      break;
    case SRSRAN_PHICH_R_1:
      res = 2;
      break;
    case SRSRAN_PHICH_R_2:
      res = 3;
      break;
  }
  memset(msg, 0, 24);
  for (int i = 0; i < 3; i++) {
    msg[i] = (bw >> (2 - i)) & 1;
  }
  msg[3] = cell->phich_length == SRSRAN_PHICH_EXT;
  for (int i = 0; i < 2; i++) {
    msg[4 + i] = (res >> (1 - i)) & 1;
  }
  for (int i = 0; i < 8; i++) {
    msg[6 + i] = ((sfn >> 2) >> (7 - i)) & 1;
  }
}

/* srsran_pbch_cp with put (pbch.c), on the reference's prb_cp_ref / prb_cp (prb_dl.c) */
static void pbch_put(cf_t* input, cf_t* output, srsran_cell_t cell)
{
  output += cell.nof_prb * SRSRAN_NRE / 2 - 36;
  for (int i = 0; i < 2; i++) {
    prb_cp_ref(&input, &output, cell.id % 3, 4, 4 * 6, true);
    output += cell.nof_prb * SRSRAN_NRE - 2 * 36 + (cell.id % 3 == 2 ? 1 : 0);
  }
  if (SRSRAN_CP_ISNORM(cell.cp)) {
    for (int i = 0; i < 2; i++) {
      prb_cp(&input, &output, 6);
      output += cell.nof_prb * SRSRAN_NRE - 2 * 36;
    }
  } else {
    prb_cp(&input, &output, 6);
    output += cell.nof_prb * SRSRAN_NRE - 2 * 36;
    prb_cp_ref(&input, &output, cell.id % 3, 4, 4 * 6, true);
  }
}

/* srsran_pbch_encode (pbch.c) of the MIB of sfn */
static int pbch_encode(srsran_cell_t cell, uint32_t sfn, cf_t* sf_symbols[SRSRAN_MAX_PORTS])
{
  static const uint8_t crc_mask[4][16] = {{0}, {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1}, {0},
                                          {0, 1, 0, 1, 0, 1, 0, 1, 0, 1, 0, 1, 0, 1, 0, 1}};
  const uint32_t       nsym          = SRSRAN_CP_ISNORM(cell.cp) ? 240 : 216, nbits = 2 * nsym;
  uint8_t              data[40], coded[120], rm[4 * 480];
  cf_t                 d[240], x[4][240], y[4][240];
  mib_pack(&cell, sfn, data);
  srsran_crc_t crc;
  if (srsran_crc_init(&crc, SRSRAN_LTE_CRC16, 16)) {
    return -1;
  }
  srsran_crc_attach(&crc, data, 24);
  for (int i = 0; i < 16; i++) {
    data[24 + i] = (data[24 + i] + crc_mask[cell.nof_ports - 1][i]) % 2;
  }
  srsran_convcoder_t enc;
  enc.R           = 3;
  enc.K           = 7;
  enc.poly[0]     = 0x6D;
  enc.poly[1]     = 0x4F;
  enc.poly[2]     = 0x57;
  enc.tail_biting = true;
  srsran_convcoder_encode(&enc, data, coded, 40);
  srsran_rm_conv_tx(coded, 120, rm, 4 * nbits);
  srsran_sequence_t seq;
  memset(&seq, 0, sizeof(seq));
  if (srsran_sequence_pbch(&seq, cell.cp, cell.id)) {
    return -1;
  }
  const uint32_t f = sfn % 4;
  srsran_scrambling_b_offset(&seq, &rm[f * nbits], f * nbits, nbits);
  srsran_modem_table_t mod;
  srsran_modem_table_lte(&mod, SRSRAN_MOD_QPSK);
  srsran_mod_modulate(&mod, &rm[f * nbits], d, nbits);
  cf_t* xp[SRSRAN_MAX_LAYERS] = {x[0], x[1], x[2], x[3]};
  cf_t* yp[SRSRAN_MAX_PORTS]  = {y[0], y[1], y[2], y[3]};
  if (cell.nof_ports > 1) {
    srsran_layermap_diversity(d, xp, cell.nof_ports, nsym);
    srsran_precoding_diversity(xp, yp, cell.nof_ports, nsym / cell.nof_ports, 1.0f);
  } else {
    memcpy(y[0], d, nsym * sizeof(cf_t));
  }
  for (uint32_t p = 0; p < cell.nof_ports; p++) {
    pbch_put(y[p], &sf_symbols[p][SRSRAN_SLOT_LEN_RE(cell.nof_prb, cell.cp)], cell);
  }
  srsran_sequence_free(&seq);
  srsran_modem_table_free(&mod);
  return 0;
}

/* put_sync, put_mib and put_pcfich of srsran_enb_dl_put_base (no CRS) when put_base, then srsran_pdcch_encode
 * of each message in order, into nof_ports grids of 14 * 12 * nof_prb cf_t (interleaved re / im). */
int ref_enb_ctrl_tx(uint32_t nof_prb, uint32_t nof_ports, uint32_t id, int cp, int phich_len, int phich_res,
                    uint32_t tti, uint32_t cfi, int put_base, uint32_t ndci, const uint8_t* payloads,
                    const uint32_t* nof_bits, const uint32_t* L, const uint32_t* ncce, const uint16_t* rnti,
                    float* grids)
{
  srsran_cell_t   cell = enb_cell(nof_prb, nof_ports, id, cp, phich_len, phich_res);
  srsran_regs_t   regs;
  srsran_pcfich_t pcfich;
  srsran_pdcch_t  pdcch;
  if (srsran_regs_init(&regs, cell) || srsran_pcfich_init(&pcfich, 0) || srsran_pcfich_set_cell(&pcfich, &regs, cell) ||
      srsran_pdcch_init_enb(&pdcch, nof_prb) || srsran_pdcch_set_cell(&pdcch, &regs, cell)) {
    return -1;
  }
  cf_t* sym[SRSRAN_MAX_PORTS] = {NULL};
  for (uint32_t p = 0; p < nof_ports; p++) {
    sym[p] = (cf_t*)grids + (size_t)p * 14 * 12 * nof_prb;
  }
  srsran_dl_sf_cfg_t sf;
  memset(&sf, 0, sizeof(sf));
  sf.tti            = tti;
  sf.cfi            = cfi;
  const uint32_t si = tti % 10;
  int            ret = 0;
  if (put_base) {
    if (si == 0 || si == 5) {
      cf_t  pss[62];
      float sss0[62], sss5[62];
      pss_generate(pss, id % 3);
      srsran_sss_generate(sss0, sss5, id);
      const float* sss = si ? sss5 : sss0;
      for (uint32_t p = 0; p < nof_ports; p++) {
        const uint32_t nre = nof_prb * SRSRAN_NRE;
        uint32_t       k   = (SRSRAN_CP_NSYMB(cell.cp) - 1) * nre + nre / 2 - 31;
        memset(&sym[p][k - 5], 0, 5 * sizeof(cf_t));
        memcpy(&sym[p][k], pss, 62 * sizeof(cf_t));
        memset(&sym[p][k + 62], 0, 5 * sizeof(cf_t));
        k = (SRSRAN_CP_NSYMB(cell.cp) - 2) * nre + nre / 2 - 31;
        memset(&sym[p][k - 5], 0, 5 * sizeof(cf_t));
        for (int i = 0; i < 62; i++) {
          sym[p][k + i] = sss[i];
        }
        memset(&sym[p][k + 62], 0, 5 * sizeof(cf_t));
      }
    }
    if (si == 0) {
      ret = pbch_encode(cell, tti / 10, sym);
    }
    if (ret == 0) {
      ret = srsran_pcfich_encode(&pcfich, &sf, sym);
    }
  }
  for (uint32_t d = 0; d < ndci && ret == 0; d++) {
    srsran_dci_msg_t msg;
    memset(&msg, 0, sizeof(msg));
    memcpy(msg.payload, payloads + d * SRSRAN_DCI_MAX_BITS, nof_bits[d]);
    msg.nof_bits      = nof_bits[d];
    msg.location.L    = L[d];
    msg.location.ncce = ncce[d];
    msg.rnti          = rnti[d];
    ret               = srsran_pdcch_encode(&pdcch, &sf, &msg, sym);
  }
  srsran_pdcch_free(&pdcch);
  srsran_pcfich_free(&pcfich);
  srsran_regs_free(&regs);
  return ret;
}
