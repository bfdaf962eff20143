/*
 * oracle/ref_pdcch_harness.c -- TEST INFRASTRUCTURE ONLY (linked into oracle/_ref/libsrsref.so).
 *
 * Drives the reference's own control-channel code, compiled from /root/reference:
 *   phch/pcfich.c, phch/pdcch.c, phch/regs.c, fec/convolutional/viterbi*.c, convcoder.c,
 *   fec/turbo/rm_conv.c, modem/mod.c, scrambling/scrambling.c
 * as the checker of the GPU PCFICH / PDCCH path (tests/test_pdcch_*.py):
 *   - REG tables (srsran_regs_pcfich_get / srsran_regs_pdcch_get on an index-valued grid),
 *   - the eNB transmit side (srsran_pcfich_encode, srsran_pdcch_encode) to build test subframes,
 *   - the UE receive side (srsran_pcfich_decode, srsran_pdcch_extract_llr, srsran_pdcch_decode_msg,
 *     srsran_pdcch_msg_corr) on the same grids and channel estimates the GPU sees.
 *
 * phch/dci.c includes the CMake-generated srsran/srsran.h and is not buildable here; pdcch.c needs
 * three of its functions, restated below from dci.c:93-413 (format sizes, FDD), dci.c:1442-1449
 * (location validity) and dci.c:1482-1512 (format names).
 */
#include <math.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "srsran/phy/common/phy_common.h"
#include "srsran/phy/phch/dci.h"
#include "srsran/phy/phch/pcfich.h"
#include "srsran/phy/phch/pdcch.h"
#include "srsran/phy/phch/ra.h"
#include "srsran/phy/phch/regs.h"
#include "srsran/phy/utils/phy_logger.h"

/* ---------------- dci.c restatement (sizes only; FDD, no CIF unless cfg says so) ---------------- */
static uint32_t riv_nbits(uint32_t nof_prb)
{
  return (uint32_t)ceilf(log2f((float)nof_prb * ((float)nof_prb + 1) / 2));
}
static bool ambiguous(uint32_t n)
{
  static const uint32_t s[10] = {12, 14, 16, 20, 24, 26, 32, 40, 44, 56};
  for (int i = 0; i < 10; i++) {
    if (n == s[i]) {
      return true;
    }
  }
  return false;
}
static uint32_t type0_P(uint32_t nof_prb) /* ra.c:60-72 */
{
  return nof_prb <= 10 ? 1 : nof_prb <= 26 ? 2 : nof_prb <= 63 ? 3 : 4;
}
static uint32_t f0_(const srsran_cell_t* c, srsran_dci_cfg_t* g)
{
  return (g->cif_enabled ? 3 : 0) + 1 + 1 + riv_nbits(c->nof_prb) + 5 + 1 + 2 + 3 +
         ((g->multiple_csi_request_enabled && !g->is_not_ue_ss) ? 2 : 1) +
         ((g->srs_request_enabled && !g->is_not_ue_ss) ? 1 : 0) + 1;
}
static uint32_t f1A(const srsran_cell_t* c, srsran_dci_cfg_t* g)
{
  uint32_t n = (g->cif_enabled ? 3 : 0) + 1 + 1 + riv_nbits(c->nof_prb) + 5 + 3 + 1 + 2 + 2 + (g->srs_request_enabled ? 1 : 0);
  while (n < f0_(c, g)) {
    n++;
  }
  if (ambiguous(n)) {
    n++;
  }
  return n;
}
static uint32_t f0(const srsran_cell_t* c, srsran_dci_cfg_t* g)
{
  uint32_t n = f0_(c, g);
  while (n < f1A(c, g)) {
    n++;
  }
  return n;
}
static uint32_t rbg_bits(const srsran_cell_t* c) { return (uint32_t)ceilf((float)c->nof_prb / type0_P(c->nof_prb)); }
uint32_t srsran_dci_format_sizeof(const srsran_cell_t* cell, srsran_dl_sf_cfg_t* sf, srsran_dci_cfg_t* cfg,
                                  srsran_dci_format_t format)
{
  srsran_dci_cfg_t zero;
  memset(&zero, 0, sizeof(zero));
  srsran_dci_cfg_t* g = cfg ? cfg : &zero;
  uint32_t          n = 0;
  (void)sf;
  switch (format) {
    case SRSRAN_DCI_FORMAT0:
      return f0(cell, g);
    case SRSRAN_DCI_FORMAT1A:
      return f1A(cell, g);
    case SRSRAN_DCI_FORMAT1:
      n = rbg_bits(cell) + 5 + 3 + 1 + 2 + 2 + (g->cif_enabled ? 3 : 0) + (cell->nof_prb > 10 ? 1 : 0);
      while (n == f0(cell, g) || n == f1A(cell, g) || ambiguous(n)) {
        n++;
      }
      return n;
    case SRSRAN_DCI_FORMAT2:
    case SRSRAN_DCI_FORMAT2A:
      n = rbg_bits(cell) + 2 + 3 + 1 + 2 * (5 + 1 + 2) + (g->cif_enabled ? 3 : 0) + (cell->nof_prb > 10 ? 1 : 0) +
          (format == SRSRAN_DCI_FORMAT2 ? (cell->nof_ports <= 2 ? 3 : 6) : (cell->nof_ports <= 2 ? 0 : 2));
      while (ambiguous(n)) {
        n++;
      }
      return n;
    default:
      return 0;
  }
}
bool srsran_dci_location_isvalid(srsran_dci_location_t* c)
{
  return c->L <= 3 && c->ncce <= 87;
}
char* srsran_dci_format_string(srsran_dci_format_t format)
{
  (void)format;
  return "Format";
}

/* utils/phy_logger.c (also srsran.h-dependent) is where the INFO / DEBUG macros of pdcch.c and
 * regs.c end up when no handler is registered; this log sink prints errors and drops the rest. */
void srsran_phy_log_print(phy_logger_level_t log_level, const char* format, ...)
{
  if (log_level == LOG_LEVEL_ERROR_S) {
    fprintf(stderr, "[ref] error in the reference control-channel code\n");
  }
  (void)format;
}

/* ---------------- harness ---------------- */
/* cyclic prefix of the cells the harness builds from now on (0 normal, 1 extended) */
static srsran_cp_t g_cp = SRSRAN_CP_NORM;
void               ref_set_cp(int ext) { g_cp = ext ? SRSRAN_CP_EXT : SRSRAN_CP_NORM; }

static srsran_cell_t mkcell(uint32_t nof_prb, uint32_t nof_ports, uint32_t id, int phich_len, int phich_res)
{
  srsran_cell_t c;
  memset(&c, 0, sizeof(c));
  c.nof_prb         = nof_prb;
  c.nof_ports       = nof_ports;
  c.id              = id;
  c.cp              = g_cp;
  c.phich_length    = (srsran_phich_length_t)phich_len;
  c.phich_resources = (srsran_phich_r_t)phich_res;
  c.frame_type      = SRSRAN_FDD;
  return c;
}

/* Grid indices (l * 12 * nof_prb + k) of the PCFICH REs (16) and of the PDCCH REs for CFI 1..3
 * in srsran_regs_*_get order; nre[c] = number of PDCCH REs for CFI c + 1. */
int ref_regs_tables_opts(uint32_t nof_prb, uint32_t nof_ports, uint32_t id, int phich_len, int phich_res,
                         uint32_t phich_mi, int mbsfn_or_sf1_6_tdd, uint32_t* pcfich, uint32_t* pdcch, uint32_t max_re,
                         uint32_t* nre)
{
  srsran_cell_t cell = mkcell(nof_prb, nof_ports, id, phich_len, phich_res);
  srsran_regs_t regs;
  if (srsran_regs_init_opts(&regs, cell, phich_mi, mbsfn_or_sf1_6_tdd != 0)) {
    return -1;
  }
  const uint32_t n    = 14 * 12 * nof_prb;
  cf_t*          grid = malloc(n * sizeof(cf_t));
  cf_t*          out  = malloc(n * sizeof(cf_t));
  for (uint32_t i = 0; i < n; i++) {
    grid[i] = (float)i;
  }
  int k = srsran_regs_pcfich_get(&regs, grid, out);
  for (int i = 0; i < k; i++) {
    pcfich[i] = (uint32_t)crealf(out[i]);
  }
  for (uint32_t cfi = 1; cfi <= 3; cfi++) {
    int m = srsran_regs_pdcch_get(&regs, cfi, grid, out);
    if (m < 0 || (uint32_t)m > max_re) {
      return -1;
    }
    nre[cfi - 1] = (uint32_t)m;
    for (int i = 0; i < m; i++) {
      pdcch[(cfi - 1) * max_re + i] = (uint32_t)crealf(out[i]);
    }
  }
  free(grid);
  free(out);
  srsran_regs_free(&regs);
  return k;
}

int ref_regs_tables_mi(uint32_t nof_prb, uint32_t nof_ports, uint32_t id, int phich_len, int phich_res,
                       uint32_t phich_mi, uint32_t* pcfich, uint32_t* pdcch, uint32_t max_re, uint32_t* nre)
{
  return ref_regs_tables_opts(nof_prb, nof_ports, id, phich_len, phich_res, phich_mi, 0, pcfich, pdcch, max_re, nre);
}

/* srsran_regs_init's tables (PHICH m_i = 1) */
int ref_regs_tables(uint32_t nof_prb, uint32_t nof_ports, uint32_t id, int phich_len, int phich_res,
                    uint32_t* pcfich, uint32_t* pdcch, uint32_t max_re, uint32_t* nre)
{
  return ref_regs_tables_mi(nof_prb, nof_ports, id, phich_len, phich_res, 1, pcfich, pdcch, max_re, nre);
}

/* eNB control region: PCFICH with `cfi` and ndci PDCCH messages (payload bits, nof_bits, L (log2),
 * ncce, rnti each) added into nof_ports grids of 14 * 12 * nof_prb cf_t (interleaved re/im). */
/* The same on the REG tables of srsran_regs_init_opts(cell, phich_mi, mbsfn_or_sf1_6_tdd): the control region a
 * TDD eNB with that PHICH m_i (and, with the extended PHICH duration, subframe 1 / 6's two-symbol PHICH) transmits. */
int ref_ctrl_tx_opts(uint32_t nof_prb, uint32_t nof_ports, uint32_t id, int phich_len, int phich_res, uint32_t phich_mi,
                     int mbsfn_or_sf1_6_tdd, uint32_t tti, uint32_t cfi, uint32_t ndci, const uint8_t* payloads,
                     const uint32_t* nof_bits, const uint32_t* L, const uint32_t* ncce, const uint16_t* rnti, float* grids)
{
  srsran_cell_t   cell = mkcell(nof_prb, nof_ports, id, phich_len, phich_res);
  srsran_regs_t   regs;
  srsran_pcfich_t pcfich;
  srsran_pdcch_t  pdcch;
  if (srsran_regs_init_opts(&regs, cell, phich_mi, mbsfn_or_sf1_6_tdd != 0) || srsran_pcfich_init(&pcfich, 0) ||
      srsran_pcfich_set_cell(&pcfich, &regs, cell) ||
      srsran_pdcch_init_enb(&pdcch, nof_prb) || srsran_pdcch_set_cell(&pdcch, &regs, cell)) {
    return -1;
  }
  cf_t* sym[SRSRAN_MAX_PORTS] = {NULL};
  for (uint32_t p = 0; p < nof_ports; p++) {
    sym[p] = (cf_t*)grids + (size_t)p * 14 * 12 * nof_prb;
  }
  srsran_dl_sf_cfg_t sf;
  memset(&sf, 0, sizeof(sf));
  sf.tti = tti;
  sf.cfi = cfi;
  int ret = srsran_pcfich_encode(&pcfich, &sf, sym);
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

int ref_ctrl_tx(uint32_t nof_prb, uint32_t nof_ports, uint32_t id, int phich_len, int phich_res, uint32_t tti, uint32_t cfi,
                uint32_t ndci, const uint8_t* payloads, const uint32_t* nof_bits, const uint32_t* L, const uint32_t* ncce,
                const uint16_t* rnti, float* grids)
{
  return ref_ctrl_tx_opts(nof_prb, nof_ports, id, phich_len, phich_res, 1, 0, tti, cfi, ndci, payloads, nof_bits, L,
                          ncce, rnti, grids);
}

/* UE control region on given grids and estimates:
 *   grids: nof_rx grids (14 * 12 * nof_prb cf_t); ce: [port][rx] full-grid estimates.
 * Runs srsran_pcfich_decode (-> *cfi, *corr) then srsran_pdcch_extract_llr; llr receives
 * 72 * nof_cce floats.  Returns nof_cce or < 0. */
static srsran_regs_t   g_regs;
static srsran_pcfich_t g_pcfich;
static srsran_pdcch_t  g_pdcch;
static bool            g_init = false;
static srsran_cell_t   g_cell;

static int rx_setup(srsran_cell_t cell, uint32_t nof_rx)
{
  if (g_init) {
    srsran_pdcch_free(&g_pdcch);
    srsran_pcfich_free(&g_pcfich);
    srsran_regs_free(&g_regs);
    g_init = false;
  }
  if (srsran_regs_init(&g_regs, cell) || srsran_pcfich_init(&g_pcfich, nof_rx) ||
      srsran_pcfich_set_cell(&g_pcfich, &g_regs, cell) || srsran_pdcch_init_ue(&g_pdcch, cell.nof_prb, nof_rx) ||
      srsran_pdcch_set_cell(&g_pdcch, &g_regs, cell)) {
    return -1;
  }
  g_cell = cell;
  g_init = true;
  return 0;
}

int ref_ctrl_rx(uint32_t nof_prb, uint32_t nof_ports, uint32_t id, int phich_len, int phich_res, uint32_t nof_rx,
                uint32_t tti, const float* grids, const float* ce, float noise, uint32_t* cfi, float* corr, float* llr)
{
  srsran_cell_t cell = mkcell(nof_prb, nof_ports, id, phich_len, phich_res);
  if (rx_setup(cell, nof_rx)) {
    return -1;
  }
  const size_t           n = (size_t)14 * 12 * nof_prb;
  cf_t*                  sym[SRSRAN_MAX_PORTS] = {NULL};
  srsran_chest_dl_res_t  res;
  memset(&res, 0, sizeof(res));
  for (uint32_t r = 0; r < nof_rx; r++) {
    sym[r] = (cf_t*)grids + r * n;
    for (uint32_t p = 0; p < nof_ports; p++) {
      res.ce[p][r] = (cf_t*)ce + (p * nof_rx + r) * n;
    }
  }
  res.noise_estimate = noise;
  srsran_dl_sf_cfg_t sf;
  memset(&sf, 0, sizeof(sf));
  sf.tti = tti;
  if (srsran_pcfich_decode(&g_pcfich, &sf, &res, sym, corr) < 0) {
    return -1;
  }
  *cfi = sf.cfi;
  if (srsran_pdcch_extract_llr(&g_pdcch, &sf, &res, sym)) {
    return -1;
  }
  const uint32_t ncce = g_pdcch.nof_cce[sf.cfi - 1];
  memcpy(llr, g_pdcch.llr, 72 * ncce * sizeof(float));
  return (int)ncce;
}

/* srsran_pdcch_decode_msg + srsran_pdcch_msg_corr on LLRs given by the caller (72 * nof_cce
 * floats for `cfi`), after ref_ctrl_rx set the cell up.  Writes the decoded payload bits, the CRC
 * remainder (the RNTI if the message is for it), whether the mean |LLR| passed the 0.3 threshold
 * and the correlation.  Returns the message's nof_bits (0 if skipped) or < 0. */
int ref_pdcch_decode(uint32_t tti, uint32_t cfi, const float* llr, uint32_t nof_cce, uint32_t L, uint32_t ncce, int format,
                     uint32_t cif_enabled, uint8_t* payload, uint16_t* crc_rem, float* corr)
{
  if (!g_init) {
    return -1;
  }
  memcpy(g_pdcch.llr, llr, 72 * nof_cce * sizeof(float));
  srsran_dl_sf_cfg_t sf;
  memset(&sf, 0, sizeof(sf));
  sf.tti = tti;
  sf.cfi = cfi;
  srsran_dci_cfg_t dcfg;
  memset(&dcfg, 0, sizeof(dcfg));
  dcfg.cif_enabled = cif_enabled != 0;
  srsran_dci_msg_t msg;
  memset(&msg, 0, sizeof(msg));
  msg.location.L    = L;
  msg.location.ncce = ncce;
  msg.format        = (srsran_dci_format_t)format;
  if (srsran_pdcch_decode_msg(&g_pdcch, &sf, &dcfg, &msg)) {
    return -1;
  }
  memcpy(payload, msg.payload, SRSRAN_DCI_MAX_BITS);
  *crc_rem = msg.rnti;
  *corr    = msg.nof_bits ? srsran_pdcch_msg_corr(&g_pdcch, &msg) : 0.0f;
  return (int)msg.nof_bits;
}

/* The reference's Viterbi decoder alone (srsran_viterbi_decode_f, the AVX2 16-bit build, tail
 * biting, K = 7, rate 1/3) on 3 * frame_length floats. */
int ref_viterbi_decode_f(const float* symbols, uint32_t frame_length, uint8_t* data)
{
  srsran_viterbi_t v;
  int              poly[3] = {0x6D, 0x4F, 0x57};
  if (srsran_viterbi_init(&v, SRSRAN_VITERBI_37, poly, SRSRAN_DCI_MAX_BITS + 16, true)) {
    return -1;
  }
  float tmp[3 * (SRSRAN_DCI_MAX_BITS + 16)];
  memcpy(tmp, symbols, 3 * frame_length * sizeof(float));
  int r = srsran_viterbi_decode_f(&v, tmp, data, frame_length);
  srsran_viterbi_free(&v);
  return r;
}

/* srsran_rm_conv_rx (rate de-matching of the PDCCH's convolutional code) */
int ref_rm_conv_rx(const float* in, uint32_t in_len, float* out, uint32_t out_len)
{
  float tmp[4096];
  memcpy(tmp, in, in_len * sizeof(float));
  return srsran_rm_conv_rx(tmp, in_len, out, out_len);
}
