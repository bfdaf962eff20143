/*
 * oracle/ref_nr_harness.c -- drives the reference NR shared-channel receive path compiled from
 * /root/reference (TEST INFRASTRUCTURE ONLY; built into oracle/_ref/ by oracle/Makefile).
 *
 * lib/src/phy/phch/sch_nr.c, ra_nr.c, fec/softbuffer.c, fec/cbsegm.c, fec/ldpc/ldpc_rm.c and the
 * LDPC decoder compile as they are; this file only gives ctypes flat entry points so the tests
 * never mirror the reference's structs: srsran_sch_nr_init_rx + srsran_dlsch_nr_decode with a
 * caller-kept reference softbuffer, srsran_ldpc_rm_rx_c, srsran_sch_nr_fill_tb_info and
 * srsran_cbsegm_ldpc_bg1/bg2.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "srsran/phy/fec/cbsegm.h"
#include "srsran/phy/fec/ldpc/ldpc_rm.h"
#include "srsran/phy/fec/softbuffer.h"
#include "srsran/phy/phch/ra_nr.h"
#include "srsran/phy/phch/sch_nr.h"
#include "srsran/phy/utils/debug.h"
#include "srsran/phy/utils/vector.h"

/* INFO()/DEBUG() in cbsegm.c and sch_nr.c call srsran_phy_log_print (phy_logger.c, behind the
 * unbuildable srsran.h) unless the verbosity makes them print; as in ref_harness.c, raise the
 * verbosity with the reference's own set_srsran_verbose_level() and silence stdout. */
#include <fcntl.h>
#include <stdio.h>
#include <unistd.h>
static int nr_quiet_fd = -1;
static void quiet_on(void)
{
  fflush(stdout);
  nr_quiet_fd = dup(1);
  int nul     = open("/dev/null", O_WRONLY);
  dup2(nul, 1);
  close(nul);
  set_srsran_verbose_level(SRSRAN_VERBOSE_DEBUG);
}
static void quiet_off(void)
{
  fflush(stdout);
  set_srsran_verbose_level(SRSRAN_VERBOSE_NONE);
  dup2(nr_quiet_fd, 1);
  close(nr_quiet_fd);
}

static srsran_mod_t qm_to_mod(uint32_t Qm)
{
  switch (Qm) {
    case 1:
      return SRSRAN_MOD_BPSK;
    case 2:
      return SRSRAN_MOD_QPSK;
    case 4:
      return SRSRAN_MOD_16QAM;
    case 6:
      return SRSRAN_MOD_64QAM;
    default:
      return SRSRAN_MOD_256QAM;
  }
}

void* ref_nr_softbuffer_new(uint32_t max_cb, uint32_t max_cb_size)
{
  srsran_softbuffer_rx_t* sb = calloc(1, sizeof(srsran_softbuffer_rx_t));
  if (srsran_softbuffer_rx_init_guru(sb, max_cb, max_cb_size) != 0) {
    free(sb);
    return NULL;
  }
  return sb;
}

void ref_nr_softbuffer_free(void* h)
{
  srsran_softbuffer_rx_free((srsran_softbuffer_rx_t*)h);
  free(h);
}

void ref_nr_softbuffer_reset(void* h) { srsran_softbuffer_rx_reset((srsran_softbuffer_rx_t*)h); }

/* copy out CB r's int8 rate-dematching buffer (n bytes), its packed data (nd bytes) and cb_crc */
int ref_nr_softbuffer_get(void* h, uint32_t r, int8_t* buf, uint32_t n, uint8_t* data, uint32_t nd)
{
  srsran_softbuffer_rx_t* sb = h;
  memcpy(buf, sb->buffer_f[r], n);
  memcpy(data, sb->data[r], nd);
  return sb->cb_crc[r] ? 1 : 0;
}

/* a persistent receiver (srsran_sch_nr_init_rx once, as a UE / gNB holds it) */
void* ref_nr_rx_new(uint32_t nof_prb, float scaling, uint32_t max_iter)
{
  srsran_sch_nr_t* q = calloc(1, sizeof(srsran_sch_nr_t));
  if (!q) {
    return NULL;
  }
  srsran_sch_nr_args_t args   = {};
  args.decoder_scaling_factor = scaling;
  args.max_nof_iter           = max_iter;
  srsran_carrier_nr_t carrier = {};
  carrier.nof_prb             = nof_prb;
  carrier.max_mimo_layers     = 4;
  quiet_on();
  if (srsran_sch_nr_init_rx(q, &args) != 0 || srsran_sch_nr_set_carrier(q, &carrier) != 0) {
    quiet_off();
    free(q);
    return NULL;
  }
  quiet_off();
  return q;
}

void ref_nr_rx_free(void* h)
{
  if (h) {
    srsran_sch_nr_free((srsran_sch_nr_t*)h);
    free(h);
  }
}

/* one srsran_dlsch_nr_decode on receiver `rx` into soft buffer `h` */
int ref_nr_rx_decode(void*         rx,
                     void*         h,
                     int           mcs_table_256qam,
                     int           lbrm,
                     uint32_t      Qm,
                     uint32_t      N_L,
                     uint32_t      tbs,
                     double        R,
                     uint32_t      rv,
                     uint32_t      nof_bits,
                     const int8_t* e_bits,
                     uint8_t*      payload,
                     int*          crc,
                     float*        avg_iter)
{
  srsran_sch_cfg_t cfg  = {};
  cfg.mcs_table         = mcs_table_256qam ? srsran_mcs_table_256qam : srsran_mcs_table_64qam;
  cfg.limited_buffer_rm = lbrm != 0;
  srsran_sch_tb_t tb    = {};
  tb.mod                = qm_to_mod(Qm);
  tb.N_L                = N_L;
  tb.tbs                = (int)tbs;
  tb.R                  = R;
  tb.rv                 = (int)rv;
  tb.nof_bits           = nof_bits;
  tb.enabled            = true;
  tb.softbuffer.rx      = (srsran_softbuffer_rx_t*)h;
  srsran_sch_tb_res_nr_t res = {};
  res.payload                = payload;
  quiet_on();
  const int r = srsran_dlsch_nr_decode((srsran_sch_nr_t*)rx, &cfg, &tb, (int8_t*)e_bits, &res);
  quiet_off();
  *crc      = res.crc ? 1 : 0;
  *avg_iter = res.avg_iter;
  return r;
}

/* one srsran_dlsch_nr_decode with a receiver of its own */
int ref_nr_decode(void*         h,
                  uint32_t      nof_prb,
                  int           mcs_table_256qam,
                  int           lbrm,
                  uint32_t      Qm,
                  uint32_t      N_L,
                  uint32_t      tbs,
                  double        R,
                  uint32_t      rv,
                  uint32_t      nof_bits,
                  float         scaling,
                  uint32_t      max_iter,
                  const int8_t* e_bits,
                  uint8_t*      payload,
                  int*          crc,
                  float*        avg_iter)
{
  void* rx = ref_nr_rx_new(nof_prb, scaling, max_iter);
  if (!rx) {
    return -100;
  }
  const int r =
      ref_nr_rx_decode(rx, h, mcs_table_256qam, lbrm, Qm, N_L, tbs, R, rv, nof_bits, e_bits, payload, crc, avg_iter);
  ref_nr_rx_free(rx);
  return r;
}

/* srsran_sch_nr_fill_tb_info -> out[15] = {bg, Qm, G, A, L_tb, L_cb, B, Bp, Kp, Kr, F, Nref, Z, Nl, C} */
int ref_nr_tb_info(uint32_t nof_prb, int mcs_table_256qam, int lbrm, uint32_t Qm, uint32_t N_L, uint32_t tbs,
                   double R, uint32_t nof_bits, uint32_t* out)
{
  srsran_carrier_nr_t carrier = {};
  carrier.nof_prb             = nof_prb;
  carrier.max_mimo_layers     = 4;
  srsran_sch_cfg_t cfg        = {};
  cfg.mcs_table               = mcs_table_256qam ? srsran_mcs_table_256qam : srsran_mcs_table_64qam;
  cfg.limited_buffer_rm       = lbrm != 0;
  srsran_sch_tb_t tb          = {};
  tb.mod                      = qm_to_mod(Qm);
  tb.N_L                      = N_L;
  tb.tbs                      = (int)tbs;
  tb.R                        = R;
  tb.nof_bits                 = nof_bits;
  srsran_sch_nr_tb_info_t t   = {};
  quiet_on();
  const int r = srsran_sch_nr_fill_tb_info(&carrier, &cfg, &tb, &t);
  quiet_off();
  const uint32_t v[15] = {t.bg, t.Qm, t.G, t.A, t.L_tb, t.L_cb, t.B, t.Bp, t.Kp, t.Kr, t.F, t.Nref, t.Z, t.Nl, t.C};
  memcpy(out, v, sizeof(v));
  return r;
}

int ref_ldpc_rm_rx_c(const int8_t* in, int8_t* out, uint32_t E, uint32_t F, int bg, uint32_t ls, uint32_t rv,
                     uint32_t Qm, uint32_t Nref)
{
  srsran_ldpc_rm_t rm = {};
  if (srsran_ldpc_rm_rx_init_c(&rm) != 0) {
    return -100;
  }
  const int r = srsran_ldpc_rm_rx_c(&rm, in, out, E, F, (srsran_basegraph_t)bg, ls, (uint8_t)rv, qm_to_mod(Qm), Nref);
  srsran_ldpc_rm_rx_free_c(&rm);
  return r;
}

int ref_cbsegm_ldpc(int bg, uint32_t tbs, uint32_t* out)
{
  srsran_cbsegm_t s = {};
  quiet_on();
  const int r = bg == 0 ? srsran_cbsegm_ldpc_bg1(&s, tbs) : srsran_cbsegm_ldpc_bg2(&s, tbs);
  quiet_off();
  const uint32_t  v[6] = {s.tbs, s.L_tb, s.L_cb, s.C, s.K1, s.Z};
  memcpy(out, v, sizeof(v));
  return r;
}

/* srsran_dlsch_nr_encode into e_bits (one bit per byte, nof_bits of them) */
int ref_nr_encode(uint32_t       nof_prb,
                  int            mcs_table_256qam,
                  int            lbrm,
                  uint32_t       Qm,
                  uint32_t       N_L,
                  uint32_t       tbs,
                  double         R,
                  uint32_t       rv,
                  uint32_t       nof_bits,
                  const uint8_t* payload,
                  uint8_t*       e_bits)
{
  srsran_sch_nr_t      q    = {};
  srsran_sch_nr_args_t args = {};
  quiet_on();
  if (srsran_sch_nr_init_tx(&q, &args) != 0) {
    quiet_off();
    return -100;
  }
  srsran_carrier_nr_t carrier = {};
  carrier.nof_prb             = nof_prb;
  carrier.max_mimo_layers     = 4;
  srsran_sch_nr_set_carrier(&q, &carrier);
  srsran_softbuffer_tx_t sb = {};
  if (srsran_softbuffer_tx_init_guru(&sb, SRSRAN_SCH_NR_MAX_NOF_CB_LDPC, SRSRAN_LDPC_MAX_LEN_ENCODED_CB) != 0) {
    srsran_sch_nr_free(&q);
    quiet_off();
    return -101;
  }
  srsran_sch_cfg_t cfg  = {};
  cfg.mcs_table         = mcs_table_256qam ? srsran_mcs_table_256qam : srsran_mcs_table_64qam;
  cfg.limited_buffer_rm = lbrm != 0;
  srsran_sch_tb_t tb    = {};
  tb.mod                = qm_to_mod(Qm);
  tb.N_L                = N_L;
  tb.tbs                = (int)tbs;
  tb.R                  = R;
  tb.rv                 = (int)rv;
  tb.nof_bits           = nof_bits;
  tb.enabled            = true;
  tb.softbuffer.tx      = &sb;
  const int r           = srsran_dlsch_nr_encode(&q, &cfg, &tb, payload, e_bits);
  quiet_off();
  srsran_softbuffer_tx_free(&sb);
  srsran_sch_nr_free(&q);
  return r;
}

/* srsran_ra_nr_tbs (ra_nr.c:502-522): a valid NR transport block size */
uint32_t ref_ra_nr_tbs(uint32_t N_re, double S, double R, uint32_t Qm, uint32_t nof_layers)
{
  return srsran_ra_nr_tbs(N_re, S, R, Qm, nof_layers);
}
