/*
 * oracle/ref_harness.c -- drives the reference turbo decoder compiled from
 * /root/reference (TEST INFRASTRUCTURE ONLY; built into oracle/_ref/ by
 * oracle/Makefile and never linked by the product library).
 *
 * Why a harness: src/phy/fec/turbo/turbodecoder.c includes "srsran/srsran.h",
 * which includes the CMake-generated "srsran/version.h".  That header does not
 * exist without running the reference's build system, so turbodecoder.c is
 * unbuildable here (no stand-in headers are written).  Everything it
 * dispatches to IS compiled from the reference as-is:
 *   - the window MAP kernels: include/srsran/phy/fec/turbo/turbodecoder_win.h
 *     instantiated below exactly as turbodecoder.c:50-73 does (SSE16, AVX16);
 *   - the generic MAP kernel: src/phy/fec/turbo/turbodecoder_gen.c;
 *   - the half-iteration driver: include/srsran/phy/fec/turbo/turbodecoder_iter.h;
 *   - QPP tables, vector ops, rate matching, CRC, encoder: their .c files.
 * Only the AUTO-dispatch glue of turbodecoder.c:129-549 is restated here
 * (init, new_cb, tdec_iteration_16, decision, run_all), so the reference's
 * own srsran_tdec_t struct and iteration code run unchanged.
 *
 * The logging hook srsran_phy_log_print (phy_logger.c, also behind srsran.h)
 * stays unresolved; it is only reached on error paths with a registered log
 * handler, so the library is loaded with RTLD_LAZY by the tests.
 */
#include <stdbool.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "srsran/phy/common/phy_common.h"
#include "srsran/phy/fec/cbsegm.h"
#include "srsran/phy/fec/crc.h"
#include "srsran/phy/fec/softbuffer.h"
#include "srsran/phy/fec/turbo/rm_turbo.h"
#include "srsran/phy/fec/turbo/tc_interl.h"
#include "srsran/phy/fec/turbo/turbocoder.h"
#include "srsran/phy/fec/turbo/turbodecoder.h"
#include "srsran/phy/utils/debug.h"
#include "srsran/phy/utils/vector.h"

#include "srsran/phy/fec/turbo/turbodecoder_gen.h"

#define WINIMP_IS_SSE16
#include "srsran/phy/fec/turbo/turbodecoder_win.h"
#undef WINIMP_IS_SSE16

#define WINIMP_IS_AVX16
#include "srsran/phy/fec/turbo/turbodecoder_win.h"
#undef WINIMP_IS_AVX16

static srsran_tdec_16bit_impl_t ref_gen_impl = {tdec_gen_init,
                                                tdec_gen_free,
                                                tdec_gen_dec,
                                                tdec_gen_extract_input,
                                                tdec_gen_decision_byte};
static srsran_tdec_16bit_impl_t ref_sse16_impl = {tdec_winsse16_init,
                                                  tdec_winsse16_free,
                                                  tdec_winsse16_dec,
                                                  tdec_winsse16_extract_input,
                                                  tdec_winsse16_decision_byte};
static srsran_tdec_16bit_impl_t ref_avx16_impl = {tdec_winavx16_init,
                                                  tdec_winavx16_free,
                                                  tdec_winavx16_dec,
                                                  tdec_winavx16_extract_input,
                                                  tdec_winavx16_decision_byte};

#define LLR_IS_16BIT
#include "srsran/phy/fec/turbo/turbodecoder_iter.h"
#undef LLR_IS_16BIT

/* The 8-bit window decoders (turbodecoder.c:76-97): SSE 16 sub-blocks, AVX2 32 sub-blocks. */
#define WINIMP_IS_SSE8
#include "srsran/phy/fec/turbo/turbodecoder_win.h"
#undef WINIMP_IS_SSE8

#define WINIMP_IS_AVX8
#include "srsran/phy/fec/turbo/turbodecoder_win.h"
#undef WINIMP_IS_AVX8

static srsran_tdec_8bit_impl_t ref_sse8_impl = {tdec_winsse8_init,
                                                tdec_winsse8_free,
                                                tdec_winsse8_dec,
                                                tdec_winsse8_extract_input,
                                                tdec_winsse8_decision_byte};
static srsran_tdec_8bit_impl_t ref_avx8_impl = {tdec_winavx8_init,
                                                tdec_winavx8_free,
                                                tdec_winavx8_dec,
                                                tdec_winavx8_extract_input,
                                                tdec_winavx8_decision_byte};

#define LLR_IS_8BIT
#include "srsran/phy/fec/turbo/turbodecoder_iter.h"
#undef LLR_IS_8BIT

/* Restated from turbodecoder.c:381-393 (this symbol is also needed by rm_turbo.c). */
uint32_t srsran_tdec_autoimp_get_subblocks(uint32_t long_cb)
{
  if (!(long_cb % 16) && long_cb > 800) {
    return 16;
  }
  if (!(long_cb % 8) && long_cb > 400) {
    return 8;
  }
  return 0;
}

uint32_t srsran_tdec_autoimp_get_subblocks_8bit(uint32_t long_cb)
{
  if (!(long_cb % 32) && long_cb > 2048) {
    return 32;
  }
  if (!(long_cb % 16) && long_cb > 800) {
    return 16;
  }
  if (!(long_cb % 8) && long_cb > 400) {
    return 8;
  }
  return 0;
}

static srsran_tdec_t tdec;
static bool          tdec_ready = false;

/* AUTO 16-bit init (turbodecoder.c:151-317, SRSRAN_TDEC_AUTO branch). */
static int harness_init(void)
{
  if (tdec_ready) {
    return 0;
  }
  srsran_tdec_t* h = &tdec;
  memset(h, 0, sizeof(*h));
  uint32_t len   = SRSRAN_TCOD_MAX_LEN_CB + SRSRAN_TCOD_TOTALTAIL;
  h->dec_type    = SRSRAN_TDEC_AUTO;
  h->max_long_cb = SRSRAN_TCOD_MAX_LEN_CB;
  h->app1        = srsran_vec_i16_malloc(len);
  h->app2        = srsran_vec_i16_malloc(len);
  h->ext1        = srsran_vec_i16_malloc(len);
  h->ext2        = srsran_vec_i16_malloc(len);
  h->syst0       = srsran_vec_i16_malloc(len);
  h->parity0     = srsran_vec_i16_malloc(len);
  h->parity1     = srsran_vec_i16_malloc(len);
  h->input_conv  = srsran_vec_i16_malloc(len * 3 + 32 * 3);
  h->dec16[0]    = &ref_gen_impl;   /* AUTO_16_SSE slot holds the generic decoder */
  h->dec16[1]    = &ref_sse16_impl; /* AUTO_16_SSEWIN */
  h->dec16[2]    = &ref_avx16_impl; /* AUTO_16_AVXWIN */
  for (int td = 0; td < SRSRAN_TDEC_NOF_AUTO_MODES_16; td++) {
    if ((h->nof_blocks16[td] = h->dec16[td]->tdec_init(&h->dec16_hdlr[td], h->max_long_cb)) < 0) {
      return -1;
    }
  }
  h->dec8[0] = &ref_sse8_impl; /* AUTO_8_SSEWIN */
  h->dec8[1] = &ref_avx8_impl; /* AUTO_8_AVXWIN */
  for (int td = 0; td < SRSRAN_TDEC_NOF_AUTO_MODES_8; td++) {
    if ((h->nof_blocks8[td] = h->dec8[td]->tdec_init(&h->dec8_hdlr[td], h->max_long_cb)) < 0) {
      return -1;
    }
  }
  for (int s = 0; s < 4; s++) {
    for (int i = 0; i < SRSRAN_NOF_TC_CB_SIZES; i++) {
      if (srsran_tc_interl_init(&h->interleaver[s][i], srsran_cbsegm_cbsize(i)) < 0) {
        return -1;
      }
      srsran_tc_interl_LTE_gen_interl(&h->interleaver[s][i], srsran_cbsegm_cbsize(i), s ? (8 << (s - 1)) : 1);
    }
  }
  h->current_cbidx = -1;
  tdec_ready       = true;
  return 0;
}

static uint32_t inter_idx(uint32_t nsb) { return nsb == 32 ? 3 : (nsb == 16 ? 2 : (nsb == 8 ? 1 : 0)); }

/* tdec_iteration_16 (turbodecoder.c:486-507), AUTO 16-bit branch only. */
static void harness_iteration(srsran_tdec_t* h, int16_t* input)
{
  uint32_t nsb          = srsran_tdec_autoimp_get_subblocks(h->current_long_cb);
  h->current_llr_type   = SRSRAN_TDEC_16;
  h->current_dec        = nsb == 16 ? 2 : (nsb == 8 ? 1 : 0);
  h->current_inter_idx  = inter_idx((uint32_t)h->nof_blocks16[h->current_dec]);
  run_tdec_iteration_16bit(h, input);
}

/* The "latest output" the reference decides on (turbodecoder.c:370-378), in natural order. */
static void latest_natural(srsran_tdec_t* h, int16_t* dst)
{
  uint32_t K   = h->current_long_cb;
  int16_t* src = !(h->n_iter % 2) ? (int16_t*)h->app1 : (int16_t*)h->ext1;
  uint32_t nsb = srsran_tdec_autoimp_get_subblocks(K);
  if (!nsb) {
    memcpy(dst, src, K * sizeof(int16_t));
    return;
  }
  uint32_t L = K / nsb;
  for (uint32_t n = 0; n < K; n++) {
    dst[n] = src[(n % L) * nsb + n / L];
  }
}

/*
 * ref_tdec8_run: srsran_tdec_run_all_8bit (turbodecoder.c:560-577) on one code block, AUTO on an AVX2
 * build: tdec_iteration_8 (turbodecoder.c:455-483) with tdec_sb_idx_8 (:426-441).  Where no 8-bit
 * decoder takes K (K <= 800) the reference widens the first 3K+12 values (convert_8_to_16) and runs the
 * 16-bit decoder; with the sub-block layout the rest of its widened buffer is left from earlier calls, so
 * this harness widens the whole layout (3 (K + 32) + 12) instead.
 *  layout_sb: as ref_tdec_run.  trace (optional): nof_iterations*K int8, latest output per half-iteration.
 */
int ref_tdec8_run(uint32_t K, const int8_t* input, int layout_sb, uint32_t nof_iterations, uint8_t* out, int8_t* trace)
{
  if (harness_init()) {
    return -1;
  }
  srsran_tdec_t* h = &tdec;
  int cbidx        = srsran_cbsegm_cbindex(K);
  if (cbidx < 0 || srsran_cbsegm_cbsize(cbidx) != (int)K || nof_iterations < 1) {
    return -1;
  }
  uint32_t nsb8 = srsran_tdec_autoimp_get_subblocks_8bit(K);
  if (nsb8 < 16) {
    uint32_t n    = layout_sb && nsb8 ? 3 * (K + 32) + 12 : 3 * K + 12;
    int16_t* wide = srsran_vec_i16_malloc(3 * (K + 32) + 12 + 64);
    memset(wide, 0, (3 * (K + 32) + 12 + 64) * sizeof(int16_t));
    for (uint32_t i = 0; i < n; i++) {
      wide[i] = input[i];
    }
    int16_t* tr16 = trace ? malloc(sizeof(int16_t) * nof_iterations * K) : NULL;
    int      ret  = ref_tdec_run(K, wide, layout_sb, nof_iterations, out, tr16);
    if (trace) {
      for (uint32_t i = 0; i < nof_iterations * K; i++) {
        trace[i] = (int8_t)tr16[i];
      }
      free(tr16);
    }
    free(wide);
    return ret;
  }
  h->force_not_sb  = layout_sb ? false : true;
  uint32_t in_len  = layout_sb ? 3 * (K + 32) + 12 : 3 * K + 12;
  int8_t*  buf     = srsran_vec_i8_malloc(3 * (K + 32) + 12 + 64);
  memset(buf, 0, 3 * (K + 32) + 12 + 64);
  memcpy(buf, input, in_len);
  h->n_iter            = 0;
  h->current_long_cb   = K;
  h->current_cbidx     = cbidx;
  h->current_llr_type  = SRSRAN_TDEC_8;
  h->current_dec       = nsb8 == 32 ? 1 : 0;
  h->current_inter_idx = inter_idx((uint32_t)h->nof_blocks8[h->current_dec]);
  do {
    run_tdec_iteration_8bit(h, buf);
    if (trace) {
      int8_t*  src = !(h->n_iter % 2) ? (int8_t*)h->app1 : (int8_t*)h->ext1;
      uint32_t L   = K / nsb8;
      for (uint32_t n = 0; n < K; n++) {
        trace[(size_t)(h->n_iter - 1) * K + n] = src[(n % L) * nsb8 + n / L];
      }
    }
  } while (h->n_iter < (int)nof_iterations);
  h->dec8[h->current_dec]->tdec_decision_byte(!(h->n_iter % 2) ? (int8_t*)h->app1 : (int8_t*)h->ext1, out, K);
  h->current_llr_type = SRSRAN_TDEC_16;
  free(buf);
  return 0;
}

/*
 * ref_tdec_run: srsran_tdec_run_all (turbodecoder.c:536-549) on one code block.
 *  layout_sb = 0: natural 3K+12 input, srsran_tdec_force_not_sb() set (as turbodecoder_test does)
 *  layout_sb = 1: rm_turbo_rx_lut layout (production path, sch.c)
 *  trace (optional): nof_iterations*K int16, latest decoder output after every half-iteration.
 */
int ref_tdec_run(uint32_t K, const int16_t* input, int layout_sb, uint32_t nof_iterations, uint8_t* out, int16_t* trace)
{
  if (harness_init()) {
    return -1;
  }
  srsran_tdec_t* h = &tdec;
  int cbidx        = srsran_cbsegm_cbindex(K);
  if (cbidx < 0 || srsran_cbsegm_cbsize(cbidx) != (int)K || nof_iterations < 1) {
    return -1;
  }
  h->force_not_sb = layout_sb ? false : true;
  /* The SB path writes tail values into the input's padding: work on a copy. */
  uint32_t in_len = layout_sb ? 3 * (K + 32) + 12 : 3 * K + 12;
  int16_t* buf    = srsran_vec_i16_malloc(3 * (K + 32) + 12 + 64);
  memset(buf, 0, (3 * (K + 32) + 12 + 64) * sizeof(int16_t));
  memcpy(buf, input, in_len * sizeof(int16_t));

  h->n_iter          = 0;
  h->current_long_cb = K;
  h->current_cbidx   = cbidx;
  do {
    harness_iteration(h, buf);
    if (trace) {
      latest_natural(h, &trace[(size_t)(h->n_iter - 1) * K]);
    }
  } while (h->n_iter < (int)nof_iterations);
  h->dec16[h->current_dec]->tdec_decision_byte(!(h->n_iter % 2) ? h->app1 : h->ext1, out, K);
  free(buf);
  return 0;
}

/* Reference turbo encoder (turbocoder.c:77-185). */
int ref_tcod_encode(uint32_t K, const uint8_t* bits, uint8_t* out)
{
  static srsran_tcod_t tcod;
  static bool          ready = false;
  if (!ready) {
    if (srsran_tcod_init(&tcod, SRSRAN_TCOD_MAX_LEN_CB)) {
      return -1;
    }
    ready = true;
  }
  return srsran_tcod_encode(&tcod, (uint8_t*)bits, out, K);
}

/* The reference's LUT transmit path of one code block: srsran_tcod_encode_lut (turbocoder.c:188-... ; no CB CRC, not
 * the last block: every one of the K / 8 input bytes encoded as given, the tail nibble written after them) when
 * `encode`, then srsran_rm_turbo_tx_lut (rm_turbo.c:345-388) into w_buff / out.  sys: K / 8 + 1 bytes (in / out),
 * parity: at least (2 K + 8) / 8 + 16 bytes (out). */
int ref_tcod_rm_tx_lut(uint32_t cb_idx, uint8_t* sys, uint8_t* parity, uint8_t* w_buff, uint8_t* out, uint32_t out_len,
                       uint32_t w_offset, uint32_t rv, int encode)
{
  static srsran_tcod_t tcod;
  static srsran_crc_t  crc_tb;
  static bool          ready = false;
  if (!ready) {
    if (srsran_tcod_init(&tcod, SRSRAN_TCOD_MAX_LEN_CB) || srsran_crc_init(&crc_tb, SRSRAN_LTE_CRC24A, 24)) {
      return -1;
    }
    srsran_rm_turbo_gentables();
    ready = true;
  }
  if (encode) {
    srsran_crc_set_init(&crc_tb, 0);
    if (srsran_tcod_encode_lut(&tcod, &crc_tb, NULL, sys, parity, cb_idx, false) < 0) {  /* 3 K + 12 on success */
      return -1;
    }
  }
  return srsran_rm_turbo_tx_lut(w_buff, sys, parity, out, cb_idx, out_len, w_offset, rv);
}

/* Reference rate de-matching + HARQ combining into an int16 soft buffer (rm_turbo.c:390-445). */
int ref_rm_turbo_rx_lut(const int16_t* in, int16_t* softbuf, uint32_t in_len, uint32_t cb_idx, uint32_t rv_idx)
{
  srsran_rm_turbo_gentables();
  return srsran_rm_turbo_rx_lut((int16_t*)in, softbuf, in_len, cb_idx, rv_idx);
}

/* Reference byte-wise CRC (crc.c:117-128). */
uint32_t ref_crc_checksum_byte(uint32_t poly, int order, const uint8_t* data, uint32_t nbits)
{
  srsran_crc_t crc;
  memset(&crc, 0, sizeof(crc));
  if (srsran_crc_init(&crc, poly, order)) {
    return 0xFFFFFFFF;
  }
  return srsran_crc_checksum_byte(&crc, data, nbits);
}

/*
 * The reference's INFO()/DEBUG() macros (debug.h:65-82) call the logger of
 * phy_logger.c unless the verbosity is at least that level, in which case they
 * print to stdout.  Around reference calls that log on their normal path we raise
 * the verbosity with the reference's own set_srsran_verbose_level() and silence
 * stdout, so the unbuildable logger is never reached.
 */
#include <fcntl.h>
#include <stdio.h>
#include <unistd.h>
static int quiet_fd = -1;
static void quiet_begin(void)
{
  fflush(stdout);
  quiet_fd = dup(1);
  int nul  = open("/dev/null", O_WRONLY);
  dup2(nul, 1);
  close(nul);
  set_srsran_verbose_level(SRSRAN_VERBOSE_DEBUG);
}
static void quiet_end(void)
{
  fflush(stdout);
  set_srsran_verbose_level(SRSRAN_VERBOSE_NONE);
  dup2(quiet_fd, 1);
  close(quiet_fd);
}

/* Reference code-block segmentation (cbsegm.c:62-117); out = {F,C,K1,K2,K1_idx,K2_idx,C1,C2,tbs}. */
int ref_cbsegm(uint32_t tbs, uint32_t* out)
{
  srsran_cbsegm_t s;
  memset(&s, 0, sizeof(s));
  quiet_begin();
  int ret = srsran_cbsegm(&s, tbs);
  quiet_end();
  out[0]  = s.F;
  out[1]  = s.C;
  out[2]  = s.K1;
  out[3]  = s.K2;
  out[4]  = s.K1_idx;
  out[5]  = s.K2_idx;
  out[6]  = s.C1;
  out[7]  = s.C2;
  out[8]  = s.tbs;
  return ret;
}

/* Reference rate matching TX (rm_turbo.c srsran_rm_turbo_tx, bitwise). */
int ref_rm_turbo_tx(const uint8_t* coded, uint32_t K, uint8_t* out, uint32_t E, uint32_t rv)
{
  static uint8_t w_buff[3 * (6144 + 4 + 32) + 64];
  memset(w_buff, 0, sizeof(w_buff));
  quiet_begin();
  /* the bitwise TX only (re)builds its circular buffer w_buff on an rv=0 call */
  int ret = srsran_rm_turbo_tx(w_buff, sizeof(w_buff), (uint8_t*)coded, 3 * K + 12, out, E, 0);
  if (rv && !ret) {
    ret = srsran_rm_turbo_tx(w_buff, sizeof(w_buff), (uint8_t*)coded, 3 * K + 12, out, E, rv);
  }
  quiet_end();
  return ret;
}

/*
 * ref_dlsch_decode_tb: decode_tb / decode_tb_cb (sch.c:371-573) composed from the
 * reference's own pieces -- srsran_cbsegm, srsran_rm_turbo_rx_lut, the turbo
 * half-iteration (turbodecoder_iter.h) with its decision_byte, srsran_crc_checksum_byte.
 * Only the sch.c loop is restated (sch.c includes the generated srsran/version.h via
 * srsran/srsran.h and cannot be compiled here).  Same arguments as oracle_dlsch_decode_tb.
 * Note: the reference turbo decoder writes tail values into the SB soft buffer's padding
 * (turbodecoder_iter.h extract_input), so only decode outputs are comparable, not padding.
 */
int ref_dlsch_decode_tb(uint32_t       tbs,
                        uint32_t       Qm,
                        uint32_t       rv,
                        uint32_t       nof_e_bits,
                        const int16_t* e_bits,
                        uint32_t       max_iterations,
                        int16_t*       softbuf,
                        uint32_t       softbuf_stride,
                        uint8_t*       cb_crc,
                        uint8_t*       cb_data,
                        uint32_t       cb_data_stride,
                        uint8_t*       data,
                        uint32_t*      cb_noi_out,
                        float*         avg_iterations)
{
  static srsran_crc_t crc_tb, crc_cb;
  static bool         crc_ready = false;
  if (harness_init()) {
    return -1;
  }
  if (!crc_ready) {
    srsran_crc_init(&crc_tb, SRSRAN_LTE_CRC24A, 24);
    srsran_crc_init(&crc_cb, SRSRAN_LTE_CRC24B, 24);
    crc_ready = true;
  }
  srsran_rm_turbo_gentables();
  srsran_cbsegm_t s;
  quiet_begin();
  int rc = srsran_cbsegm(&s, tbs);
  quiet_end();
  if (rc) {
    return -1;
  }
  if (s.tbs == 0 || s.C == 0) {
    return 0;
  }
  if (s.F) {
    return -2;
  }
  if (s.C > SRSRAN_MAX_CODEBLOCKS) {
    return -1;
  }
  srsran_tdec_t* h   = &tdec;
  float          avg = 0;
  h->force_not_sb    = false;
  for (uint32_t cb = 0; cb < s.C; cb++) {
    const uint32_t cb_len     = cb < s.C1 ? s.K1 : s.K2;
    const uint32_t cb_len_idx = cb < s.C1 ? s.K1_idx : s.K2_idx;
    const uint32_t rlen       = s.C == 1 ? cb_len : cb_len - 24;
    if (!cb_crc[cb]) {
      const uint32_t Gp    = nof_e_bits / Qm;
      const uint32_t gamma = Gp % s.C;
      const uint32_t n_e   = Qm * (Gp / s.C);
      uint32_t       rp    = cb * n_e;
      uint32_t       n_e2  = n_e;
      if (cb > s.C - gamma) {
        n_e2 = n_e + Qm;
        rp   = (s.C - gamma) * n_e + (cb - (s.C - gamma)) * n_e2;
      }
      /* buffer_f[cb] is srsran_vec_i16_malloc'ed (aligned) in the reference: stage it */
      static int16_t* sb = NULL;
      if (!sb) {
        sb = srsran_vec_i16_malloc(SOFTBUFFER_SIZE + 64);
      }
      memcpy(sb, &softbuf[(size_t)cb * softbuf_stride], softbuf_stride * sizeof(int16_t));
      srsran_rm_turbo_rx_lut((int16_t*)&e_bits[rp], sb, n_e2, cb_len_idx, rv);
      h->n_iter          = 0;
      h->current_long_cb = cb_len;
      h->current_cbidx   = (int)cb_len_idx;
      uint32_t noi = 0;
      bool     early = false;
      do {
        harness_iteration(h, sb);
        h->dec16[h->current_dec]->tdec_decision_byte(!(h->n_iter % 2) ? h->app1 : h->ext1, &data[cb * rlen / 8],
                                                     cb_len);
        avg += 1;
        noi++;
        srsran_crc_t*  crc     = s.C > 1 ? &crc_cb : &crc_tb;
        const uint32_t len_crc = s.C > 1 ? cb_len : s.tbs + 24;
        if (!srsran_crc_checksum_byte(crc, &data[cb * rlen / 8], len_crc) && noi >= 2) {
          cb_crc[cb] = 1;
          early      = true;
        }
      } while (noi < max_iterations && !early);
      memcpy(&softbuf[(size_t)cb * softbuf_stride], sb, softbuf_stride * sizeof(int16_t));
      if (cb_noi_out) {
        cb_noi_out[cb] = noi;
      }
    } else {
      memcpy(&data[cb * rlen / 8], &cb_data[(size_t)cb * cb_data_stride], rlen / 8);
      if (cb_noi_out) {
        cb_noi_out[cb] = 0;
      }
    }
  }
  bool tb_ok = true;
  for (uint32_t i = 0; i < s.C && tb_ok; i++) {
    tb_ok = cb_crc[i];
  }
  if (!tb_ok) {
    for (uint32_t i = 0; i < s.C; i++) {
      if (cb_crc[i]) {
        const uint32_t cb_len = i < s.C1 ? s.K1 : s.K2;
        const uint32_t rlen   = s.C == 1 ? cb_len : cb_len - 24;
        memcpy(&cb_data[(size_t)i * cb_data_stride], &data[i * rlen / 8], rlen / 8);
      }
    }
  }
  if (avg_iterations) {
    *avg_iterations = avg / (float)s.C;
  }
  if (!tb_ok) {
    return -1;
  }
  if (s.C == 1) {
    return 0;
  }
  if (srsran_crc_match_byte(&crc_tb, data, s.tbs)) {
    return 0;
  }
  memset(cb_crc, 0, s.C);
  return -1;
}

/*
 * ref_dlsch_decode_tb8: decode_tb with q->llr_is_8bit (sch.c:409-428) over the reference's own 8-bit pieces --
 * srsran_rm_turbo_rx_lut_8bit into the soft buffer row used as int8, srsran_tdec_iteration_8bit (tdec_iteration_8:
 * the 8-bit window decoders of K > 800, the 16-bit ones on the widened input otherwise) with its decision_byte,
 * srsran_crc_checksum_byte.  Same arguments as ref_dlsch_decode_tb with int8 e bits.  For K <= 800 the whole
 * sub-block layout is widened, as ref_tdec8_run does (convert_8_to_16 widens 3K + 12 values only).
 */
int ref_dlsch_decode_tb8(uint32_t      tbs,
                         uint32_t      Qm,
                         uint32_t      rv,
                         uint32_t      nof_e_bits,
                         const int8_t* e_bits,
                         uint32_t      max_iterations,
                         int16_t*      softbuf,
                         uint32_t      softbuf_stride,
                         uint8_t*      cb_crc,
                         uint8_t*      cb_data,
                         uint32_t      cb_data_stride,
                         uint8_t*      data,
                         uint32_t*     cb_noi_out,
                         float*        avg_iterations)
{
  static srsran_crc_t crc_tb, crc_cb;
  static bool         crc_ready = false;
  if (harness_init()) {
    return -1;
  }
  if (!crc_ready) {
    srsran_crc_init(&crc_tb, SRSRAN_LTE_CRC24A, 24);
    srsran_crc_init(&crc_cb, SRSRAN_LTE_CRC24B, 24);
    crc_ready = true;
  }
  srsran_rm_turbo_gentables();
  srsran_cbsegm_t s;
  quiet_begin();
  int rc = srsran_cbsegm(&s, tbs);
  quiet_end();
  if (rc) {
    return -1;
  }
  if (s.tbs == 0 || s.C == 0) {
    return 0;
  }
  if (s.F) {
    return -2;
  }
  if (s.C > SRSRAN_MAX_CODEBLOCKS) {
    return -1;
  }
  srsran_tdec_t*  h    = &tdec;
  float           avg  = 0;
  static int8_t*  sb8  = NULL;
  static int16_t* wide = NULL;
  if (!sb8) {
    sb8  = srsran_vec_i8_malloc(2 * (SOFTBUFFER_SIZE + 64));
    wide = srsran_vec_i16_malloc(SOFTBUFFER_SIZE + 64);
  }
  h->force_not_sb = false;
  for (uint32_t cb = 0; cb < s.C; cb++) {
    const uint32_t cb_len     = cb < s.C1 ? s.K1 : s.K2;
    const uint32_t cb_len_idx = cb < s.C1 ? s.K1_idx : s.K2_idx;
    const uint32_t rlen       = s.C == 1 ? cb_len : cb_len - 24;
    if (!cb_crc[cb]) {
      const uint32_t Gp    = nof_e_bits / Qm;
      const uint32_t gamma = Gp % s.C;
      const uint32_t n_e   = Qm * (Gp / s.C);
      uint32_t       rp    = cb * n_e;
      uint32_t       n_e2  = n_e;
      if (cb > s.C - gamma) {
        n_e2 = n_e + Qm;
        rp   = (s.C - gamma) * n_e + (cb - (s.C - gamma)) * n_e2;
      }
      memcpy(sb8, &softbuf[(size_t)cb * softbuf_stride], softbuf_stride * sizeof(int16_t));
      srsran_rm_turbo_rx_lut_8bit((int8_t*)&e_bits[rp], sb8, n_e2, cb_len_idx, rv);
      const uint32_t nsb8 = srsran_tdec_autoimp_get_subblocks_8bit(cb_len);
      if (nsb8 < 16) {
        const uint32_t n = nsb8 ? 3 * (cb_len + 32) + 12 : 3 * cb_len + 12;
        for (uint32_t i = 0; i < n; i++) {
          wide[i] = sb8[i];
        }
      }
      h->n_iter          = 0;
      h->current_long_cb = cb_len;
      h->current_cbidx   = (int)cb_len_idx;
      uint32_t noi       = 0;
      bool     early     = false;
      do {
        uint8_t* dst = &data[cb * rlen / 8];
        if (nsb8 >= 16) {
          h->current_llr_type  = SRSRAN_TDEC_8;
          h->current_dec       = nsb8 == 32 ? 1 : 0;
          h->current_inter_idx = inter_idx((uint32_t)h->nof_blocks8[h->current_dec]);
          run_tdec_iteration_8bit(h, sb8);
          h->dec8[h->current_dec]->tdec_decision_byte(!(h->n_iter % 2) ? (int8_t*)h->app1 : (int8_t*)h->ext1, dst,
                                                      cb_len);
        } else {
          harness_iteration(h, wide);
          h->dec16[h->current_dec]->tdec_decision_byte(!(h->n_iter % 2) ? h->app1 : h->ext1, dst, cb_len);
        }
        avg += 1;
        noi++;
        srsran_crc_t*  crc     = s.C > 1 ? &crc_cb : &crc_tb;
        const uint32_t len_crc = s.C > 1 ? cb_len : s.tbs + 24;
        if (!srsran_crc_checksum_byte(crc, dst, len_crc) && noi >= 2) {
          cb_crc[cb] = 1;
          early      = true;
        }
      } while (noi < max_iterations && !early);
      h->current_llr_type = SRSRAN_TDEC_16;
      memcpy(&softbuf[(size_t)cb * softbuf_stride], sb8, softbuf_stride * sizeof(int16_t));
      if (cb_noi_out) {
        cb_noi_out[cb] = noi;
      }
    } else {
      memcpy(&data[cb * rlen / 8], &cb_data[(size_t)cb * cb_data_stride], rlen / 8);
      if (cb_noi_out) {
        cb_noi_out[cb] = 0;
      }
    }
  }
  bool tb_ok = true;
  for (uint32_t i = 0; i < s.C && tb_ok; i++) {
    tb_ok = cb_crc[i];
  }
  if (!tb_ok) {
    for (uint32_t i = 0; i < s.C; i++) {
      if (cb_crc[i]) {
        const uint32_t cb_len = i < s.C1 ? s.K1 : s.K2;
        const uint32_t rlen   = s.C == 1 ? cb_len : cb_len - 24;
        memcpy(&cb_data[(size_t)i * cb_data_stride], &data[i * rlen / 8], rlen / 8);
      }
    }
  }
  if (avg_iterations) {
    *avg_iterations = avg / (float)s.C;
  }
  if (!tb_ok) {
    return -1;
  }
  if (s.C == 1) {
    return 0;
  }
  if (srsran_crc_match_byte(&crc_tb, data, s.tbs)) {
    return 0;
  }
  memset(cb_crc, 0, s.C);
  return -1;
}
