/* oracle/nr_sch_oracle.c -- CPU restatement of srsRAN's NR shared-channel receive path
 * (TEST INFRASTRUCTURE ONLY: only tests/, smoke() and bench.py's cpu_baseline load it).
 *
 * Follows (reference file:line, lib/src/phy/):
 *   LDPC code block segmentation     fec/cbsegm.c:51-60, 152-277 (srsran_cbsegm_ldpc_bg1/bg2)
 *   base graph selection             phch/sch_nr.c:33-45
 *   LBRM: n_prb_lbrm, N_ref, TBS     phch/sch_nr.c:53-112, phch/ra_nr.c:449-522 (n_info > 3824 branch)
 *   TB info                          phch/sch_nr.c:114-176
 *   E per code block                 phch/sch_nr.c:178-189
 *   LDPC rate dematching (int8)      fec/ldpc/ldpc_rm.c:99-160 (init_rm), 297-338, 396-410, 675-706
 *   decode loop + TB assembly        phch/sch_nr.c:554-750, including the reference's input offset:
 *                                    a code block already decoded (cb_crc set) does not advance the
 *                                    LLR read pointer (sch_nr.c:633-636 vs :682)
 * The LDPC decoder is oracle/ldpc_oracle.c (SCALE_SIMD arithmetic: the reference's NR SCH uses the
 * AVX2/AVX512 decoder, sch_nr.c:290-300). */
#include "nr_sch_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "ldpc_oracle.h"

#define CEIL(n, d) (((n) + (d)-1) / (d))

static int select_ls(uint32_t Kp, uint32_t Kb, uint32_t* Z)
{
  if (CEIL(Kp, Kb) > 384) {
    return -1;
  }
  for (uint32_t z = CEIL(Kp, Kb); z <= 384; z++) {
    if (oracle_ldpc_ls_index((int)z) >= 0) {
      *Z = z;
      return 0;
    }
  }
  return -1;
}

int oracle_nr_cbsegm(int bg, uint32_t tbs, oracle_nr_cbsegm_t* s)
{
  memset(s, 0, sizeof(*s));
  if (tbs == 0) {
    return 0;
  }
  const uint32_t L    = tbs <= 3824 ? 16 : 24;
  const uint32_t K_cb = bg == 0 ? 8448 : 3840;
  const uint32_t B    = tbs + L;
  uint32_t       C, Bp;
  if (B <= K_cb) {
    C  = 1;
    Bp = B;
  } else {
    C  = CEIL(B, K_cb - 24);
    Bp = B + 24 * C;
  }
  const uint32_t Kp = Bp / C;
  uint32_t       Kb = 22;
  if (bg == 1) {
    Kb = B > 640 ? 10 : (B > 560 ? 9 : (B > 192 ? 8 : 6));
  }
  uint32_t Z = 0;
  if (select_ls(Kp, Kb, &Z)) {
    return -1;
  }
  s->tbs  = tbs;
  s->L_tb = L;
  s->L_cb = C > 1 ? 24 : 0;
  s->C    = C;
  s->K    = Z * (bg == 0 ? 22 : 10);
  s->Z    = Z;
  return 0;
}

int oracle_nr_select_bg(uint32_t tbs, double R)
{
  return ((tbs <= 292) || (tbs <= 3824 && R <= 0.67) || (R <= 0.25)) ? 1 : 0;
}

static uint32_t n_prb_lbrm(uint32_t nof_prb)
{
  if (nof_prb <= 66) {
    return 32;
  }
  if (nof_prb <= 107) {
    return 107;
  }
  if (nof_prb <= 135) {
    return 135;
  }
  if (nof_prb <= 162) {
    return 162;
  }
  if (nof_prb <= 217) {
    return 217;
  }
  return 273;
}

/* srsran_ra_nr_tbs for n_info > 3824 (always the case for the LBRM reference TB) */
static uint32_t tbs_large(uint32_t N_re, double R, uint32_t Qm, uint32_t layers)
{
  const uint32_t n_info = (uint32_t)(N_re * 1.0 * R * Qm * layers);
  const uint32_t n      = (uint32_t)(floor(log2(n_info - 24.0)) - 5.0);
  uint32_t       nip    = (1u << n) * (uint32_t)round((double)(n_info - 24.0) / (double)(1u << n));
  if (nip < 3840) {
    nip = 3840;
  }
  if (R <= 0.25) {
    const uint32_t C = CEIL(nip + 24u, 3816u);
    return 8u * C * CEIL(nip + 24u, 8u * C) - 24u;
  }
  if (nip > 8424) {
    const uint32_t C = CEIL(nip + 24u, 8424u);
    return 8u * C * CEIL(nip + 24u, 8u * C) - 24u;
  }
  return 8u * CEIL(nip + 24u, 8u) - 24u;
}

uint32_t oracle_nr_Nref(uint32_t nof_prb, int mcs_table_256qam, uint32_t max_mimo_layers)
{
  const uint32_t N_re  = 156 * n_prb_lbrm(nof_prb);
  const uint32_t Qm    = mcs_table_256qam ? 8 : 6;
  const uint32_t tbs   = tbs_large(N_re, 948.0 / 1024.0, Qm, max_mimo_layers < 4 ? max_mimo_layers : 4);
  const double   R     = 2.0 / 3.0;
  oracle_nr_cbsegm_t s;
  if (oracle_nr_cbsegm(oracle_nr_select_bg(tbs, R), tbs, &s)) {
    return 0;
  }
  return (uint32_t)ceil((double)tbs / (double)(s.C * R));
}

int oracle_nr_tb_info(uint32_t tbs, double R, uint32_t Qm, uint32_t G, uint32_t Nl, int lbrm, uint32_t nof_prb,
                      int mcs_table_256qam, oracle_nr_tb_info_t* t)
{
  memset(t, 0, sizeof(*t));
  t->bg = oracle_nr_select_bg(tbs, R);
  oracle_nr_cbsegm_t s;
  if (oracle_nr_cbsegm(t->bg, tbs, &s)) {
    return -1;
  }
  t->Qm   = Qm;
  t->A    = tbs;
  t->L_tb = s.L_tb;
  t->L_cb = s.L_cb;
  t->B    = s.tbs + s.L_tb;
  t->Bp   = t->B + s.L_cb * s.C;
  t->Kp   = s.C ? t->Bp / s.C : 0;
  t->Kr   = s.K;
  t->F    = t->Kr - t->Kp;
  t->Z    = s.Z;
  t->G    = G;
  t->Nl   = Nl;
  t->Nref = lbrm ? oracle_nr_Nref(nof_prb, mcs_table_256qam, 4) : 384 * 66;  // SRSRAN_LDPC_MAX_LEN_ENCODED_CB
  t->C    = s.C;
  return 0;
}

uint32_t oracle_nr_E(const oracle_nr_tb_info_t* t, uint32_t j)
{
  const uint32_t q = t->Nl * t->Qm;
  if (j <= t->C - (t->G / q) % t->C - 1) {
    return q * (t->G / (q * t->C));
  }
  return q * CEIL(t->G, q * t->C);
}

/* init_rm: k0 and Ncb (ldpc_rm.c:99-160) */
static void rm_params(int bg, uint32_t ls, uint32_t rv, uint32_t Nref, uint32_t* k0, uint32_t* Ncb)
{
  static const uint32_t BASEK0[4][2] = {{0, 0}, {17, 13}, {33, 25}, {56, 43}};
  const uint32_t        N            = ls * (bg == 0 ? 66 : 50);
  if (N <= Nref) {
    *Ncb = N;
    *k0  = ls * BASEK0[rv][bg];
  } else {
    *Ncb = Nref;
    *k0  = ls * ((BASEK0[rv][bg] * Nref) / N);
  }
}

int oracle_ldpc_rm_rx_c(const int8_t* in, int8_t* out, uint32_t E, uint32_t F, int bg, uint32_t ls, uint32_t rv,
                        uint32_t Qm, uint32_t Nref)
{
  if (Qm == 0 || E % Qm) {
    return -1;
  }
  uint32_t k0, Ncb;
  rm_params(bg, ls, rv, Nref, &k0, &Ncb);
  const uint32_t K   = ls * (bg == 0 ? 22 : 10);
  const uint32_t end = K - 2 * ls, ini = end - F;
  /* bit de-interleaver: tmp[i cols + j] = in[j rows + i] */
  int8_t*        tmp  = malloc(E ? E : 1);
  const uint32_t cols = E / Qm;
  for (uint32_t j = 0; j < cols; j++) {
    for (uint32_t i = 0; i < Qm; i++) {
      tmp[i * cols + j] = in[j * Qm + i];
    }
  }
  /* bit selection with saturating accumulation (infinity7 = 63), filler bits = 127 */
  for (uint32_t i = ini; i < end; i++) {
    out[i] = 127;
  }
  uint32_t k = 0, j = 0;
  while (k < E) {
    const uint32_t p = (k0 + j) % Ncb;
    if (!(p >= ini && p < end)) {
      long t = (long)out[p] + tmp[k];
      t      = t > 63 ? 63 : (t < -63 ? -63 : t);
      out[p] = (int8_t)t;
      k++;
    }
    j++;
  }
  free(tmp);
  return (int)(k0 + E < Ncb ? k0 + E : Ncb);
}

static uint32_t crc_bits_msb(uint32_t poly, int order, const uint8_t* bits, uint32_t n)
{
  const uint32_t top = 1u << (order - 1), mask = (1u << order) - 1u;
  uint32_t       crc = 0;
  for (uint32_t i = 0; i < n; i++) {
    crc ^= (bits[i] & 1) ? top : 0;
    crc = ((crc & top) ? ((crc << 1) ^ poly) : (crc << 1)) & mask;
  }
  return crc;
}

int oracle_nr_sch_decode(const oracle_nr_tb_info_t* t,
                         uint32_t                   rv,
                         const int8_t*              e_bits,
                         float                      scaling,
                         int                        max_iter,
                         int8_t*                    softbuf,
                         uint32_t                   softbuf_stride,
                         uint8_t*                   cb_crc,
                         uint8_t*                   cb_data,
                         uint32_t                   cb_data_stride,
                         uint8_t*                   payload,
                         int*                       tb_crc,
                         float*                     avg_iter)
{
  const uint32_t CRC24A = 0x1864CFB, CRC24B = 0x1800063, CRC16 = 0x11021;
  const uint32_t Z = t->Z, C = t->C;
  const uint32_t nllr = Z * (t->bg == 0 ? 66 : 50);
  uint8_t*       msg  = malloc(t->Kr);
  const int8_t*  in   = e_bits;
  uint32_t       iter_sum = 0, cb_ok = 0, j = 0;
  *tb_crc                 = 0;
  for (uint32_t r = 0; r < C; r++) {
    const uint32_t E = oracle_nr_E(t, j);
    j++;
    if (cb_crc[r]) { /* already decoded: skipped, and the read pointer does not move */
      cb_ok++;
      continue;
    }
    int8_t*   buf  = softbuf + (size_t)r * softbuf_stride;
    const int n    = oracle_ldpc_rm_rx_c(in, buf, E, t->F, t->bg, Z, rv, t->Qm, t->Nref);
    uint32_t  poly = t->L_tb == 24 ? CRC24A : CRC16;
    int       ord  = (int)t->L_tb;
    if (t->L_cb) {
      poly = CRC24B;
      ord  = 24;
    }
    const int ret = oracle_ldpc_decode_c(t->bg, (int)Z, ORACLE_LDPC_SCALE_SIMD, scaling, max_iter, buf, (uint32_t)n,
                                         poly, ord, msg);
    (void)nllr;
    iter_sum += ret == 0 ? (uint32_t)max_iter : (uint32_t)ret;
    cb_crc[r] = ret != 0;
    if (cb_crc[r]) {
      const uint32_t cb_len = t->Kp - t->L_cb;
      uint8_t*       d      = cb_data + (size_t)r * cb_data_stride;
      /* srsran_bit_pack_vector: whole bytes, then the remaining bits MSB-aligned */
      for (uint32_t b = 0; b < (cb_len + 7) / 8; b++) {
        uint8_t v = 0;
        for (uint32_t q = 0; q < 8; q++) {
          const uint32_t i = 8 * b + q;
          v                = (uint8_t)((v << 1) | (i < cb_len ? (msg[i] & 1) : 0));
        }
        d[b] = v;
      }
      cb_ok++;
    }
    in += E;
  }
  *avg_iter = C ? (float)iter_sum / (float)C : NAN;
  free(msg);
  if (cb_ok != C) {
    return 0;
  }
  uint32_t off = 0, checksum2 = 0;
  for (uint32_t r = 0; r < C; r++) {
    uint32_t cb_len = t->Kp - t->L_cb;
    if (r == C - 1) {
      cb_len -= t->L_tb;
    }
    memcpy(payload + off, cb_data + (size_t)r * cb_data_stride, cb_len / 8);
    off += cb_len / 8;
    if (C > 1 && r == C - 1) {
      const uint8_t* d = cb_data + (size_t)r * cb_data_stride + cb_len / 8;
      for (uint32_t b = 0; b < t->L_tb / 8; b++) {
        checksum2 = (checksum2 << 8) | d[b];
      }
    }
  }
  if (C == 1) {
    *tb_crc = 1;
  } else {
    uint8_t* bits = malloc(t->A);
    for (uint32_t i = 0; i < t->A; i++) {
      bits[i] = (payload[i / 8] >> (7 - i % 8)) & 1;
    }
    const uint32_t checksum1 = crc_bits_msb(t->L_tb == 24 ? CRC24A : CRC16, (int)t->L_tb, bits, t->A);
    free(bits);
    *tb_crc = checksum1 == checksum2;
  }
  return 0;
}
