/*
 * oracle/sch_oracle.c -- CPU restatement of srsRAN_4G's DL-SCH receive pieces.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker for the HIP DL-SCH path).
 *
 * Restated (paths relative to /root/reference/lib):
 *  - CRC table + byte-wise checksum      src/phy/fec/crc.c:30-48, 117-128, 189-195;
 *                                        include/srsran/phy/fec/crc.h:57-76
 *  - code-block segmentation             src/phy/fec/cbsegm.c:45-117
 *  - turbo rate de-matching table        src/phy/fec/turbo/rm_turbo.c:175-248 (36.212 5.1.4.1)
 *    + sub-block layout remap            rm_turbo.c:249-273
 *  - rx_lut (HARQ combine, int16 wrap)   rm_turbo.c:390-445 (AVX variant 707-811 is
 *                                        equivalent to the scalar loop at 437-439)
 *  - decode_tb / decode_tb_cb            src/phy/phch/sch.c:371-573 (CB E-length
 *    quirk at 404-407, min 2 half-its, CRC early stop, TB CRC, cb_crc bookkeeping)
 *  - rate matching TX (for synthetic TBs) rm_turbo.c srsran_rm_turbo_tx (36.212 5.1.4.1)
 *
 * Pinning: rx tables / rx_lut, CRC and cbsegm are checked against the reference
 * compiled from /root/reference (oracle/_ref) in tests/test_sch_oracle.py.  sch.c
 * itself is not buildable here (it includes srsran/srsran.h -> generated
 * srsran/version.h), so the decode_tb loop is a restatement built only from pinned
 * pieces; see DESIGN.md.
 */
#include "sch_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "tdec_oracle.h"

/* ---------------- CRC ---------------- */
void oracle_crc_table(uint32_t poly, int order, uint32_t table[256])
{
  const uint32_t pad        = order < 8 ? 8 - order : 0;
  const uint32_t ord        = order + pad - 8;
  const uint64_t polynom    = (uint64_t)poly << pad;
  const uint64_t crchighbit = ((uint64_t)1 << (order - 1)) << pad;
  const uint64_t mask       = ((((uint64_t)1 << (order - 1)) - 1) << 1) | 1;
  for (uint32_t i = 0; i < 256; i++) {
    uint64_t crc = (uint64_t)i << ord;
    for (int j = 0; j < 8; j++) {
      const int bit = (crc & crchighbit) != 0;
      crc <<= 1;
      if (bit) {
        crc ^= polynom;
      }
    }
    table[i] = (uint32_t)((crc >> pad) & mask);
  }
}

uint32_t oracle_crc_checksum_byte(uint32_t poly, int order, const uint8_t* data, uint32_t nbits)
{
  uint32_t table[256];
  oracle_crc_table(poly, order, table);
  const uint64_t mask = ((((uint64_t)1 << (order - 1)) - 1) << 1) | 1;
  uint64_t       crc  = 0;
  for (uint32_t i = 0; i < nbits / 8; i++) {
    uint32_t idx = order > 8 ? (uint32_t)((crc >> (order - 8)) & 0xff) ^ data[i]
                             : (uint32_t)((crc << (8 - order)) & 0xff) ^ data[i];
    crc          = (crc << 8) ^ table[idx];
  }
  return (uint32_t)(crc & mask);
}

/* ---------------- cbsegm ---------------- */
int oracle_cbsegm(uint32_t tbs, oracle_cbsegm_t* s)
{
  memset(s, 0, sizeof(*s));
  if (tbs == 0) {
    return 0;
  }
  const uint32_t B = tbs + 24, Z = 6144;
  uint32_t       Bp;
  s->tbs = tbs;
  if (B <= Z) {
    s->C = 1;
    Bp   = B;
  } else {
    s->C = (B + (Z - 24) - 1) / (Z - 24);
    Bp   = B + 24 * s->C;
  }
  /* cbindex: first table size >= ceil(Bp/C) (cbsegm.c:119-131) */
  uint32_t need = (Bp - 1) / s->C + 1;
  int      idx1 = -1;
  for (int i = 0; i < 188; i++) {
    if (oracle_cb_size(i) >= need) {
      idx1 = i;
      break;
    }
  }
  if (idx1 < 0) {
    return -1;
  }
  s->K1     = oracle_cb_size(idx1);
  s->K1_idx = idx1;
  if (s->C == 1) {
    s->K2 = 0;
    s->K2_idx = 0;
    s->C2 = 0;
    s->C1 = 1;
  } else {
    s->K2     = idx1 > 0 ? oracle_cb_size(idx1 - 1) : s->K1;
    s->K2_idx = idx1 > 0 ? idx1 - 1 : 0;
    s->C2     = (s->C * s->K1 - Bp) / (s->K1 - s->K2);
    s->C1     = s->C - s->C2;
  }
  s->F = s->C1 * s->K1 + s->C2 * s->K2 - Bp;
  return 0;
}

/* ---------------- rate de-matching (36.212 5.1.4.1) ---------------- */
static const uint8_t P_TC[32] = {0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30,
                                 1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31};

/*
 * table[k] (k < 3K+12): decoder-input index of the k-th non-dummy bit of the
 * circular buffer read from k0(rv).  layout_sb selects the sub-block remap applied
 * for window decoders (rm_turbo.c:249-273): 1 the 16-bit decoder's sub-blocks, 2 the 8-bit decoder's
 * (rm_turbo_rx_lut_8bit); natural index of d^(j)_i is 3i+j.
 */
int oracle_rm_rx_table(uint32_t K, uint32_t rv, int layout_sb, uint16_t* table)
{
  const uint32_t D = K + 4, R = (D + 31) / 32, Kp = 32 * R, ND = Kp - D, Ncb = 3 * Kp;
  const uint32_t k0 = R * (2 * ((Ncb + 8 * R - 1) / (8 * R)) * rv + 2);
  const uint32_t out_len = 3 * K + 12;
  const uint32_t nsb     = layout_sb == 2 ? oracle_nof_subblocks_8bit(K) : layout_sb ? oracle_nof_subblocks(K) : 0;
  uint32_t       k = 0, jj = 0;
  while (k < out_len) {
    const uint32_t w = (k0 + jj) % Ncb;
    jj++;
    int32_t  y;
    uint32_t stream;
    if (w < Kp) {
      stream = 0;
      y      = P_TC[w / R] + 32 * (w % R);
    } else if (((w - Kp) & 1) == 0) {
      const uint32_t kk = (w - Kp) / 2;
      stream            = 1;
      y                 = P_TC[kk / R] + 32 * (kk % R);
    } else {
      const uint32_t kk = (w - Kp - 1) / 2;
      stream            = 2;
      y                 = (P_TC[kk / R] + 32 * (kk % R) + 1) % Kp;
    }
    const int32_t i = y - (int32_t)ND;
    if (i < 0) {
      continue; /* dummy (NULL) bit */
    }
    uint32_t n = 3 * (uint32_t)i + stream;
    if (nsb) {
      if (n < 3 * K) {
        const uint32_t L = K / nsb, x = n / 3;
        n                = (n % 3) * (K + 32) + (x % L) * nsb + x / L;
      } else {
        n = (n - 3 * K) + 3 * (K + 32);
      }
    }
    table[k++] = (uint16_t)n;
  }
  return 0;
}

int oracle_rm_turbo_rx(uint32_t K, uint32_t rv, int layout_sb, const int16_t* in, uint32_t E, int16_t* softbuf)
{
  const uint32_t out_len = 3 * K + 12;
  uint16_t*      t       = malloc(out_len * sizeof(uint16_t));
  oracle_rm_rx_table(K, rv, layout_sb, t);
  for (uint32_t i = 0; i < E; i++) {
    softbuf[t[i % out_len]] = (int16_t)(softbuf[t[i % out_len]] + in[i]);
  }
  free(t);
  return 0;
}

/* TX: coded bits (natural 3K+12 from the turbo encoder) -> E rate-matched bits. */
int oracle_rm_turbo_tx(uint32_t K, uint32_t rv, const uint8_t* coded, uint32_t E, uint8_t* out)
{
  const uint32_t out_len = 3 * K + 12;
  uint16_t*      t       = malloc(out_len * sizeof(uint16_t));
  oracle_rm_rx_table(K, rv, 0, t);
  for (uint32_t i = 0; i < E; i++) {
    out[i] = coded[t[i % out_len]];
  }
  free(t);
  return 0;
}

/* ---------------- DL-SCH decode_tb (sch.c:371-573) ---------------- */
#define LTE_CRC24A 0x1864CFB
#define LTE_CRC24B 0x1800063

/* The decoder's output after each of max_iterations half-iterations (natural order, int16) for code block K of
 * soft buffer row sb: the 16-bit AUTO decoder, or with llr8 the 8-bit one (rows holding int8 LLRs in the 8-bit
 * layout, as buffer_f[cb] cast to int8_t* in sch.c:409-428).  Where no 8-bit decoder takes K (K <= 800) the
 * reference widens the input for a 16-bit decoder (convert_8_to_16, turbodecoder.c:470-481); the whole layout is
 * widened here (the reference converts only 3K + 12 values and leaves the rest of its sub-block layout buffer
 * stale -- see DESIGN.md). */
static void tdec_trace(uint32_t K, const int16_t* sb, int llr8, uint32_t max_iterations, int16_t* trace)
{
  uint8_t tmp[768];
  if (!llr8) {
    oracle_tdec_run(K, sb, 1, max_iterations, tmp, trace);
    return;
  }
  const int8_t*  sb8  = (const int8_t*)sb;
  const uint32_t nsb8 = oracle_nof_subblocks_8bit(K);
  if (nsb8 >= 16) {
    int8_t* t8 = malloc((size_t)max_iterations * K);
    oracle_tdec8_run(K, sb8, max_iterations, tmp, t8);
    for (size_t i = 0; i < (size_t)max_iterations * K; i++) {
      trace[i] = t8[i];
    }
    free(t8);
    return;
  }
  const uint32_t n    = nsb8 ? 3 * (K + 32) + 12 : 3 * K + 12;
  int16_t*       wide = calloc(3 * (K + 32) + 12, sizeof(int16_t));
  for (uint32_t i = 0; i < n; i++) {
    wide[i] = sb8[i];
  }
  oracle_tdec_run(K, wide, 1, max_iterations, tmp, trace);
  free(wide);
}

static int decode_tb(uint32_t       tbs,
                     uint32_t       Qm,
                     uint32_t       rv,
                     uint32_t       nof_e_bits,
                     const void*    e_bits,
                     int            llr8,
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
  oracle_cbsegm_t s;
  if (oracle_cbsegm(tbs, &s)) {
    return -1;
  }
  if (s.tbs == 0 || s.C == 0) {
    return 0;
  }
  if (s.F) {
    return -2;
  }
  if (s.C > 32) { /* SRSRAN_MAX_CODEBLOCKS (sch.c:383-386) */
    return -1;
  }
  float avg = 0;
  for (uint32_t cb = 0; cb < s.C; cb++) {
    const uint32_t cb_len = cb < s.C1 ? s.K1 : s.K2;
    const uint32_t rlen   = s.C == 1 ? cb_len : cb_len - 24;
    if (!cb_crc[cb]) {
      const uint32_t Gp    = nof_e_bits / Qm;
      const uint32_t gamma = Gp % s.C;
      const uint32_t n_e   = Qm * (Gp / s.C);
      uint32_t       rp    = cb * n_e;
      uint32_t       n_e2  = n_e;
      if (cb > s.C - gamma) { /* sch.c:404-407: '>' not '>='  */
        n_e2 = n_e + Qm;
        rp   = (s.C - gamma) * n_e + (cb - (s.C - gamma)) * n_e2;
      }
      int16_t* sb = &softbuf[(size_t)cb * softbuf_stride];
      if (llr8) { /* srsran_rm_turbo_rx_lut_8bit: int8 wrap-around on the 8-bit decoder's layout */
        uint16_t*     t  = malloc((3 * cb_len + 12) * sizeof(uint16_t));
        int8_t*       s8 = (int8_t*)sb;
        const int8_t* e8 = (const int8_t*)e_bits + rp;
        oracle_rm_rx_table(cb_len, rv, 2, t);
        for (uint32_t i = 0; i < n_e2; i++) {
          const uint16_t p = t[i % (3 * cb_len + 12)];
          s8[p]            = (int8_t)(s8[p] + e8[i]);
        }
        free(t);
      } else {
        oracle_rm_turbo_rx(cb_len, rv, 1, (const int16_t*)e_bits + rp, n_e2, sb);
      }

      /* iterations with early stop: decision after every half-iteration */
      int16_t* trace = malloc((size_t)max_iterations * cb_len * sizeof(int16_t));
      tdec_trace(cb_len, sb, llr8, max_iterations, trace);
      uint32_t noi   = 0;
      int      early = 0;
      uint8_t  dec[768];
      do {
        const int16_t* row = &trace[(size_t)noi * cb_len];
        for (uint32_t b = 0; b < cb_len / 8; b++) {
          uint8_t v = 0;
          for (int t = 0; t < 8; t++) {
            v |= (uint8_t)((row[8 * b + t] > 0) << (7 - t));
          }
          dec[b] = v;
        }
        memcpy(&data[cb * rlen / 8], dec, cb_len / 8);
        avg += 1;
        noi++;
        const uint32_t len_crc = s.C > 1 ? cb_len : s.tbs + 24;
        const uint32_t poly    = s.C > 1 ? LTE_CRC24B : LTE_CRC24A;
        if (!oracle_crc_checksum_byte(poly, 24, &data[cb * rlen / 8], len_crc) && noi >= 2) {
          cb_crc[cb] = 1;
          early      = 1;
        }
      } while (noi < max_iterations && !early);
      free(trace);
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
  int tb_ok = 1;
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
  if (oracle_crc_checksum_byte(LTE_CRC24A, 24, data, s.tbs + 24) == 0) {
    return 0;
  }
  memset(cb_crc, 0, s.C); /* srsran_softbuffer_rx_reset_cb_crc */
  return -1;
}

int oracle_dlsch_decode_tb(uint32_t tbs, uint32_t Qm, uint32_t rv, uint32_t nof_e_bits, const int16_t* e_bits,
                           uint32_t max_iterations, int16_t* softbuf, uint32_t softbuf_stride, uint8_t* cb_crc,
                           uint8_t* cb_data, uint32_t cb_data_stride, uint8_t* data, uint32_t* cb_noi_out,
                           float* avg_iterations)
{
  return decode_tb(tbs, Qm, rv, nof_e_bits, e_bits, 0, max_iterations, softbuf, softbuf_stride, cb_crc, cb_data,
                   cb_data_stride, data, cb_noi_out, avg_iterations);
}

/* decode_tb with q->llr_is_8bit (sch.c:409-428): int8 e bits, srsran_rm_turbo_rx_lut_8bit into the soft buffer rows
 * (int16 rows used as int8), srsran_tdec_iteration_8bit */
int oracle_dlsch_decode_tb8(uint32_t tbs, uint32_t Qm, uint32_t rv, uint32_t nof_e_bits, const int8_t* e_bits,
                            uint32_t max_iterations, int16_t* softbuf, uint32_t softbuf_stride, uint8_t* cb_crc,
                            uint8_t* cb_data, uint32_t cb_data_stride, uint8_t* data, uint32_t* cb_noi_out,
                            float* avg_iterations)
{
  return decode_tb(tbs, Qm, rv, nof_e_bits, e_bits, 1, max_iterations, softbuf, softbuf_stride, cb_crc, cb_data,
                   cb_data_stride, data, cb_noi_out, avg_iterations);
}

/* ---------------- DL-SCH encode (synthetic TBs; sch.c encode_tb semantics, K- first) ---------------- */
int oracle_dlsch_encode_tb(uint32_t tbs, uint32_t Qm, uint32_t rv, uint32_t nof_e_bits, const uint8_t* tb_bytes, uint8_t* e_bits)
{
  return oracle_dlsch_encode_tb_x(tbs, Qm, rv, nof_e_bits, tb_bytes, e_bits, 0);
}

/* tb_crc_xor != 0 corrupts the TB CRC24A before CB segmentation: every CB CRC then passes
 * while the TB CRC fails (exercises sch.c:558-570). */
int oracle_dlsch_encode_tb_x(uint32_t       tbs,
                             uint32_t       Qm,
                             uint32_t       rv,
                             uint32_t       nof_e_bits,
                             const uint8_t* tb_bytes,
                             uint8_t*       e_bits,
                             uint32_t       tb_crc_xor)
{
  oracle_cbsegm_t s;
  if (oracle_cbsegm(tbs, &s) || s.F) {
    return -1;
  }
  /* TB bits + CRC24A */
  uint8_t* tb = malloc(tbs / 8 + 3);
  memcpy(tb, tb_bytes, tbs / 8);
  uint32_t crc = oracle_crc_checksum_byte(LTE_CRC24A, 24, tb, tbs) ^ tb_crc_xor;
  tb[tbs / 8]     = (uint8_t)(crc >> 16);
  tb[tbs / 8 + 1] = (uint8_t)(crc >> 8);
  tb[tbs / 8 + 2] = (uint8_t)crc;
  const uint32_t Gp = nof_e_bits / Qm, gamma = Gp % s.C;
  uint32_t       rp = 0, wp = 0;
  uint8_t        cbbytes[768 + 3], bits[6144], coded[3 * 6144 + 12];
  for (uint32_t i = 0; i < s.C; i++) {
    /* sch.c:285-290: the encoder places the C2 blocks of K2 first */
    const uint32_t cb_len = i < s.C2 ? s.K2 : s.K1;
    const uint32_t rlen   = s.C > 1 ? cb_len - 24 : cb_len;
    const uint32_t n_e    = i <= s.C - gamma - 1 ? Qm * (Gp / s.C) : Qm * ((Gp + s.C - 1) / s.C);
    if (s.C > 1) {
      memcpy(cbbytes, &tb[rp / 8], rlen / 8);
      crc                     = oracle_crc_checksum_byte(LTE_CRC24B, 24, cbbytes, rlen);
      cbbytes[rlen / 8]     = (uint8_t)(crc >> 16);
      cbbytes[rlen / 8 + 1] = (uint8_t)(crc >> 8);
      cbbytes[rlen / 8 + 2] = (uint8_t)crc;
    } else {
      memcpy(cbbytes, tb, cb_len / 8);
    }
    for (uint32_t b = 0; b < cb_len; b++) {
      bits[b] = (cbbytes[b / 8] >> (7 - b % 8)) & 1;
    }
    oracle_tcod_encode(cb_len, bits, coded);
    oracle_rm_turbo_tx(cb_len, rv, coded, n_e, &e_bits[wp]);
    rp += rlen;
    wp += n_e;
  }
  free(tb);
  return (int)wp;
}

/* Bit-serial CRC (polynomial remainder m(x)*x^order mod P, zero init): the quantity
 * srsran_crc_checksum computes for any bit length (crc.c:92-141). */
uint32_t oracle_crc_bits(uint32_t poly, int order, const uint8_t* bits, uint32_t nbits)
{
  const uint64_t top  = (uint64_t)1 << order;
  const uint64_t mask = top - 1;
  uint64_t       crc  = 0;
  for (uint32_t i = 0; i < nbits; i++) {
    const uint64_t fb = ((crc >> (order - 1)) & 1) ^ (bits[i] & 1);
    crc               = (crc << 1) & mask;
    if (fb) {
      crc ^= (poly & mask);
    }
  }
  return (uint32_t)crc;
}

/* ulsch_deinterleave (sch.c:994-1021) without RI bits: ulsch_interleave_gen (sch.c:661-682) numbers the
 * positions j Qm + i rows Qm + k in (row j, column i, bit k) order, srsran_vec_lut_sis (vector.c:147-152)
 * stores g[number] = q[position].  Positions past rows N_symb Qm are neither read nor written. */
void oracle_ulsch_deinterleave(const int16_t* q, int16_t* g, uint32_t Qm, uint32_t H_prime_total, uint32_t N_symb)
{
  const uint32_t rows = H_prime_total / N_symb;
  uint32_t       idx  = 0;
  for (uint32_t j = 0; j < rows; j++) {
    for (uint32_t i = 0; i < N_symb; i++) {
      for (uint32_t k = 0; k < Qm; k++) {
        g[idx++] = q[j * Qm + i * rows * Qm + k];
      }
    }
  }
}
