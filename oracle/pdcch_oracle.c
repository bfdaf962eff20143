/*
 * oracle/pdcch_oracle.c -- TEST INFRASTRUCTURE ONLY: plain-C restatement of the PDCCH candidate
 * decode that the GPU kernel (srsran_4g_amd/csrc/pdcch_kernel.hip) follows step for step.
 *
 *   rm_conv rx    fec/turbo/rm_conv.c:120-175 (srsran_rm_conv_rx, float soft combining)
 *   Viterbi       fec/convolutional/viterbi.c:546-585 (srsran_viterbi_decode_f: gain 500 / max|x|,
 *                 srsran_vec_quant_fus with the build's fused multiply-add), viterbi.c:129-157
 *                 (tail biting: 5 copies, middle one kept), viterbi37_avx2_16bit.c:176-313 (uint16
 *                 path metrics that wrap -- the renormalisation's byte shifts always find 0 --, modulo
 *                 compare, branch metric avg(avg(b0^s0, b1^s1), b2^s2) >> 3) and :105-131 (chainback
 *                 reading decisions 6 steps past the frame, which the update never wrote: zeros)
 *   CRC / RNTI    phch/pdcch.c:313-350 (srsran_pdcch_dci_decode), CRC16 0x11021
 * Pinned against the compiled reference (tests/test_pdcch_oracle.py).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define NCOLS 32
#define RX_NULL 10000.0f /* SRSRAN_RX_NULL (rm_conv.h) */
static const uint8_t PERM_CC[NCOLS] = {1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
                                       0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30};

/* 36.212 5.1.4.2: sub-block interleaver of the convolutional code; output[3i + j] */
void ora_rm_conv_rx(const float* in, uint32_t in_len, float* out, uint32_t out_len)
{
  uint8_t  inv[NCOLS];
  float    tmp[3 * NCOLS * 8];
  for (int i = 0; i < NCOLS; i++) {
    inv[PERM_CC[i]] = (uint8_t)i;
  }
  const int nrows  = (int)((out_len / 3 - 1) / NCOLS + 1);
  const int Kp     = nrows * NCOLS;
  int       ndummy = Kp - (int)(out_len / 3);
  if (ndummy < 0) {
    ndummy = 0;
  }
  for (int i = 0; i < 3 * Kp; i++) {
    tmp[i] = RX_NULL;
  }
  for (uint32_t k = 0, j = 0; k < in_len;) {
    const int di = (int)(j % Kp) / nrows, dj = (int)(j % Kp) % nrows;
    if (dj * NCOLS + PERM_CC[di] >= ndummy) {
      if (tmp[j] == RX_NULL) {
        tmp[j] = in[k];
      } else if (in[k] != RX_NULL) {
        tmp[j] += in[k];
      }
      k++;
    }
    if (++j == (uint32_t)(3 * Kp)) {
      j = 0;
    }
  }
  for (uint32_t i = 0; i < out_len / 3; i++) {
    const int di = (int)(i + ndummy) / NCOLS, dj = (int)(i + ndummy) % NCOLS;
    for (int j = 0; j < 3; j++) {
      const float o  = tmp[Kp * j + inv[dj] * nrows + di];
      out[i * 3 + j] = o != RX_NULL ? o : 0.0f;
    }
  }
}

static int parity(int x)
{
  x ^= x >> 16;
  x ^= x >> 8;
  x ^= x >> 4;
  x ^= x >> 2;
  x ^= x >> 1;
  return x & 1;
}

/* Tail-biting K = 7 rate-1/3 Viterbi decode of frame_length bits from 3 * frame_length floats. */
void ora_viterbi_decode_f(const float* x, uint32_t frame_length, uint8_t* data)
{
  static const int poly[3] = {0x6D, 0x4F, 0x57};
  const uint32_t   len     = 3 * frame_length;
  float            mx      = 0.0f;
  int              have    = 0;
  for (uint32_t i = 0; i < len; i++) {
    if (fabsf(x[i]) > mx) {
      mx   = fabsf(x[i]);
      have = 1;
    }
  }
  float max = 1e-9f;
  if (have && isnormal(mx)) {
    max = mx;
  }
  const float gain = 500.0f / max;
  uint16_t    sym[3 * 144];
  for (uint32_t i = 0; i < len; i++) {
    int32_t t = (int32_t)fmaf(gain, x[i], 32767.5f);
    t         = t < 0 ? 0 : (t > 65535 ? 65535 : t);
    sym[i]    = (uint16_t)t;
  }
  uint16_t bt[3][32];
  for (int s = 0; s < 32; s++) {
    for (int p = 0; p < 3; p++) {
      bt[p][s] = parity((2 * s) & poly[p]) ? 65535 : 0;
    }
  }
  const uint32_t nsteps = 5 * frame_length;
  static uint64_t dec[5 * 144 + 6];
  memset(dec, 0, sizeof(dec));
  uint16_t m[64], nm[64];
  for (int s = 0; s < 64; s++) {
    m[s] = 63;
  }
  for (uint32_t t = 0; t < nsteps; t++) {
    const uint16_t* y = &sym[3 * (t % frame_length)];
    uint64_t        d = 0;
    for (int s = 0; s < 32; s++) {
      const uint16_t a  = (uint16_t)(((bt[0][s] ^ y[0]) + (bt[1][s] ^ y[1]) + 1) >> 1);
      const uint16_t bm = (uint16_t)((((bt[2][s] ^ y[2]) + a + 1) >> 1) >> 3);
      const uint16_t mb = (uint16_t)(8191 - bm);
      const uint16_t m0 = (uint16_t)(m[s] + bm), m1 = (uint16_t)(m[s + 32] + mb);
      const uint16_t m2 = (uint16_t)(m[s] + mb), m3 = (uint16_t)(m[s + 32] + bm);
      const int      d0 = (int16_t)(uint16_t)(m0 - m1) > 0, d1 = (int16_t)(uint16_t)(m2 - m3) > 0;
      nm[2 * s]         = d0 ? m1 : m0;
      nm[2 * s + 1]     = d1 ? m3 : m2;
      d |= (uint64_t)d0 << (2 * s) | (uint64_t)d1 << (2 * s + 1);
    }
    dec[t] = d;
    memcpy(m, nm, sizeof(m));
  }
  /* chainback from the best state; decisions t >= nsteps are zero (viterbi37_avx2_16bit.c:112-131) */
  uint32_t best = 0;
  uint16_t mn   = 65535;
  for (uint32_t s = 0; s < 64; s++) {
    if (m[s] <= mn) {
      best = s;
      mn   = m[s];
    }
  }
  uint32_t st = best;
  for (int n = (int)nsteps - 1; n >= 0; n--) {
    const uint32_t k = (uint32_t)(dec[n + 6] >> st) & 1u;
    st               = (st >> 1) | (k << 5);
    if (n >= (int)(2 * frame_length) && n < (int)(3 * frame_length)) {
      data[n - 2 * frame_length] = (uint8_t)k;
    }
  }
}

/* srsran_pdcch_dci_decode on the E LLRs of a candidate: returns the CRC remainder (RNTI). */
uint16_t ora_pdcch_dci_decode(const float* e, uint32_t E, uint32_t nof_bits, uint8_t* data)
{
  float rm[3 * 144];
  memset(rm, 0, sizeof(rm));
  const uint32_t coded_len = 3 * (nof_bits + 16);
  ora_rm_conv_rx(e, E, rm, coded_len);
  ora_viterbi_decode_f(rm, nof_bits + 16, data);
  uint32_t crc = 0;
  for (uint32_t i = 0; i < nof_bits; i++) {
    const uint32_t fb = ((crc >> 15) & 1u) ^ data[i];
    crc               = (crc << 1) & 0xffffu;
    if (fb) {
      crc ^= 0x1021u;
    }
  }
  uint32_t p = 0;
  for (int i = 0; i < 16; i++) {
    p = (p << 1) | data[nof_bits + i];
  }
  return (uint16_t)(p ^ crc);
}
