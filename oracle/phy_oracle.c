/*
 * oracle/phy_oracle.c -- CPU restatement of the PDSCH LLR stages (TEST INFRASTRUCTURE ONLY:
 * imported by tests/ and bench.py's cpu_baseline, never by the product library).
 *
 *   oracle_demod_soft_s     srsran_demod_soft_demodulate_s (modem/demod_soft.c:871-894) as built
 *                           for x86 with SSE/AVX2 (the reference's release flags, oracle/Makefile):
 *                           - BPSK  demod_bpsk_lte_s   (demod_soft.c:96-101)      scalar, truncating
 *                           - QPSK  demod_qpsk_lte_s   (demod_soft.c:115-118) -> srsran_vec_convert_fi_simd
 *                                   (vector_simd.c:436-472): blocks of 16 values truncate + saturate
 *                                   (simd.h:1866-1871, AVX2 _mm256_cvttps_epi32/_mm256_packs_epi32),
 *                                   the tail truncates + wraps
 *                           - 16QAM demod_16qam_lte_s_sse (demod_soft.c:250-299): blocks of 4 symbols
 *                                   round half-even + saturate, the tail truncates
 *                           - 64QAM demod_64qam_lte_s_sse (demod_soft.c:569-644): same split
 *                           - 256QAM demod_256qam_lte_s (demod_soft.c:824-844)  scalar float
 *   oracle_sequence_apply_s srsran_sequence_apply_s (common/sequence.c:507-561): LTE Gold sequence
 *                           (36.211 7.2, Nc = 1600), LLR negated (int16 wrap) where c(n) = 1
 *   oracle_pdsch_seed       sequence_pdsch_seed (phch/sequences.c:62-65)
 * Pinned against the reference compiled into oracle/_ref (tests/test_phy_oracle.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "phy_oracle.h"

static int16_t sat16(int32_t v) { return v > 32767 ? 32767 : (v < -32768 ? -32768 : (int16_t)v); }

/* x86 float -> int32 conversions: out-of-range gives INT32_MIN ("integer indefinite") */
static int32_t cvt_rn(float x)
{
  if (!(x >= -2147483648.0f && x < 2147483648.0f)) {
    return INT32_MIN;
  }
  return (int32_t)nearbyintf(x); /* default rounding mode: to nearest, ties to even */
}
static int32_t cvt_tz(float x)
{
  if (!(x >= -2147483648.0f && x < 2147483648.0f)) {
    return INT32_MIN;
  }
  return (int32_t)x;
}
static int32_t cvt_tz_d(double x)
{
  if (!(x >= -2147483648.0 && x < 2147483648.0)) {
    return INT32_MIN;
  }
  return (int32_t)x;
}
static int16_t abs16(int16_t v) { return (int16_t)(v < 0 ? (uint16_t)(-(int32_t)v) : (uint16_t)v); } /* _mm_abs_epi16 */
static int16_t wrap16(int32_t v) { return (int16_t)(uint16_t)(uint32_t)v; }

int oracle_demod_soft_s(int mod, const float* sym, int16_t* llr, int n)
{
  switch (mod) {
    case 0: /* BPSK */
      for (int i = 0; i < n; i++) {
        const float t = -100.0f * (sym[2 * i] + sym[2 * i + 1]);
        llr[i]        = wrap16(cvt_tz_d((double)t * 0.70710678118654752440));
      }
      return 0;
    case 1: { /* QPSK: scale = (float)(-100 * M_SQRT2) */
      const float scale = (float)(-100.0 * 1.41421356237309504880);
      const int   len   = 2 * n;
      int         i     = 0;
      for (; i + 16 <= len; i += 16) {
        for (int k = 0; k < 16; k++) {
          llr[i + k] = sat16(cvt_tz(sym[i + k] * scale));
        }
      }
      for (; i < len; i++) {
        llr[i] = wrap16(cvt_tz(sym[i] * scale));
      }
      return 0;
    }
    case 2: { /* 16QAM */
      const int16_t off  = (int16_t)(2 * 400 / sqrtf(10));
      const int     nsse = 4 * (n / 4);
      for (int i = 0; i < nsse; i++) {
        const int16_t re = sat16(cvt_rn(sym[2 * i] * -400.0f));
        const int16_t im = sat16(cvt_rn(sym[2 * i + 1] * -400.0f));
        llr[4 * i + 0]   = re;
        llr[4 * i + 1]   = im;
        llr[4 * i + 2]   = wrap16(abs16(re) - off);
        llr[4 * i + 3]   = wrap16(abs16(im) - off);
      }
      const float offf = 2 * 400 / sqrtf(10);
      for (int i = nsse; i < n; i++) {
        const int16_t yre = wrap16(cvt_tz(400.0f * sym[2 * i]));
        const int16_t yim = wrap16(cvt_tz(400.0f * sym[2 * i + 1]));
        llr[4 * i + 0]    = wrap16(-(int32_t)yre);
        llr[4 * i + 1]    = wrap16(-(int32_t)yim);
        llr[4 * i + 2]    = wrap16(cvt_tz((float)abs(yre) - offf));
        llr[4 * i + 3]    = wrap16(cvt_tz((float)abs(yim) - offf));
      }
      return 0;
    }
    case 3: { /* 64QAM */
      const int16_t off1 = (int16_t)(4 * 700 / sqrtf(42));
      const int16_t off2 = (int16_t)(2 * 700 / sqrtf(42));
      const int     nsse = 4 * (n / 4);
      for (int i = 0; i < nsse; i++) {
        for (int c = 0; c < 2; c++) {
          const int16_t s = sat16(cvt_rn(sym[2 * i + c] * -700.0f));
          const int16_t a = wrap16(abs16(s) - off1);
          llr[6 * i + c]     = s;
          llr[6 * i + 2 + c] = a;
          llr[6 * i + 4 + c] = wrap16(abs16(a) - off2);
        }
      }
      for (int i = nsse; i < n; i++) {
        for (int c = 0; c < 2; c++) {
          const int16_t y = wrap16(cvt_tz(700.0f * sym[2 * i + c]));
          const int16_t a = wrap16((int16_t)abs(y) - off1);
          llr[6 * i + c]     = wrap16(-(int32_t)y);
          llr[6 * i + 2 + c] = a;
          llr[6 * i + 4 + c] = wrap16((int16_t)abs(a) - off2);
        }
      }
      return 0;
    }
    case 4: { /* 256QAM */
      const float t1 = 8.0f / sqrtf(170.0f), t2 = 4.0f / sqrtf(170.0f), t3 = 2.0f / sqrtf(170.0f);
      for (int i = 0; i < n; i++) {
        float re = -sym[2 * i], im = -sym[2 * i + 1];
        int16_t* o = &llr[8 * i];
        o[0]       = wrap16(cvt_tz(1000 * re));
        o[1]       = wrap16(cvt_tz(1000 * im));
        re         = fabsf(re) - t1;
        im         = fabsf(im) - t1;
        o[2]       = wrap16(cvt_tz(1000 * re));
        o[3]       = wrap16(cvt_tz(1000 * im));
        re         = fabsf(re) - t2;
        im         = fabsf(im) - t2;
        o[4]       = wrap16(cvt_tz(1000 * re));
        o[5]       = wrap16(cvt_tz(1000 * im));
        re         = fabsf(re) - t3;
        im         = fabsf(im) - t3;
        o[6]       = wrap16(cvt_tz(1000 * re));
        o[7]       = wrap16(cvt_tz(1000 * im));
      }
      return 0;
    }
    default:
      return -1;
  }
}

/* ---- LTE Gold sequence (36.211 7.2): state bit i = x(n + i), new bit into bit 30 ---- */
static uint32_t step_x1(uint32_t s) { return (s >> 1) ^ (((s ^ (s >> 3)) & 1u) << 30); }
static uint32_t step_x2(uint32_t s) { return (s >> 1) ^ (((s ^ (s >> 1) ^ (s >> 2) ^ (s >> 3)) & 1u) << 30); }

void oracle_sequence_bits(uint32_t seed, uint8_t* c, uint32_t len)
{
  uint32_t x1 = 1, x2 = seed & 0x7FFFFFFFu;
  for (int n = 0; n < 1600; n++) {
    x1 = step_x1(x1);
    x2 = step_x2(x2);
  }
  for (uint32_t i = 0; i < len; i++) {
    c[i] = (uint8_t)((x1 ^ x2) & 1u);
    x1   = step_x1(x1);
    x2   = step_x2(x2);
  }
}

void oracle_sequence_apply_s(const int16_t* in, int16_t* out, uint32_t len, uint32_t seed)
{
  uint32_t x1 = 1, x2 = seed & 0x7FFFFFFFu;
  for (int n = 0; n < 1600; n++) {
    x1 = step_x1(x1);
    x2 = step_x2(x2);
  }
  for (uint32_t i = 0; i < len; i++) {
    out[i] = ((x1 ^ x2) & 1u) ? wrap16(-(int32_t)in[i]) : in[i];
    x1     = step_x1(x1);
    x2     = step_x2(x2);
  }
}

uint32_t oracle_pdsch_seed(uint16_t rnti, int q, uint32_t nslot, uint32_t cell_id)
{
  return ((uint32_t)rnti << 14) + ((uint32_t)q << 13) + ((nslot / 2) << 9) + cell_id;
}
