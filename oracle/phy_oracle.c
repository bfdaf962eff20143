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

/* ======================= MIMO predecoding (precoding.c, mat.c) =======================
 * The scalar ("gen") formulas of the CSI variants the PDSCH uses (pdsch.c:325 always
 * allocates q->csi, so srsran_predecoding_type takes the *_csi paths):
 *   PORT0  srsran_predecoding_single_csi       precoding.c:307-355
 *   CDD    srsran_predecoding_ccd_2x2_mmse_csi precoding.c:1043-1121 (even/odd CDD precoder)
 *   SM     srsran_predecoding_multiplex_2x2_mmse_csi precoding.c:1437-1540 (codebooks 0..2)
 *   2x2    srsran_mat_2x2_mmse_csi_gen         mat.c:63-109
 * Plain IEEE float, every complex op spelled out, no contraction (built with
 * -ffp-contract=off).  The reference's SIMD bodies use rcp_ps approximations; those agree
 * with this restatement to ~1e-3 relative (tests/test_phy_oracle.py). */
typedef struct {
  float r, i;
} cpx;
static cpx cadd(cpx a, cpx b) { return (cpx){a.r + b.r, a.i + b.i}; }
static cpx csub(cpx a, cpx b) { return (cpx){a.r - b.r, a.i - b.i}; }
static cpx cmul(cpx a, cpx b) { return (cpx){a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r}; }
static cpx cconj(cpx a) { return (cpx){a.r, -a.i}; }
static cpx cneg(cpx a) { return (cpx){-a.r, -a.i}; }
static cpx cscale(cpx a, float s) { return (cpx){a.r * s, a.i * s}; }
static cpx cmulj(cpx a) { return (cpx){-a.i, a.r}; }

static void mmse_csi_gen(cpx y0, cpx y1, cpx h00, cpx h01, cpx h10, cpx h11, cpx* x0, cpx* x1, float* csi0,
                         float* csi1, float noise, float norm)
{
  const cpx c00 = cconj(h00), c01 = cconj(h01), c10 = cconj(h10), c11 = cconj(h11);
  cpx       a00 = cadd(cmul(c00, h00), cmul(c10, h10));
  a00.r += noise;
  const cpx a01 = cadd(cmul(c00, h01), cmul(c10, h11));
  const cpx a10 = cadd(cmul(c01, h00), cmul(c11, h10));
  cpx       a11 = cadd(cmul(c01, h01), cmul(c11, h11));
  a11.r += noise;
  const cpx   det = csub(cmul(a00, a11), cmul(a01, a10));
  const float den = det.r * det.r + det.i * det.i;
  const cpx   rcp = {det.r / den, -det.i / den};
  const cpx   nrm = cscale(rcp, norm);
  const cpx   b00 = cmul(a11, nrm), b01 = cmul(cneg(a01), nrm), b10 = cmul(cneg(a10), nrm), b11 = cmul(a00, nrm);
  const cpx   w00 = cadd(cmul(b00, c00), cmul(b01, c01));
  const cpx   w01 = cadd(cmul(b00, c10), cmul(b01, c11));
  const cpx   w10 = cadd(cmul(b10, c00), cmul(b11, c01));
  const cpx   w11 = cadd(cmul(b10, c10), cmul(b11, c11));
  *x0             = cadd(cmul(y0, w00), cmul(y1, w01));
  *x1             = cadd(cmul(y0, w10), cmul(y1, w11));
  *csi0           = 1.0f / b00.r;
  *csi1           = 1.0f / b11.r;
}

/* y[rx][n], h[port][rx][n] (port-major, then rx), x[layer][n], csi[layer][n]; cf32 interleaved.
 * scheme: 0 PORT0, 3 CDD, 2 SPATIALMUX (srsran_tx_scheme_t). */
int oracle_predecode(int          scheme,
                     int          nrx,
                     int          nports,
                     int          nlayers,
                     int          codebook,
                     const float* y,
                     const float* h,
                     float*       x,
                     float*       csi,
                     int          n,
                     float        scaling,
                     float        noise)
{
  const cpx* Y = (const cpx*)y;
  const cpx* H = (const cpx*)h;
  cpx*       X = (cpx*)x;
#define HH(p, r, k) H[((size_t)(p)*nrx + (r)) * n + (k)]
  if (scheme == 0) {
    if (nports != 1 || nlayers != 1) {
      return -1;
    }
    const float norm = 1.0f / scaling;
    for (int k = 0; k < n; k++) {
      cpx   r  = {0, 0};
      float hh = 0;
      for (int p = 0; p < nrx; p++) {
        const cpx hv = HH(0, p, k);
        r            = cadd(r, cmul(Y[(size_t)p * n + k], cconj(hv)));
        hh += hv.r * hv.r + hv.i * hv.i;
      }
      csi[k] = hh + noise;
      const cpx t = cscale(r, norm);
      X[k]        = (cpx){t.r / csi[k], t.i / csi[k]};
    }
    return 0;
  }
  if (nrx != 2 || nports != 2 || nlayers != 2) {
    return -1;
  }
  float norm;
  if (scheme == 3) {
    norm = 2.0f / scaling;
  } else if (scheme == 2) {
    if (codebook == 0) {
      norm = (float)1.41421356237309504880 / scaling;
    } else if (codebook == 1 || codebook == 2) {
      norm = 2.0f / scaling;
    } else {
      return -1;
    }
  } else {
    return -1;
  }
  for (int k = 0; k < n; k++) {
    const cpx a = HH(0, 0, k), b = HH(0, 1, k), c = HH(1, 0, k), d = HH(1, 1, k); /* h[port][rx] */
    cpx       h00, h01, h10, h11;
    if (scheme == 3) {
      if ((k & 1) == 0) {
        h00 = cadd(a, c);
        h10 = cadd(b, d);
        h01 = csub(a, c);
        h11 = csub(b, d);
      } else {
        h00 = csub(a, c);
        h10 = csub(b, d);
        h01 = cadd(a, c);
        h11 = cadd(b, d);
      }
    } else if (codebook == 0) {
      h00 = a;
      h01 = c;
      h10 = b;
      h11 = d;
    } else if (codebook == 1) {
      h00 = cadd(a, c);
      h01 = csub(a, c);
      h10 = cadd(b, d);
      h11 = csub(b, d);
    } else {
      h00 = cadd(a, cmulj(c));
      h01 = csub(a, cmulj(c));
      h10 = cadd(b, cmulj(d));
      h11 = csub(b, cmulj(d));
    }
    mmse_csi_gen(Y[k], Y[(size_t)n + k], h00, h01, h10, h11, &X[k], &X[(size_t)n + k], &csi[k], &csi[(size_t)n + k],
                 noise, norm);
  }
#undef HH
  return 0;
}

/* ======================= CSI correction (pdsch.c:523-618), SSE build =======================
 * e: nof_bits int16 LLRs (after descrambling), csi: nof_bits/qm values of the codeword.
 * Reproduces the SSE body exactly, including _mm_blend_ps(.., 3) handing the two symbols of a
 * QPSK/64QAM pair each other's CSI on the middle lanes, _mm_cvtps_pi16 (round-half-even,
 * saturate) and _mm_mulhi_pi16; the scalar tail truncates (float)e * (csi / csi_max). */
static int16_t cvt_pi16(float x) { return sat16(cvt_rn(x)); }
static int16_t mulhi16(int16_t a, int16_t b) { return (int16_t)(((int32_t)a * (int32_t)b) >> 16); }

void oracle_csi_correction(int mod, const float* csi, int16_t* e, uint32_t nof_bits)
{
  const uint32_t qm = (uint32_t[]){1, 2, 4, 6, 8}[mod];
  const uint32_t ns = nof_bits / qm;
  float          mx = 1.0f;
  if (ns) {
    mx = csi[0];
    for (uint32_t k = 1; k < ns; k++) {
      mx = csi[k] > mx ? csi[k] : mx;
    }
  }
  const float scale = 32767 / mx;
  int64_t     i     = 0;
  uint32_t    s     = 0;
  switch (mod) {
    case 1:
      for (; i < (int64_t)nof_bits - 3; i += 4, s += 2) {
        const int16_t c0 = cvt_pi16(csi[s] * scale), c1 = cvt_pi16(csi[s + 1] * scale);
        const int16_t c[4] = {c1, c1, c0, c0};
        for (int k = 0; k < 4; k++) {
          e[i + k] = mulhi16(e[i + k], c[k]);
        }
      }
      break;
    case 2:
      for (; i < (int64_t)nof_bits - 3; i += 4, s++) {
        const int16_t c = cvt_pi16(csi[s] * scale);
        for (int k = 0; k < 4; k++) {
          e[i + k] = mulhi16(e[i + k], c);
        }
      }
      break;
    case 3:
      for (; i < (int64_t)nof_bits - 11; i += 12, s += 2) {
        const int16_t c1 = cvt_pi16(csi[s] * scale), c3 = cvt_pi16(csi[s + 1] * scale);
        const int16_t c[12] = {c1, c1, c1, c1, c3, c3, c1, c1, c3, c3, c3, c3};
        for (int k = 0; k < 12; k++) {
          e[i + k] = mulhi16(e[i + k], c[k]);
        }
      }
      break;
    case 4:
      for (; i < (int64_t)nof_bits - 7; i += 8, s++) {
        const int16_t c = cvt_pi16(csi[s] * scale);
        for (int k = 0; k < 8; k++) {
          e[i + k] = mulhi16(e[i + k], c);
        }
      }
      break;
    default:
      break;
  }
  for (uint32_t k = (uint32_t)(i / qm); k < ns; k++) {
    const float c = csi[k] / mx;
    for (uint32_t b = 0; b < qm; b++) {
      e[qm * k + b] = wrap16(cvt_tz((float)e[qm * k + b] * c));
    }
  }
}
