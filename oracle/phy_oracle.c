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

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif
#ifndef M_1_PI
#define M_1_PI 0.31830988618379067154
#endif
#ifndef M_SQRT1_2
#define M_SQRT1_2 0.70710678118654752440
#endif
void sincosf(float x, float* s, float* c); /* glibc (GNU extension; -std=c11 hides the declaration) */

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
 *   TXD    srsran_predecoding_diversity_csi    precoding.c:671-700 (2 ports, SFBC pairs)
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
 * scheme: 0 PORT0, 1 DIVERSITY, 3 CDD, 2 SPATIALMUX (srsran_tx_scheme_t).  DIVERSITY writes n/2
 * symbols per layer and csi[0][0..n) (both REs of a pair get the pair's |h|^2 sum). */
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
  if (scheme == 1 && nports == 4) {
    /* srsran_predecoding_diversity_csi, 4 ports (precoding.c:714-775): SFBC + FSTD groups of 4 REs,
     * ports (0, 2) on REs 4i, 4i+1 and (1, 3) on 4i+2, 4i+3; m_ap groups (a trailing half group is
     * not decoded: those outputs stay 0 here); CSI a_k * scaling / nof_rxant per RE */
    if (nlayers != 4 || nrx < 1 || nrx > 4) {
      return -1;
    }
    const int m_ap = (n % 4) ? ((n - 2) / 4) : n / 4;
    memset(X, 0, sizeof(cpx) * (size_t)4 * n);
    memset(csi, 0, sizeof(float) * (size_t)n);
    for (int i = 0; i < m_ap; i++) {
      cpx   x0 = {0, 0}, x1 = {0, 0}, x2 = {0, 0}, x3 = {0, 0};
      float a0 = 0, a1 = 0, a2 = 0, a3 = 0;
      for (int p = 0; p < nrx; p++) {
        cpx h00 = HH(0, p, 4 * i), h01 = HH(2, p, 4 * i), h10 = HH(0, p, 4 * i + 1), h11 = HH(2, p, 4 * i + 1);
        a0 += h00.r * h00.r + h00.i * h00.i + h11.r * h11.r + h11.i * h11.i;
        a1 += h10.r * h10.r + h10.i * h10.i + h01.r * h01.r + h01.i * h01.i;
        const cpx r0 = Y[(size_t)p * n + 4 * i], r1 = Y[(size_t)p * n + 4 * i + 1];
        x0           = cadd(x0, cadd(cmul(cconj(h00), r0), cmul(h11, cconj(r1))));
        x1           = cadd(x1, cadd(cmul(cneg(h01), cconj(r0)), cmul(cconj(h10), r1)));
        h00          = HH(1, p, 4 * i + 2);
        h01          = HH(3, p, 4 * i + 2);
        h10          = HH(1, p, 4 * i + 3);
        h11          = HH(3, p, 4 * i + 3);
        a2 += h00.r * h00.r + h00.i * h00.i + h11.r * h11.r + h11.i * h11.i;
        a3 += h10.r * h10.r + h10.i * h10.i + h01.r * h01.r + h01.i * h01.i;
        const cpx r2 = Y[(size_t)p * n + 4 * i + 2], r3 = Y[(size_t)p * n + 4 * i + 3];
        x2           = cadd(x2, cadd(cmul(cconj(h00), r2), cmul(h11, cconj(r3))));
        x3           = cadd(x3, cadd(cmul(cneg(h01), cconj(r2)), cmul(cconj(h10), r3)));
      }
      const float a[4]  = {a0 * scaling, a1 * scaling, a2 * scaling, a3 * scaling};
      const cpx   xs[4] = {x0, x1, x2, x3};
      for (int l = 0; l < 4; l++) {
        csi[4 * i + l]             = a[l] / (float)nrx;
        X[(size_t)l * n + i] = (cpx){(float)((double)(xs[l].r / a[l]) * 1.41421356237309504880),
                                     (float)((double)(xs[l].i / a[l]) * 1.41421356237309504880)};
      }
    }
    return 0;
  }
  if (scheme == 1) {
    if (nports != 2 || nlayers != 2 || nrx < 1 || nrx > 4) {
      return -1;
    }
    for (int i = 0; i < n / 2; i++) {
      float hh = 0;
      cpx   x0 = {0, 0}, x1 = {0, 0};
      for (int p = 0; p < nrx; p++) {
        const cpx h00 = HH(0, p, 2 * i), h01 = HH(0, p, 2 * i + 1), h10 = HH(1, p, 2 * i), h11 = HH(1, p, 2 * i + 1);
        hh += h00.r * h00.r + h00.i * h00.i + h11.r * h11.r + h11.i * h11.i;
        const cpx r0 = Y[(size_t)p * n + 2 * i], r1 = Y[(size_t)p * n + 2 * i + 1];
        if (hh == 0) {
          hh = 1e-4f;
        }
        x0 = cadd(x0, cadd(cmul(cconj(h00), r0), cmul(h11, cconj(r1))));
        x1 = cadd(x1, cadd(cmul(cneg(h10), cconj(r0)), cmul(cconj(h01), r1)));
      }
      csi[2 * i]     = hh;
      csi[2 * i + 1] = hh;
      hh *= scaling;
      /* (x / hh) in float, then * M_SQRT2 in double (complex float * double), stored as float */
      X[i]                = (cpx){(float)((double)(x0.r / hh) * 1.41421356237309504880),
                                  (float)((double)(x0.i / hh) * 1.41421356237309504880)};
      X[(size_t)n + i]     = (cpx){(float)((double)(x1.r / hh) * 1.41421356237309504880),
                                   (float)((double)(x1.i / hh) * 1.41421356237309504880)};
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
  /* the release build (-Ofast: -freciprocal-math) hoists 1 / csi_max out of the loop and multiplies */
  const float rcp = 1.0f / mx;
  for (uint32_t k = (uint32_t)(i / qm); k < ns; k++) {
    const float c = csi[k] * rcp;
    for (uint32_t b = 0; b < qm; b++) {
      e[qm * k + b] = wrap16(cvt_tz((float)e[qm * k + b] * c));
    }
  }
}

/* ======================= 8-bit LLR chain (pdsch.c:691-737 with q->llr_is_8bit) =======================
 *   oracle_demod_soft_b      srsran_demod_soft_demodulate_b (demod_soft.c:896-919), x86 SSE build:
 *                            - BPSK  demod_bpsk_lte_b (demod_soft.c:89-94): scalar, truncating
 *                            - QPSK  demod_qpsk_lte_b -> srsran_vec_convert_fb_simd (vector_simd.c:524-589):
 *                                    16-value SSE blocks truncate + saturate (packs_epi32, packs_epi16), the tail
 *                                    truncates + wraps
 *                            - 16QAM demod_16qam_lte_b_sse (demod_soft.c:301-364): 8-symbol blocks round half-even +
 *                                    saturate to int8; abs_epi8 / sub_epi8 wrap (|-128| = -128, offset (int8)18.97);
 *                                    the tail truncates and subtracts the float offset
 *                            - 64QAM demod_64qam_lte_b_sse (demod_soft.c:650-730): same split, offsets 24 and 12
 *                            - 256QAM demod_256qam_lte_b (demod_soft.c:800-822): scalar float, truncating
 *   oracle_sequence_apply_c  srsran_sequence_state_apply_c (sequence.c:563-618): LLR negated (int8 wrap)
 *   oracle_csi_correction_b  csi_correction's llr_is_8bit branch (pdsch.c:538-545): (int8)((float)e * csi[i] /
 *                            csi_max), the division turned into a multiply by 1 / csi_max as -Ofast builds it
 * Pinned against _ref (demod / sequence compiled from the reference; csi_correction restated in
 * ref_pdsch_tx_harness.c and built with the reference's flags), tests/test_phy_oracle.py. */
static int8_t sat8(int32_t v) { return v > 127 ? 127 : (v < -128 ? -128 : (int8_t)v); }
static int8_t wrap8(int32_t v) { return (int8_t)(uint8_t)(uint32_t)v; }
static int8_t abs8(int8_t v) { return wrap8(v < 0 ? -(int32_t)v : (int32_t)v); } /* _mm_abs_epi8 */

int oracle_demod_soft_b(int mod, const float* sym, int8_t* llr, int n)
{
  switch (mod) {
    case 0: /* BPSK */
      for (int i = 0; i < n; i++) {
        const float t = -20.0f * (sym[2 * i] + sym[2 * i + 1]);
        llr[i]        = wrap8(cvt_tz_d((double)t * 0.70710678118654752440));
      }
      return 0;
    case 1: { /* QPSK: scale = (float)(-20 * M_SQRT2) */
      const float scale = (float)(-20.0 * 1.41421356237309504880);
      const int   len   = 2 * n;
      int         i     = 0;
      for (; i + 16 <= len; i += 16) {
        for (int k = 0; k < 16; k++) {
          llr[i + k] = sat8(cvt_tz(sym[i + k] * scale));
        }
      }
      for (; i < len; i++) {
        llr[i] = wrap8(cvt_tz(sym[i] * scale));
      }
      return 0;
    }
    case 2: { /* 16QAM */
      const int8_t off  = (int8_t)(2 * 30 / sqrtf(10));
      const float  offf = 2 * 30 / sqrtf(10);
      const int    nsse = 8 * (n / 8);
      for (int i = 0; i < n; i++) {
        for (int c = 0; c < 2; c++) {
          const float x = sym[2 * i + c];
          if (i < nsse) {
            const int8_t s  = sat8(cvt_rn(x * -30.0f));
            llr[4 * i + c]     = s;
            llr[4 * i + 2 + c] = wrap8(abs8(s) - off);
          } else {
            const int8_t y  = wrap8(cvt_tz(30.0f * x));
            llr[4 * i + c]     = wrap8(-(int32_t)y);
            llr[4 * i + 2 + c] = wrap8(cvt_tz((float)abs(y) - offf));
          }
        }
      }
      return 0;
    }
    case 3: { /* 64QAM */
      const int8_t off1 = (int8_t)(4 * 40 / sqrtf(42));
      const int8_t off2 = (int8_t)(2 * 40 / sqrtf(42));
      const int    nsse = 8 * (n / 8);
      for (int i = 0; i < n; i++) {
        for (int c = 0; c < 2; c++) {
          const float x = sym[2 * i + c];
          if (i < nsse) {
            const int8_t s = sat8(cvt_rn(x * -40.0f));
            const int8_t a = wrap8(abs8(s) - off1);
            llr[6 * i + c]     = s;
            llr[6 * i + 2 + c] = a;
            llr[6 * i + 4 + c] = wrap8(abs8(a) - off2);
          } else {
            const int8_t y = wrap8(cvt_tz(40.0f * x));
            const int8_t a = wrap8((int32_t)wrap8(abs(y)) - off1);
            llr[6 * i + c]     = wrap8(-(int32_t)y);
            llr[6 * i + 2 + c] = a;
            llr[6 * i + 4 + c] = wrap8((int32_t)wrap8(abs(a)) - off2);
          }
        }
      }
      return 0;
    }
    case 4: { /* 256QAM */
      const float t[3] = {8.0f / sqrtf(170.0f), 4.0f / sqrtf(170.0f), 2.0f / sqrtf(170.0f)};
      for (int i = 0; i < n; i++) {
        float v[2] = {-sym[2 * i], -sym[2 * i + 1]};
        for (int l = 0; l < 4; l++) {
          for (int c = 0; c < 2; c++) {
            if (l) {
              v[c] = fabsf(v[c]) - t[l - 1];
            }
            llr[8 * i + 2 * l + c] = wrap8(cvt_tz(50 * v[c]));
          }
        }
      }
      return 0;
    }
    default:
      return -1;
  }
}

void oracle_sequence_apply_c(const int8_t* in, int8_t* out, uint32_t len, uint32_t seed)
{
  uint32_t x1 = 1, x2 = seed & 0x7FFFFFFFu;
  for (int n = 0; n < 1600; n++) {
    x1 = step_x1(x1);
    x2 = step_x2(x2);
  }
  for (uint32_t i = 0; i < len; i++) {
    out[i] = ((x1 ^ x2) & 1u) ? wrap8(-(int32_t)in[i]) : in[i];
    x1     = step_x1(x1);
    x2     = step_x2(x2);
  }
}

void oracle_csi_correction_b(int mod, const float* csi, int8_t* e, uint32_t nof_bits)
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
  const float rcp = 1.0f / mx;
  for (uint32_t k = 0; k < ns; k++) {
    const float c = csi[k] * rcp;
    for (uint32_t b = 0; b < qm; b++) {
      e[qm * k + b] = wrap8(cvt_tz((float)e[qm * k + b] * c));
    }
  }
}

/* ======================= DL channel estimation (chest_dl.c, refsignal_dl.c) =======================
 * srsUE default configuration (srsue/src/phy/phy_common.cc:83-107, main.cc defaults): estimator
 * AVERAGE, Gauss smoothing filter order 4 / stddev 1.0, noise algorithm REFS, normal subframe,
 * normal or extended CP, FDD.  Restated (chest_dl.c and refsignal_dl.c include the generated srsran.h):
 *   CRS             srsran_refsignal_cs_set_cell  refsignal_dl.c:65-119, fidx/nsymbol 249-266
 *   LS              estimate_port                 chest_dl.c:806-834
 *   noise (REFS)    estimate_noise_pilots         chest_dl.c:325-400
 *   time average    average_pilots                chest_dl.c:557-600
 *   smoothing       srsran_conv_same_cf           convolution.c:182-218 (edge extrapolation)
 *   Gauss filter    srsran_chest_set_smooth_filter_gauss chest_common.c:70-95
 *   interpolation   srsran_interp_linear_offset   interp.c:258-285, then copy to all symbols
 *   CFO             chest_estimate_cfo            chest_dl.c:621-641
 * grid: [rx][2 nsymb * 12 * nof_prb] cf32; ce: [port][rx][2 nsymb * 12 * nof_prb] (nsymb 7 / 6). */
#define NRE 12
static const float kPi = 3.14159265358979323846f;

static uint32_t crs_v(uint32_t port, uint32_t l)
{
  switch (port) {
    case 0:
      return (l % 2) ? 3 : 0;
    case 1:
      return (l % 2) ? 0 : 3;
    case 2:
      return l == 0 ? 0 : 3;
    default:
      return l == 0 ? 3 : 0;
  }
}
static uint32_t crs_fidx(uint32_t cell_id, uint32_t l, uint32_t port) { return (crs_v(port, l) + cell_id % 6) % 6; }
/* srsran_refsignal_cs_nsymbol (refsignal_dl.c:254-266); nsymb = SRSRAN_CP_NSYMB: 7 normal, 6 extended CP */
static uint32_t crs_nsymbol(uint32_t l, uint32_t port, uint32_t nsymb)
{
  return port < 2 ? ((l % 2) ? (l / 2 + 1) * nsymb - 3 : (l / 2) * nsymb) : 1 + l * nsymb;
}
static uint32_t crs_nof_symbols(uint32_t port) { return port < 2 ? 4 : 2; }

/* pilots of port pair pp (ports 2pp, 2pp+1) for subframe sf: [nsym][2 * nof_prb]; cp 0 normal, 1 extended
 * (N_cp = 1 / 0 in c_init, refsignal_dl.c:81-97) */
void oracle_crs_pilots_cp(uint32_t cell_id, uint32_t nof_prb, uint32_t pp, uint32_t sf, uint32_t cp, float* out)
{
  const uint32_t nsymb = cp ? 6 : 7, N_cp = cp ? 0 : 1;
  cpx*           P        = (cpx*)out;
  const uint32_t nsym_slot = crs_nof_symbols(2 * pp) / 2;
  uint8_t        c[4 * 110];
  for (uint32_t s = 0; s < 2; s++) {
    const uint32_t ns = 2 * sf + s;
    for (uint32_t l = 0; l < nsym_slot; l++) {
      const uint32_t lp     = crs_nsymbol(l, 2 * pp, nsymb);
      const uint32_t c_init = 1024 * (7 * (ns + 1) + lp + 1) * (2 * cell_id + 1) + 2 * cell_id + N_cp;
      oracle_sequence_bits(c_init, c, 4 * 110);
      for (uint32_t i = 0; i < 2 * nof_prb; i++) {
        const uint32_t mp = i + 110 - nof_prb;
        P[2 * nof_prb * (s * nsym_slot + l) + i] =
            (cpx){(1 - 2 * (float)c[2 * mp]) * (float)0.70710678118654752440,
                  (1 - 2 * (float)c[2 * mp + 1]) * (float)0.70710678118654752440};
      }
    }
  }
}

void oracle_crs_pilots(uint32_t cell_id, uint32_t nof_prb, uint32_t pp, uint32_t sf, float* out)
{
  oracle_crs_pilots_cp(cell_id, nof_prb, pp, sf, 0, out);
}

static float avg_power(const cpx* x, uint32_t n)
{
  float acc = 0;
  for (uint32_t k = 0; k < n; k++) {
    acc += x[k].r * x[k].r + x[k].i * x[k].i;
  }
  return n ? acc / (float)n : 0.f;
}

static float noise_pilots(const cpx* pe, uint32_t nsym, uint32_t nref, uint32_t fidx0)
{
  cpx tmp[20 * 110]; /* nref <= 20 N_RB / 3 (MBSFN subframes) */
  if (nsym < 3) { /* chest_dl.c:345-354 */
    for (uint32_t k = 0; k < nref - 2; k++) {
      cpx t  = cadd(cadd(pe[k], pe[k + 1]), pe[k + 2]);
      t      = cscale(t, 1.0f / 3.0f);
      tmp[k] = csub(pe[k + 1], t);
    }
    return avg_power(tmp, nref - 2);
  }
  float    sum   = 0;
  uint32_t count = 0;
  for (uint32_t i = 1; i < nsym - 1; i++) {
    const uint32_t off = ((fidx0 < 3) ^ (i & 1)) ? 0 : 1;
    const cpx*     cur = pe + i * nref;
    for (uint32_t k = 0; k < nref; k++) {
      tmp[k] = cur[k];
    }
    for (int nb = 0; nb < 2; nb++) {
      const cpx* o = pe + (nb == 0 ? i - 1 : i + 1) * nref;
      for (uint32_t k = 0; k < nref - off; k++) {
        tmp[off + k] = cadd(o[k], tmp[off + k]);
      }
      for (uint32_t k = 0; k < nref + off - 1; k++) {
        tmp[k] = cadd(o[1 - off + k], tmp[k]);
      }
      if (off) {
        tmp[0] = cadd(tmp[0], csub(cscale(o[0], 2.0f), o[1]));
      } else {
        tmp[nref - 1] = cadd(tmp[nref - 1], csub(cscale(o[nref - 2], 2.0f), o[nref - 1]));
      }
    }
    for (uint32_t k = 0; k < nref; k++) {
      tmp[k] = csub(cur[k], cscale(tmp[k], 1.0f / 5.0f));
    }
    sum += avg_power(tmp, nref);
    count++;
  }
  return sum / (float)count;
}

static void conv_same(const cpx* in, const float* f, cpx* out, uint32_t N, uint32_t M)
{
  cpx first[16], last[16];
  for (uint32_t i = 0; i < M + M / 2; i++) {
    first[i] = i < M / 2 ? csub(cscale(in[1], (float)(2 + M / 2 - i)), cscale(in[0], (float)(1 + M / 2 - i)))
                         : in[i - M / 2];
    last[i] = i >= M - 1 ? csub(cscale(in[N - 1], (float)(2 + i - M / 2)), cscale(in[N - 2], (float)(1 + i - M / 2)))
                         : in[N - M + i + 1];
  }
  uint32_t i = 0;
  for (; i < M / 2; i++) {
    cpx acc = {0, 0};
    for (uint32_t k = 0; k < M; k++) {
      acc = cadd(acc, cscale(first[i + k], f[k]));
    }
    out[i] = acc;
  }
  for (; i < N - M / 2; i++) {
    cpx acc = {0, 0};
    for (uint32_t k = 0; k < M; k++) {
      acc = cadd(acc, cscale(in[i - M / 2 + k], f[k]));
    }
    out[i] = acc;
  }
  for (uint32_t j = 0; i < N; i++, j++) {
    cpx acc = {0, 0};
    for (uint32_t k = 0; k < M; k++) {
      acc = cadd(acc, cscale(last[j + k], f[k]));
    }
    out[i] = acc;
  }
}

void oracle_conv_same(const float* in, const float* f, float* out, uint32_t N, uint32_t M)
{
  conv_same((const cpx*)in, f, (cpx*)out, N, M);
}

uint32_t oracle_gauss_filter(float* f, uint32_t order, float std_dev)
{
  const uint32_t len = order + 1;
  const int      c   = (int)(len - 1) / 2;
  float          s   = 0;
  for (uint32_t i = 0; i < len; i++) {
    f[i] = expf(-powf((float)((int)i - c), 2) / (2.0f * powf(std_dev, 2)));
  }
  for (uint32_t i = 0; i < len; i++) {
    s += f[i];
  }
  for (uint32_t i = 0; i < len; i++) {
    f[i] *= 1.0f / s;
  }
  return len;
}

static void interp_linear_offset(const cpx* in, cpx* out, uint32_t len, uint32_t M, uint32_t off_st, uint32_t off_end)
{
  for (uint32_t j = 0; j < off_st; j++) {
    const cpx d = csub(in[1], in[0]);
    const cpx t = cscale(d, (float)(j + 1));
    out[off_st - j - 1] = csub(in[0], (cpx){t.r / (float)M, t.i / (float)M});
  }
  const float rM = (float)1 / M;
  uint32_t    i  = 0;
  for (; i < len - 1; i++) {
    const cpx d = cscale(csub(in[i + 1], in[i]), rM);
    for (uint32_t j = 0; j < M; j++) {
      out[i * M + j + off_st] = cadd(in[i], cscale(d, (float)j));
    }
  }
  if (len > 1) {
    const cpx d = csub(in[len - 1], in[len - 2]);
    for (uint32_t j = 0; j < off_end; j++) {
      const cpx t = cscale(d, (float)j);
      out[i * M + j + off_st] = cadd(in[i], (cpx){t.r / (float)M, t.i / (float)M});
    }
  }
}

/* out[0..5]: noise_estimate, rsrp, rssi, cfo, per (rx,port) noise not returned.
 * nsym_pp[0] / [1]: CRS symbols of ports 0 / 1 and 2 / 3 in this subframe (srsran_refsignal_cs_nof_symbols,
 * refsignal_dl.c:169-226): 4 / 2, fewer in the DwPTS of a TDD special subframe. */
static int chest_dl_impl(const float* grid, uint32_t nof_prb, uint32_t cell_id, uint32_t nports, uint32_t nrx,
                         uint32_t sf_idx, uint32_t symbol_sz, uint32_t cp, const uint32_t nsym_pp[2], float* ce,
                         float* out)
{
  const uint32_t nsymb = cp ? 6 : 7; /* SRSRAN_CP_NSYMB */
  const uint32_t nre = NRE * nof_prb, nsf = 2 * nsymb * nre;
  const cpx*     G   = (const cpx*)grid;
  cpx*           CE  = (cpx*)ce;
  float          filt[8];
  const uint32_t flen = oracle_gauss_filter(filt, 4, 1.0f);
  static cpx     pil[2][4 * 2 * 110];
  oracle_crs_pilots_cp(cell_id, nof_prb, 0, sf_idx, cp, (float*)pil[0]);
  oracle_crs_pilots_cp(cell_id, nof_prb, 1, sf_idx, cp, (float*)pil[1]);
  float noise[4][4], rsrp[4][4], rssi[4][4], cfo = 0;
  for (uint32_t rx = 0; rx < nrx; rx++) {
    const cpx* in = G + (size_t)rx * nsf;
    for (uint32_t port = 0; port < nports; port++) {
      const uint32_t nsym = nsym_pp[port < 2 ? 0 : 1], nref = 2 * nof_prb, np = nsym * nref;
      cpx            recv[4 * 220], pe[4 * 220], avg[4 * 220], tmp[4 * 220];
      for (uint32_t l = 0; l < nsym; l++) {
        const uint32_t sym = crs_nsymbol(l, port, nsymb);
        uint32_t       f   = crs_fidx(cell_id, l, port);
        for (uint32_t i = 0; i < nref; i++, f += 6) {
          recv[l * nref + i] = in[sym * nre + f];
        }
      }
      for (uint32_t k = 0; k < np; k++) {
        pe[k] = cmul(recv[k], cconj(pil[port / 2][k]));
      }
      rsrp[rx][port] = avg_power(recv, np);
      float rs       = 0;
      for (uint32_t l = 0; l < nsym; l++) {
        const cpx* t = in + crs_nsymbol(l, port, nsymb) * nre;
        for (uint32_t k = 0; k < nre; k++) {
          rs += t[k].r * t[k].r + t[k].i * t[k].i;
        }
      }
      rssi[rx][port] = rs / (float)nsym;
      if (nsym == 4) { /* chest_estimate_cfo (port-0 geometry), kept from the last port processed */
        cpx sum = {0, 0};
        for (uint32_t i = 0; i < 2; i++) {
          for (uint32_t k = 0; k < np / 4; k++) {
            sum = cadd(sum, cmul(pe[i * np / 4 + k], cconj(pe[(i + 2) * np / 4 + k])));
          }
        }
        const float n  = (float)symbol_sz;
        const float ng = (float)(int)ceilf(144.0f * n / 2048.0f); /* SRSRAN_CP_LEN_NORM(1, n) */
        cfo            = -atan2f(sum.i, sum.r) * n / ((float)nsymb * (n + ng)) / 2 / kPi;
      }
      const uint32_t fidx0 = crs_fidx(cell_id, 0, port);
      noise[rx][port]      = noise_pilots(pe, nsym, nref, fidx0);
      /* average_pilots: time average into a 3-subcarrier grid, then smoothing */
      uint32_t nr = nref, ns = nsym;
      if (nsym > 1) {
        const cpx* a = fidx0 < 3 ? pe : pe + nref;
        const cpx* b = fidx0 < 3 ? pe + nref : pe;
        for (uint32_t k = 0; k < nref; k++) {
          tmp[2 * k]     = a[k];
          tmp[2 * k + 1] = b[k];
        }
        for (uint32_t l = 2; l < nsym - 1; l += 2) {
          const cpx* c = fidx0 < 3 ? pe + l * nref : pe + (l + 1) * nref;
          const cpx* d = fidx0 < 3 ? pe + (l + 1) * nref : pe + l * nref;
          for (uint32_t k = 0; k < nref; k++) {
            tmp[2 * k]     = cadd(tmp[2 * k], c[k]);
            tmp[2 * k + 1] = cadd(tmp[2 * k + 1], d[k]);
          }
        }
        nr *= 2;
        for (uint32_t k = 0; k < nr; k++) {
          pe[k] = cscale(tmp[k], 2.0f / (float)nsym);
        }
        ns = 1;
      }
      (void)ns;
      conv_same(pe, filt, avg, nr, flen);
      cpx* row = CE + ((size_t)port * nrx + rx) * nsf;
      if (nsym > 1) {
        const uint32_t off = cell_id % 3;
        interp_linear_offset(avg, row, nr, 3, off, 3 - off);
      } else {
        const uint32_t off = crs_fidx(cell_id, 0, port);
        interp_linear_offset(avg, row, nr, 6, off, 6 - off);
      }
      for (uint32_t l = 1; l < 2 * nsymb; l++) {
        memcpy(row + l * nre, row, nre * sizeof(cpx));
      }
    }
  }
  float n = 0;
  for (uint32_t rx = 0; rx < nrx; rx++) {
    float s = 0;
    for (uint32_t p = 0; p < nports; p++) {
      s += noise[rx][p];
    }
    n += s / (float)nports;
  }
  out[0] = n / (float)nrx;
  float best = -1e9f;
  for (uint32_t p = 0; p < nports; p++) {
    float s = 0;
    for (uint32_t rx = 0; rx < nrx; rx++) {
      s += rsrp[rx][p];
    }
    s /= (float)nrx;
    best = s > best ? s : best;
  }
  out[1] = best;
  float r = 0;
  for (uint32_t rx = 0; rx < nrx; rx++) {
    r += 4 * rssi[rx][0] / (float)nof_prb / (float)NRE;
  }
  out[2] = r / (float)nrx;
  out[3] = cfo;
  return 0;
}

int oracle_chest_dl_cp(const float* grid, uint32_t nof_prb, uint32_t cell_id, uint32_t nports, uint32_t nrx,
                       uint32_t sf_idx, uint32_t symbol_sz, uint32_t cp, float* ce, float* out)
{
  const uint32_t nsym_pp[2] = {4, 2};
  return chest_dl_impl(grid, nof_prb, cell_id, nports, nrx, sf_idx, symbol_sz, cp, nsym_pp, ce, out);
}

/* a TDD special subframe: nsym01 / nsym23 CRS symbols of ports 0-1 / 2-3 in its DwPTS (the chest_dl.c paths for
 * 1-3 symbols: noise 345-354 / 363, time average 571-589, frequency interpolation 488-499) */
int oracle_chest_dl_tdd(const float* grid, uint32_t nof_prb, uint32_t cell_id, uint32_t nports, uint32_t nrx,
                        uint32_t sf_idx, uint32_t symbol_sz, uint32_t cp, uint32_t nsym01, uint32_t nsym23, float* ce,
                        float* out)
{
  const uint32_t nsym_pp[2] = {nsym01, nsym23};
  return chest_dl_impl(grid, nof_prb, cell_id, nports, nrx, sf_idx, symbol_sz, cp, nsym_pp, ce, out);
}

int oracle_chest_dl(const float* grid, uint32_t nof_prb, uint32_t cell_id, uint32_t nports, uint32_t nrx,
                    uint32_t sf_idx, uint32_t symbol_sz, float* ce, float* out)
{
  return oracle_chest_dl_cp(grid, nof_prb, cell_id, nports, nrx, sf_idx, symbol_sz, 0, ce, out);
}

/* ======================= chest_dl.c beyond srsUE's defaults (round 4) =======================
 *   estimator INTERPOLATE  average_pilots without the time average (chest_dl.c:571-599), frequency
 *                          interpolation per CRS symbol (interpolate_pilots 476-505: interp_lin, M = 6) and
 *                          the time interpolation between the CRS symbols (510-554, interp.c:147-188)
 *   noise PSS / EMPTY      estimate_noise_pss (402-419) / estimate_noise_empty_sc (422-433) in subframes 0 and
 *                          5, after the interpolation (731-745); other subframes keep q->noise_estimate
 *   automatic filter       Gauss order 4, stddev 200 x q->noise_estimate[rx][port] (706-707): the REFS value
 *                          of this subframe, the kept value with PSS / EMPTY
 *   correct_sync_error     chest_dl_estimate_correct_sync_error (750-804) on the rx grid before estimation
 * estimator: 0 AVERAGE, 1 INTERPOLATE; noise_alg: 0 REFS, 1 PSS, 2 EMPTY; filt_order 0 = automatic;
 * noise_state [4 rx][4 port] in / out (q->noise_estimate); pss: the 62 PSS values of N_id_2 (may be NULL unless
 * noise_alg = PSS); grid is modified in place by the sync correction; out: noise, rsrp, rssi, cfo, sync_error. */

/* srsran_vec_apply_cfo (vector_simd.c:1723-1774, AVX2 + FMA build): 8 phase lanes advanced by w^8, scalar tail */
static cpx cprod_fma(cpx a, cpx b)
{
  const float t1 = a.i * b.i, t2 = a.i * b.r;
  return (cpx){fmaf(a.r, b.r, -t1), fmaf(a.r, b.i, t2)};
}
void oracle_apply_cfo(const float* x, float cfo, float* z, uint32_t len)
{
  const float twopi = 2.0f * (float)M_PI;
  float       s, c;
  sincosf(twopi * cfo, &s, &c);
  const cpx w = {c, s};
  cpx       ph[8];
  ph[0] = (cpx){1.0f, 0.0f};
  for (int k = 1; k < 8; k++) {
    ph[k] = cprod_fma(ph[k - 1], w);
  }
  const cpx  w8 = cprod_fma(ph[7], w);
  const cpx* X  = (const cpx*)x;
  cpx*       Z  = (cpx*)z;
  uint32_t   i  = 0;
  for (; i + 8 <= len; i += 8) {
    for (int k = 0; k < 8; k++) {
      Z[i + k] = cprod_fma(X[i + k], ph[k]);
      ph[k]    = cprod_fma(ph[k], w8);
    }
  }
  cpx p = ph[0];
  for (; i < len; i++) {
    Z[i] = cprod_fma(X[i], p);
    p    = cprod_fma(p, w);
  }
}

/* srsran_interp_linear_vector3 (interp.c:158-188) with to_right, len = vector length */
static void interp_vector(const cpx* in0, const cpx* in1, const cpx* start, cpx* between, uint32_t d, uint32_t M,
                          uint32_t nre)
{
  const float rd = (float)1 / d;
  for (uint32_t k = 0; k < nre; k++) {
    const cpx diff = cscale(csub(in1[k], in0[k]), rd);
    cpx       b    = cadd(start ? start[k] : in0[k], diff);
    between[k]     = b;
    for (uint32_t i = 1; i < M; i++) {
      b                    = cadd(b, diff);
      between[i * nre + k] = b;
    }
  }
}

/* srsran_vec_estimate_frequency (vector_simd.c:1776-1818) in scalar order */
float oracle_estimate_frequency(const float* xf, uint32_t len);
static float estimate_frequency(const cpx* x, uint32_t len) { return oracle_estimate_frequency((const float*)x, len); }
float oracle_estimate_frequency(const float* xf, uint32_t len)
{
  const cpx* x   = (const cpx*)xf;
  cpx        sum = {0, 0};
  for (uint32_t i = 1; i < len; i++) {
    sum = cadd(sum, cmul(x[i], cconj(x[i - 1])));
  }
  return (float)(-atan2f(sum.i, sum.r) * M_1_PI * 0.5f);  /* -cargf(sum) * M_1_PI * 0.5f */
}

/* nsym01 / nsym23: CRS symbols of ports 0-1 / 2-3 (4 / 2 in normal subframes, fewer in a TDD special subframe's
 * DwPTS; INTERPOLATE there: 1 symbol -> its row everywhere, 3 (normal CP) -> rows 0, 4, 7 with 8..13 extrapolated,
 * chest_dl.c:511-531) */
int oracle_chest_dl_ext_tdd(float* grid, uint32_t nof_prb, uint32_t cell_id, uint32_t nports, uint32_t nrx,
                            uint32_t sf_idx, uint32_t symbol_sz, uint32_t cp, uint32_t estimator, uint32_t noise_alg,
                            uint32_t filt_order, float filt_std, uint32_t sync, const float* pss, float* noise_state,
                            uint32_t nsym01, uint32_t nsym23, float* ce, float* out);
int oracle_chest_dl_ext(float* grid, uint32_t nof_prb, uint32_t cell_id, uint32_t nports, uint32_t nrx, uint32_t sf_idx,
                        uint32_t symbol_sz, uint32_t cp, uint32_t estimator, uint32_t noise_alg, uint32_t filt_order,
                        float filt_std, uint32_t sync, const float* pss, float* noise_state, float* ce, float* out)
{
  return oracle_chest_dl_ext_tdd(grid, nof_prb, cell_id, nports, nrx, sf_idx, symbol_sz, cp, estimator, noise_alg,
                                 filt_order, filt_std, sync, pss, noise_state, 4, 2, ce, out);
}

/* filter_type: 0 GAUSS (coef0 = order, coef1 = stddev; coef0 <= 0 automatic: order 4, stddev 200 x noise), 1 TRIANGLE
 * (coef0 = w: {w, 1 - 2w, w}, chest_common.c:62-68), 2 NONE (no average_pilots: the LS estimates interpolated as
 * they are, chest_dl.c:724-725 -- with AVERAGE and more than one CRS symbol the first 4 N_RB of them as one comb of
 * spacing 3, 476-481) */
int oracle_chest_dl_ext_f(float* grid, uint32_t nof_prb, uint32_t cell_id, uint32_t nports, uint32_t nrx,
                          uint32_t sf_idx, uint32_t symbol_sz, uint32_t cp, uint32_t estimator, uint32_t noise_alg,
                          uint32_t filter_type, float coef0, float coef1, uint32_t sync, const float* pss,
                          float* noise_state, uint32_t nsym01, uint32_t nsym23, float* ce, float* out);
int oracle_chest_dl_ext_tdd(float* grid, uint32_t nof_prb, uint32_t cell_id, uint32_t nports, uint32_t nrx,
                            uint32_t sf_idx, uint32_t symbol_sz, uint32_t cp, uint32_t estimator, uint32_t noise_alg,
                            uint32_t filt_order, float filt_std, uint32_t sync, const float* pss, float* noise_state,
                            uint32_t nsym01, uint32_t nsym23, float* ce, float* out)
{
  return oracle_chest_dl_ext_f(grid, nof_prb, cell_id, nports, nrx, sf_idx, symbol_sz, cp, estimator, noise_alg, 0,
                               (float)filt_order, filt_std, sync, pss, noise_state, nsym01, nsym23, ce, out);
}

/* the smoothing filter of chest_interpolate_noise_est (chest_dl.c:700-717); returns its length (0: none, or a
 * Gauss filter whose sum is not normal -- srsran_conv_same_cf then writes zeros) */
static uint32_t oracle_filter(uint32_t filter_type, float coef0, float coef1, float noise, float* filt)
{
  if (filter_type == 1) {
    filt[0] = filt[2] = coef0;
    filt[1]           = 1 - 2 * coef0;
    return 3;
  }
  if (filter_type == 2) {
    return 0;
  }
  uint32_t flen = coef0 > 0 ? oracle_gauss_filter(filt, (uint32_t)coef0, coef1) : oracle_gauss_filter(filt, 4, noise * 200.0f);
  float    s    = 0;
  for (uint32_t k = 0; k < flen; k++) {
    s += filt[k];
  }
  return isnormal(s) ? flen : 0;
}

int oracle_chest_dl_ext_f(float* grid, uint32_t nof_prb, uint32_t cell_id, uint32_t nports, uint32_t nrx,
                          uint32_t sf_idx, uint32_t symbol_sz, uint32_t cp, uint32_t estimator, uint32_t noise_alg,
                          uint32_t filter_type, float coef0, float coef1, uint32_t sync, const float* pss,
                          float* noise_state, uint32_t nsym01, uint32_t nsym23, float* ce, float* out)
{
  const uint32_t nsymb = cp ? 6 : 7;
  const int      none  = filter_type == 2;
  const uint32_t nre = NRE * nof_prb, nsf = 2 * nsymb * nre, nref = 2 * nof_prb;
  cpx*           G   = (cpx*)grid;
  cpx*           CE  = (cpx*)ce;
  static cpx     pil[2][4 * 2 * 110];
  oracle_crs_pilots_cp(cell_id, nof_prb, 0, sf_idx, cp, (float*)pil[0]);
  oracle_crs_pilots_cp(cell_id, nof_prb, 1, sf_idx, cp, (float*)pil[1]);
  float rsrp[4][4], rssi[4][4], cfo = 0, sync_err00 = 0;
  for (uint32_t rx = 0; rx < nrx; rx++) {
    cpx* in = G + (size_t)rx * nsf;
    if (sync) { /* chest_dl.c:750-804 */
      float pwr_sum = 0, serr = 0;
      for (uint32_t port = 0; port < nports; port++) {
        const uint32_t nsym = port < 2 ? nsym01 : nsym23, np = nsym * nref;
        cpx            pe[4 * 220];
        for (uint32_t l = 0; l < nsym; l++) {
          const uint32_t sym = crs_nsymbol(l, port, nsymb);
          uint32_t       f   = crs_fidx(cell_id, l, port);
          for (uint32_t i = 0; i < nref; i++, f += 6) {
            pe[l * nref + i] = cmul(in[sym * nre + f], cconj(pil[port / 2][l * nref + i]));
          }
        }
        const float k   = (float)symbol_sz / 6.0f;
        float       sum = 0;
        for (uint32_t l = 0; l < nsym; l++) {
          sum += estimate_frequency(pe + l * nref, nref) * k;
        }
        const float pwr = avg_power(pe, np);
        const float se  = sum / (float)nsym;
        if (rx == 0 && port == 0) {
          sync_err00 = se;
        }
        if (!isinf(sum) && !isnan(sum) && !isinf(pwr) && !isnan(pwr)) {
          serr += se * pwr;
          pwr_sum += pwr;
        }
      }
      if (isnormal(pwr_sum)) {
        serr /= pwr_sum;
      }
      if (isnormal(serr) && fabsf(serr) > 0.05f) {
        const float f = serr / (float)symbol_sz;
        for (uint32_t i = 0; i < 2 * nsymb; i++) {
          oracle_apply_cfo((const float*)(in + i * nre), f, (float*)(in + i * nre), nre);
        }
      }
    }
    for (uint32_t port = 0; port < nports; port++) {
      const uint32_t nsym = port < 2 ? nsym01 : nsym23, np = nsym * nref;
      cpx            recv[4 * 220], pe[4 * 220], avg[4 * 220], tmp[4 * 220];
      for (uint32_t l = 0; l < nsym; l++) {
        const uint32_t sym = crs_nsymbol(l, port, nsymb);
        uint32_t       f   = crs_fidx(cell_id, l, port);
        for (uint32_t i = 0; i < nref; i++, f += 6) {
          recv[l * nref + i] = in[sym * nre + f];
        }
      }
      for (uint32_t k = 0; k < np; k++) {
        pe[k] = cmul(recv[k], cconj(pil[port / 2][k]));
      }
      rsrp[rx][port] = avg_power(recv, np);
      float rs       = 0;
      for (uint32_t l = 0; l < nsym; l++) {
        const cpx* t = in + crs_nsymbol(l, port, nsymb) * nre;
        for (uint32_t k = 0; k < nre; k++) {
          rs += t[k].r * t[k].r + t[k].i * t[k].i;
        }
      }
      rssi[rx][port] = rs / (float)nsym;
      if (nsym == 4) {
        cpx sum = {0, 0};
        for (uint32_t i = 0; i < 2; i++) {
          for (uint32_t k = 0; k < np / 4; k++) {
            sum = cadd(sum, cmul(pe[i * np / 4 + k], cconj(pe[(i + 2) * np / 4 + k])));
          }
        }
        const float n  = (float)symbol_sz;
        const float ng = (float)(int)ceilf(144.0f * n / 2048.0f);
        cfo            = -atan2f(sum.i, sum.r) * n / ((float)nsymb * (n + ng)) / 2 / kPi;
      }
      const uint32_t fidx0 = crs_fidx(cell_id, 0, port);
      float*         ns    = &noise_state[rx * 4 + port];
      if (noise_alg == 0) {
        *ns = noise_pilots(pe, nsym, nref, fidx0);
      }
      float          filt[8];
      const uint32_t flen = oracle_filter(filter_type, coef0, coef1, *ns, filt);
      cpx*           row  = CE + ((size_t)port * nrx + rx) * nsf;
      if (estimator == 0) {
        uint32_t nr = nref;
        if (none) {
          nr = nsym > 1 ? 2 * nref : nref;
        } else if (nsym > 1) {
          const cpx* a = fidx0 < 3 ? pe : pe + nref;
          const cpx* b = fidx0 < 3 ? pe + nref : pe;
          for (uint32_t k = 0; k < nref; k++) {
            tmp[2 * k]     = a[k];
            tmp[2 * k + 1] = b[k];
          }
          for (uint32_t l = 2; l < nsym - 1; l += 2) {
            const cpx* c = fidx0 < 3 ? pe + l * nref : pe + (l + 1) * nref;
            const cpx* d = fidx0 < 3 ? pe + (l + 1) * nref : pe + l * nref;
            for (uint32_t k = 0; k < nref; k++) {
              tmp[2 * k]     = cadd(tmp[2 * k], c[k]);
              tmp[2 * k + 1] = cadd(tmp[2 * k + 1], d[k]);
            }
          }
          nr *= 2;
          for (uint32_t k = 0; k < nr; k++) {
            pe[k] = cscale(tmp[k], 2.0f / (float)nsym);
          }
        }
        if (none) {
          memcpy(avg, pe, nr * sizeof(cpx));
        } else if (flen) {
          conv_same(pe, filt, avg, nr, flen);
        } else {
          memset(avg, 0, nr * sizeof(cpx));
        }
        if (nsym > 1) {
          const uint32_t off = cell_id % 3;
          interp_linear_offset(avg, row, nr, 3, off, 3 - off);
        } else {
          interp_linear_offset(avg, row, nr, 6, fidx0, 6 - fidx0);
        }
        for (uint32_t l = 1; l < 2 * nsymb; l++) {
          memcpy(row + l * nre, row, nre * sizeof(cpx));
        }
      } else if (nsym == 1) { /* one CRS symbol: interpolated into row 0, copied everywhere (chest_dl.c:488-515) */
        if (none) {
          memcpy(avg, pe, nref * sizeof(cpx));
        } else if (flen) {
          conv_same(pe, filt, avg, nref, flen);
        } else {
          memset(avg, 0, nref * sizeof(cpx));
        }
        interp_linear_offset(avg, row, nref, 6, fidx0, 6 - fidx0);
        for (uint32_t l = 1; l < 2 * nsymb; l++) {
          memcpy(row + l * nre, row, nre * sizeof(cpx));
        }
      } else {
        for (uint32_t l = 0; l < nsym; l++) { /* smoothing of every CRS symbol, then interpolation into its row */
          if (none) {
            memcpy(avg + l * nref, pe + l * nref, nref * sizeof(cpx));
          } else if (flen) {
            conv_same(pe + l * nref, filt, avg + l * nref, nref, flen);
          } else {
            memset(avg + l * nref, 0, nref * sizeof(cpx));
          }
          const uint32_t off = crs_fidx(cell_id, l, port);
          interp_linear_offset(avg + l * nref, row + crs_nsymbol(l, port, nsymb) * nre, nref, 6, off, 6 - off);
        }
#define CES(i) (row + (size_t)(i)*nre)
        if (!cp && port < 2 && nsym == 3) { /* chest_dl.c:520-527: the nsymbols != 4 branch */
          interp_vector(CES(0), CES(4), NULL, CES(1), 4, 3, nre);
          interp_vector(CES(4), CES(7), NULL, CES(5), 3, 2, nre);
          interp_vector(CES(4), CES(7), CES(7), CES(8), 3, 6, nre);
        } else if (!cp) {
          if (port < 2) {
            interp_vector(CES(0), CES(4), NULL, CES(1), 4, 3, nre);
            interp_vector(CES(4), CES(7), NULL, CES(5), 3, 2, nre);
            interp_vector(CES(7), CES(11), NULL, CES(8), 4, 3, nre);
            interp_vector(CES(7), CES(11), CES(11), CES(12), 4, 2, nre);
          } else {
            interp_vector(CES(8), CES(1), CES(1), CES(0), 7, 1, nre);
            interp_vector(CES(1), CES(8), NULL, CES(2), 7, 6, nre);
            interp_vector(CES(1), CES(8), NULL, CES(9), 7, 5, nre);
          }
        } else {
          if (port < 2) {
            interp_vector(CES(0), CES(3), NULL, CES(1), 3, 2, nre);
            interp_vector(CES(3), CES(6), NULL, CES(4), 3, 2, nre);
            interp_vector(CES(6), CES(9), NULL, CES(7), 3, 2, nre);
            interp_vector(CES(6), CES(9), CES(9), CES(10), 3, 2, nre);
          } else {
            interp_vector(CES(7), CES(1), CES(1), CES(0), 6, 1, nre);
            interp_vector(CES(1), CES(7), NULL, CES(2), 6, 5, nre);
            interp_vector(CES(1), CES(7), NULL, CES(8), 6, 4, nre);
          }
        }
#undef CES
      }
      if (noise_alg != 0 && (sf_idx == 0 || sf_idx == 5)) {
        const uint32_t kp = (nsymb - 1) * nre + nre / 2 - 31;
        if (noise_alg == 1) { /* estimate_noise_pss: nof_ports * avg|ce * pss - rx|^2 * M_SQRT1_2 */
          cpx t[62];
          for (uint32_t k = 0; k < 62; k++) {
            const cpx p = {pss[2 * k], pss[2 * k + 1]};
            t[k]        = csub(cmul(row[kp + k], p), in[kp + k]);
          }
          *ns = (float)nports * avg_power(t, 62) * (float)M_SQRT1_2;
        } else { /* estimate_noise_empty_sc */
          const uint32_t ks = (nsymb - 2) * nre + nre / 2 - 31;
          *ns = avg_power(in + ks - 5, 5) + avg_power(in + ks + 62, 5) + avg_power(in + kp - 5, 5) +
                avg_power(in + kp + 62, 5);
        }
      }
    }
  }
  float n = 0;
  for (uint32_t rx = 0; rx < nrx; rx++) {
    float s = 0;
    for (uint32_t p = 0; p < nports; p++) {
      s += noise_state[rx * 4 + p];
    }
    n += s / (float)nports;
  }
  out[0] = n / (float)nrx;
  float best = -1e9f;
  for (uint32_t p = 0; p < nports; p++) {
    float s = 0;
    for (uint32_t rx = 0; rx < nrx; rx++) {
      s += rsrp[rx][p];
    }
    s /= (float)nrx;
    best = s > best ? s : best;
  }
  out[1] = best;
  float r = 0;
  for (uint32_t rx = 0; rx < nrx; rx++) {
    r += 4 * rssi[rx][0] / (float)nof_prb / (float)NRE;
  }
  out[2] = r / (float)nrx;
  out[3] = cfo;
  out[4] = sync ? sync_err00 : 0.0f;
  return 0;
}

/* ======================= MBSFN subframes (round 5) =======================
 * srsran_refsignal_mbsfn_gen_seq (refsignal_dl.c:382-422): the MBSFN reference signals of subframe sf, area
 * N_MBSFN: for l = 0..2 (grid symbols 2 / 6 / 10 of the extended-CP layout, l' = symbol mod 6 in slot 2 sf for l = 0,
 * 2 sf + 1 otherwise), c_init = 512 (7 (ns + 1) + l' + 1)(2 N_MBSFN + 1) + N_MBSFN, r(m) from c(2m'), c(2m' + 1),
 * m' = m + 3 (110 - N_RB), m < 6 N_RB.  out: [3][6 N_RB] cf32 */
void oracle_mbsfn_pilots(uint32_t nof_prb, uint32_t area, uint32_t sf, float* out)
{
  cpx*    P = (cpx*)out;
  uint8_t c[20 * 110];
  for (uint32_t l = 0; l < 3; l++) {
    const uint32_t lp = (2 + 4 * l) % 6, ns = l ? 2 * sf + 1 : 2 * sf;
    oracle_sequence_bits(512 * (7 * (ns + 1) + lp + 1) * (2 * area + 1) + area, c, 20 * 110);
    for (uint32_t i = 0; i < 6 * nof_prb; i++) {
      const uint32_t mp = i + 3 * (110 - nof_prb);
      P[6 * nof_prb * l + i] = (cpx){(1 - 2 * (float)c[2 * mp]) * (float)0.70710678118654752440,
                                     (1 - 2 * (float)c[2 * mp + 1]) * (float)0.70710678118654752440};
    }
  }
}

/* srsran_chest_dl_estimate_cfg on an MBSFN subframe (estimate_port_mbsfn, chest_dl.c:836-865, with
 * chest_interpolate_noise_est 642-747, average_pilots 557-600, interpolate_pilots 437-555), INTERPOLATE, ports 0 / 1:
 *   LS over the CRS of symbol 0 (2 N_RB; the CRS of port pair 0 / subframe sf, its first symbol) and the MBSFN
 *   reference signals of grid symbols 2 / 6 / 10 at subcarriers 2i + (0, 1, 0) (srsran_refsignal_mbsfn_get_sf,
 *   refsignal_dl.c:474-502), 20 N_RB estimates; REFS noise over them as 3 rows of floor(20 N_RB / 3) with fidx 1
 *   (estimate_noise_pilots 331-342); PSS / EMPTY keep noise_state (subframes 0 / 5 are not MBSFN); the CRS row
 *   copied and each MBSFN row filtered (average_pilots 591-599); frequency interpolation into rows 0 (spacing 6),
 *   2 / 6 / 10 (spacing 2, offsets 0 / 1 / 0), time interpolation 517-521.  Rows 12 / 13 of ce are not written;
 *   rsrp / rssi / cfo are not measured (the caller keeps them).  out[0] = the noise estimate (fill_res). */
int oracle_chest_dl_mbsfn(const float* grid, uint32_t nof_prb, uint32_t cell_id, uint32_t nports, uint32_t nrx,
                          uint32_t sf_idx, uint32_t cp, uint32_t area, uint32_t noise_alg, uint32_t filter_type,
                          float coef0, float coef1, float* noise_state, float* ce, float* out)
{
  if (nports > 2) {
    return -1;
  }
  const uint32_t nsymb = cp ? 6 : 7, N = nof_prb;
  const uint32_t nre = NRE * N, nsf = 2 * nsymb * nre, nref = 2 * N, nm = 6 * N, np = 20 * N;
  const cpx*     G  = (const cpx*)grid;
  cpx*           CE = (cpx*)ce;
  static cpx     pil[4 * 2 * 110], mp[18 * 110], pe[20 * 110], avg[20 * 110], tmp[20 * 110];
  oracle_crs_pilots_cp(cell_id, N, 0, sf_idx, cp, (float*)pil);
  oracle_mbsfn_pilots(N, area, sf_idx, (float*)mp);
  for (uint32_t rx = 0; rx < nrx; rx++) {
    const cpx* in = G + (size_t)rx * nsf;
    for (uint32_t port = 0; port < nports; port++) {
      const uint32_t fidx0 = crs_fidx(cell_id, 0, port);
      for (uint32_t i = 0; i < nref; i++) {
        pe[i] = cmul(in[crs_nsymbol(0, port, nsymb) * nre + fidx0 + 6 * i], cconj(pil[i]));
      }
      for (uint32_t l = 0; l < 3; l++) {
        for (uint32_t i = 0; i < nm; i++) {
          pe[nref + l * nm + i] = cmul(in[(2 + 4 * l) * nre + (l == 1 ? 1 : 0) + 2 * i], cconj(mp[l * nm + i]));
        }
      }
      float* ns = &noise_state[rx * 4 + port];
      if (noise_alg == 0) {
        *ns = noise_pilots(pe, 3, np / 3, 1);
      }
      float          filt[8];
      const uint32_t flen = oracle_filter(filter_type, coef0, coef1, *ns, filt);
      memcpy(avg, pe, nref * sizeof(cpx));
      for (uint32_t l = 0; l < 3; l++) {
        if (filter_type == 2) {
          memcpy(avg + nref + l * nm, pe + nref + l * nm, nm * sizeof(cpx));
        } else if (flen) {
          conv_same(pe + nref + l * nm, filt, avg + nref + l * nm, nm, flen);
        } else {
          memset(avg + nref + l * nm, 0, nm * sizeof(cpx));
        }
      }
      (void)tmp;
      cpx* row = CE + ((size_t)port * nrx + rx) * nsf;
#define CES(i) (row + (size_t)(i)*nre)
      interp_linear_offset(avg, CES(0), nref, 6, fidx0, 6 - fidx0);
      for (uint32_t l = 0; l < 3; l++) {
        const uint32_t f = l == 1 ? 1 : 0;
        interp_linear_offset(avg + nref + l * nm, CES(2 + 4 * l), nm, 2, f, f ? 1 : 2);
      }
      interp_vector(CES(0), CES(2), NULL, CES(1), 2, 1, nre);
      interp_vector(CES(2), CES(6), NULL, CES(3), 4, 3, nre);
      interp_vector(CES(6), CES(10), NULL, CES(7), 4, 3, nre);
      interp_vector(CES(6), CES(10), CES(10), CES(11), 4, 1, nre);
#undef CES
    }
  }
  float n = 0;
  for (uint32_t rx = 0; rx < nrx; rx++) {
    float s = 0;
    for (uint32_t p = 0; p < nports; p++) {
      s += noise_state[rx * 4 + p];
    }
    n += s / (float)nports;
  }
  out[0] = n / (float)nrx;
  return 0;
}

/* srsran_pss_generate (pss.c:341-368): the argument in double, cosf / sinf of its float */
void oracle_pss_generate(uint32_t N_id_2, float* signal)
{
  const float root[3] = {25.0f, 29.0f, 34.0f};
  for (int i = 0; i < 62; i++) {
    const double v   = i < 31 ? ((float)i * ((float)i + 1.0)) : (((float)i + 2.0) * ((float)i + 1.0));
    const float  arg = (float)((float)-1 * M_PI * root[N_id_2] * v / 63.0);
    signal[2 * i]     = cosf(arg);
    signal[2 * i + 1] = sinf(arg);
  }
}
