/*
 * oracle/tdec_oracle.c -- CPU restatement of srsRAN_4G's LTE turbo decoder.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * decoder in srsran_4g_amd/csrc.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  The product library never links it.
 *
 * Parity status: PINNED.  tests/test_oracle.py checks this restatement against
 * the reference decoder compiled from /root/reference (oracle/_ref, see
 * oracle/Makefile) on random inputs for all 188 code-block sizes, and against the
 * committed golden vectors in tests/golden/ (made by tests/golden/make_golden.py
 * from oracle/_ref).
 *
 * What is restated (reference file:line, paths relative to /root/reference/lib):
 *  - AUTO 16-bit dispatch per code-block size K, AVX2 build
 *      src/phy/fec/turbo/turbodecoder.c:381-408, 486-507
 *      K <= 400 or K%8  -> generic full-length max-log-MAP, int16 wrap-around
 *      408..800, K%8==0 -> 8-sub-block sliding window, saturating int16
 *      K > 800, K%16==0 -> 16-sub-block sliding window, saturating int16
 *  - generic MAP: src/phy/fec/turbo/turbodecoder_gen.c:58-198, 226-236
 *  - window MAP:  include/srsran/phy/fec/turbo/turbodecoder_win.h:480-832
 *    (beta_trellis 500-548, beta 551-681, alpha 684-832, 40-step overlap,
 *     normalisation every 2 steps, lane shifts move_right/move_left incl. the
 *     AVX 128-bit-lane fix-ups at 579-612 and 716-746 which amount to a clean
 *     one-lane shift)
 *  - half-iteration driver: include/srsran/phy/fec/turbo/turbodecoder_iter.h:72-144
 *  - QPP interleaver: src/phy/fec/turbo/tc_interl_lte.c:39-107
 *  - hard decision MSB-first: turbodecoder_gen.c:260-277, turbodecoder_win.h:973-993
 *  - input layouts: natural 3K+12 (turbodecoder_gen.c:238-258, win.h:880-923) and
 *    the sub-block layout written by rm_turbo_rx_lut (rm_turbo.c:249-273,
 *    turbodecoder_iter.h:59-69, 90-97).
 *
 * The reference processes the window decoders in a sub-block-interleaved
 * ("SB") order so that SIMD lane s holds sub-block s.  This restatement keeps
 * every array in natural bit order and loops over (sub-block, step) explicitly;
 * the arithmetic per (sub-block, step) is identical, and the SB re-permuted QPP
 * tables of the reference are the natural tables conjugated by that relabeling.
 */
#include "tdec_oracle.h"

#include <stdlib.h>
#include <string.h>

#define INF 10000
#define WIN_OVERLAP 40

static const uint16_t cb_sizes[188] = {
    40,   48,   56,   64,   72,   80,   88,   96,   104,  112,  120,  128,  136,  144,  152,  160,  168,  176,  184,
    192,  200,  208,  216,  224,  232,  240,  248,  256,  264,  272,  280,  288,  296,  304,  312,  320,  328,  336,
    344,  352,  360,  368,  376,  384,  392,  400,  408,  416,  424,  432,  440,  448,  456,  464,  472,  480,  488,
    496,  504,  512,  528,  544,  560,  576,  592,  608,  624,  640,  656,  672,  688,  704,  720,  736,  752,  768,
    784,  800,  816,  832,  848,  864,  880,  896,  912,  928,  944,  960,  976,  992,  1008, 1024, 1056, 1088, 1120,
    1152, 1184, 1216, 1248, 1280, 1312, 1344, 1376, 1408, 1440, 1472, 1504, 1536, 1568, 1600, 1632, 1664, 1696, 1728,
    1760, 1792, 1824, 1856, 1888, 1920, 1952, 1984, 2016, 2048, 2112, 2176, 2240, 2304, 2368, 2432, 2496, 2560, 2624,
    2688, 2752, 2816, 2880, 2944, 3008, 3072, 3136, 3200, 3264, 3328, 3392, 3456, 3520, 3584, 3648, 3712, 3776, 3840,
    3904, 3968, 4032, 4096, 4160, 4224, 4288, 4352, 4416, 4480, 4544, 4608, 4672, 4736, 4800, 4864, 4928, 4992, 5056,
    5120, 5184, 5248, 5312, 5376, 5440, 5504, 5568, 5632, 5696, 5760, 5824, 5888, 5952, 6016, 6080, 6144};

/* 36.212 Table 5.1.3-3 QPP coefficients (tc_interl_lte.c:39-61). */
static const uint16_t qpp_f1[188] = {
    3,   7,   19,  7,   7,   11,  5,   11,  7,   41,  103, 15,  9,   17,  9,   21,  101, 21,  57, 23,  13,
    27,  11,  27,  85,  29,  33,  15,  17,  33,  103, 19,  19,  37,  19,  21,  21,  115, 193, 21, 133, 81,
    45,  23,  243, 151, 155, 25,  51,  47,  91,  29,  29,  247, 29,  89,  91,  157, 55,  31,  17, 35,  227,
    65,  19,  37,  41,  39,  185, 43,  21,  155, 79,  139, 23,  217, 25,  17,  127, 25,  239, 17, 137, 215,
    29,  15,  147, 29,  59,  65,  55,  31,  17,  171, 67,  35,  19,  39,  19,  199, 21,  211, 21, 43,  149,
    45,  49,  71,  13,  17,  25,  183, 55,  127, 27,  29,  29,  57,  45,  31,  59,  185, 113, 31, 17,  171,
    209, 253, 367, 265, 181, 39,  27,  127, 143, 43,  29,  45,  157, 47,  13,  111, 443, 51,  51, 451, 257,
    57,  313, 271, 179, 331, 363, 375, 127, 31,  33,  43,  33,  477, 35,  233, 357, 337, 37,  71, 71,  37,
    39,  127, 39,  39,  31,  113, 41,  251, 43,  21,  43,  45,  45,  161, 89,  323, 47,  23,  47, 263};
static const uint16_t qpp_f2[188] = {
    10,  12,  42,  16,  18,  20,  22,  24,  26,  84,  90,  32,  34,  108, 38,  120, 84,  44,  46,  48,  50,
    52,  36,  56,  58,  60,  62,  32,  198, 68,  210, 36,  74,  76,  78,  120, 82,  84,  86,  44,  90,  46,
    94,  48,  98,  40,  102, 52,  106, 72,  110, 168, 114, 58,  118, 180, 122, 62,  84,  64,  66,  68,  420,
    96,  74,  76,  234, 80,  82,  252, 86,  44,  120, 92,  94,  48,  98,  80,  102, 52,  106, 48,  110, 112,
    114, 58,  118, 60,  122, 124, 84,  64,  66,  204, 140, 72,  74,  76,  78,  240, 82,  252, 86,  88,  60,
    92,  846, 48,  28,  80,  102, 104, 954, 96,  110, 112, 114, 116, 354, 120, 610, 124, 420, 64,  66,  136,
    420, 216, 444, 456, 468, 80,  164, 504, 172, 88,  300, 92,  188, 96,  28,  240, 204, 104, 212, 192, 220,
    336, 228, 232, 236, 120, 244, 248, 168, 64,  130, 264, 134, 408, 138, 280, 142, 480, 146, 444, 120, 152,
    462, 234, 158, 80,  96,  902, 166, 336, 170, 86,  174, 176, 178, 120, 182, 184, 186, 94,  190, 480};

int oracle_cb_index(uint32_t K)
{
  for (int i = 0; i < 188; i++) {
    if (cb_sizes[i] == K) {
      return i;
    }
  }
  return -1;
}

uint32_t oracle_cb_size(int idx) { return (idx >= 0 && idx < 188) ? cb_sizes[idx] : 0; }

/* turbodecoder.c:381-393 (AVX2 build): 16 / 8 / 0 sub-blocks. */
uint32_t oracle_nof_subblocks(uint32_t K)
{
  if (K % 16 == 0 && K > 800) {
    return 16;
  }
  if (K % 8 == 0 && K > 400) {
    return 8;
  }
  return 0;
}

/* tc_interl_lte.c:69-107 with interl_win == 1 (natural domain). */
int oracle_qpp(uint32_t K, uint16_t* fwd, uint16_t* rev)
{
  int idx = oracle_cb_index(K);
  if (idx < 0) {
    return -1;
  }
  uint64_t f1 = qpp_f1[idx], f2 = qpp_f2[idx];
  for (uint64_t i = 0; i < K; i++) {
    uint64_t j = (f1 * i + f2 * i * i) % K;
    fwd[i]     = (uint16_t)j;
    if (rev) {
      rev[j] = (uint16_t)i;
    }
  }
  return 0;
}

static inline int16_t sat16(int v) { return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v)); }
static inline int16_t wrap16(int v) { return (int16_t)v; }
static inline int16_t max16(int16_t a, int16_t b) { return a > b ? a : b; }

/* ------------------------------------------------------------------------- */
/* Window decoder (turbodecoder_win.h:480-832), one sub-block at a time.      */
/* ------------------------------------------------------------------------- */

/* One backward trellis step, saturating (win.h:641-664). */
static void win_beta_step(int16_t o[8], int16_t x, int16_t y)
{
  int16_t xy = sat16(x + y);
  int16_t n[8];
  n[0] = max16(o[0], sat16(o[4] + xy));
  n[1] = max16(sat16(o[0] + xy), o[4]);
  n[2] = max16(sat16(o[1] + x), sat16(o[5] + y));
  n[3] = max16(sat16(o[1] + y), sat16(o[5] + x));
  n[4] = max16(sat16(o[2] + y), sat16(o[6] + x));
  n[5] = max16(sat16(o[2] + x), sat16(o[6] + y));
  n[6] = max16(sat16(o[3] + xy), o[7]);
  n[7] = max16(o[3], sat16(o[7] + xy));
  memcpy(o, n, sizeof(n));
}

/* Forward trellis candidates (win.h:767-785): c0 = bit-0 branch, c1 = bit-1. */
static void win_alpha_cand(const int16_t o[8], int16_t x, int16_t y, int16_t c0[8], int16_t c1[8])
{
  int16_t xy = sat16(x + y);
  c0[0]      = o[0];
  c0[1]      = sat16(o[3] + y);
  c0[2]      = sat16(o[4] + y);
  c0[3]      = o[7];
  c0[4]      = o[1];
  c0[5]      = sat16(o[2] + y);
  c0[6]      = sat16(o[5] + y);
  c0[7]      = o[6];
  c1[0]      = sat16(o[1] + xy);
  c1[1]      = sat16(o[2] + x);
  c1[2]      = sat16(o[5] + x);
  c1[3]      = sat16(o[6] + xy);
  c1[4]      = sat16(o[0] + xy);
  c1[5]      = sat16(o[3] + x);
  c1[6]      = sat16(o[4] + x);
  c1[7]      = sat16(o[7] + xy);
}

/* normalize() at win.h:480-498 (16-bit: subtract state 0, saturating). */
static void win_norm(int16_t o[8])
{
  for (int i = 1; i < 8; i++) {
    o[i] = sat16(o[i] - o[0]);
  }
  o[0] = 0;
}

/* beta_trellis (win.h:500-548): the last sub-block's end state from the tail, int16 wrap. */
static void win_trellis(const int16_t* xt, const int16_t* yt, int16_t o[8])
{
  o[0] = 0;
  for (int i = 1; i < 8; i++) {
    o[i] = -INF;
  }
  for (int t = 2; t >= 0; t--) {
    int16_t x = xt[t], y = yt[t], xy = wrap16(x + y), mb[8], n[8];
    mb[0] = wrap16(o[4] + xy);
    mb[1] = o[4];
    mb[2] = wrap16(o[5] + y);
    mb[3] = wrap16(o[5] + x);
    mb[4] = wrap16(o[6] + x);
    mb[5] = wrap16(o[6] + y);
    mb[6] = o[7];
    mb[7] = wrap16(o[7] + xy);
    n[0]  = o[0];
    n[1]  = wrap16(o[0] + xy);
    n[2]  = wrap16(o[1] + x);
    n[3]  = wrap16(o[1] + y);
    n[4]  = wrap16(o[2] + y);
    n[5]  = wrap16(o[2] + x);
    n[6]  = wrap16(o[3] + xy);
    n[7]  = o[3];
    for (int i = 0; i < 8; i++) {
      o[i] = max16(mb[i], n[i]);
    }
  }
}

/*
 * One window-MAP constituent decode (tdec_win*_dec, win.h:860-868).
 *  x[0..K+2]: systematic input incl. 3 tail values, natural order
 *  app[0..K-1] or NULL: a-priori, added with saturation (win.h:636-639, 762-765)
 *  y[0..K+2]: parity incl. tail
 *  out[0..K-1]: LLR = max1 - max0 (saturating)
 */
static void win_map(uint32_t nsb, uint32_t K, const int16_t* x, const int16_t* app, const int16_t* y, int16_t* out)
{
  const uint32_t L = K / nsb;
  int16_t(*beta)[8] = malloc(sizeof(int16_t[8]) * (size_t)(L + 1) * nsb);
  int16_t tb[16][8], ta[16][8];

#define XK(s, k) (app ? sat16(x[(s)*L + (k)] + app[(s)*L + (k)]) : x[(s)*L + (k)])
#define YK(s, k) (y[(s)*L + (k)])

  /* beta, j == 0 pass: training over the first 40 steps of each sub-block (win.h:622-630). */
  for (uint32_t s = 0; s < nsb; s++) {
    int16_t o[8];
    for (int i = 0; i < 8; i++) {
      o[i] = -INF;
    }
    for (int k = WIN_OVERLAP - 1; k >= 0; k--) {
      win_beta_step(o, XK(s, k), YK(s, k));
      if (k % 2 == 0 && k != 0) {
        win_norm(o);
      }
    }
    memcpy(tb[s], o, sizeof(o));
  }
  /* beta, j == 1 pass: sub-block s starts from sub-block s+1's training state
   * (move_right), the last one from the tail trellis (win.h:577-620). */
  for (uint32_t s = 0; s < nsb; s++) {
    int16_t o[8];
    if (s + 1 < nsb) {
      memcpy(o, tb[s + 1], sizeof(o));
    } else {
      win_trellis(&x[K], &y[K], o);
    }
    int16_t(*b)[8] = &beta[(size_t)s * (L + 1)];
    memcpy(b[L], o, sizeof(o));
    for (int k = (int)L - 1; k >= 0; k--) {
      win_beta_step(o, XK(s, k), YK(s, k));
      memcpy(b[k], o, sizeof(o));
      if (k % 2 == 0 && k != 0) {
        win_norm(o);
      }
    }
  }

  /* alpha, j == 0 pass: training over the last 40 steps of each sub-block (win.h:747-756). */
  for (uint32_t s = 0; s < nsb; s++) {
    int16_t o[8], c0[8], c1[8];
    for (int i = 0; i < 8; i++) {
      o[i] = -INF;
    }
    for (int k = 0; k < WIN_OVERLAP; k++) {
      win_alpha_cand(o, XK(s, L - WIN_OVERLAP + k), YK(s, L - WIN_OVERLAP + k), c0, c1);
      for (int i = 0; i < 8; i++) {
        o[i] = max16(c0[i], c1[i]);
      }
      if (k % 2 == 0 && k != 0) {
        win_norm(o);
      }
    }
    memcpy(ta[s], o, sizeof(o));
  }
  /* alpha, j == 1 pass: sub-block s starts from s-1's training state (move_left),
   * sub-block 0 from the known zero state (win.h:715-746, 758-830). */
  for (uint32_t s = 0; s < nsb; s++) {
    int16_t o[8], c0[8], c1[8];
    if (s == 0) {
      o[0] = 0;
      for (int i = 1; i < 8; i++) {
        o[i] = -INF;
      }
    } else {
      memcpy(o, ta[s - 1], sizeof(o));
    }
    int16_t(*b)[8] = &beta[(size_t)s * (L + 1)];
    for (uint32_t k = 0; k < L; k++) {
      win_alpha_cand(o, XK(s, k), YK(s, k), c0, c1);
      int16_t m0 = -32768, m1 = -32768;
      for (int i = 0; i < 8; i++) {
        m0 = max16(m0, sat16(b[k + 1][i] + c0[i]));
        m1 = max16(m1, sat16(b[k + 1][i] + c1[i]));
      }
      out[s * L + k] = sat16(m1 - m0);
      for (int i = 0; i < 8; i++) {
        o[i] = max16(c0[i], c1[i]);
      }
      if (k % 2 == 0 && k != 0) {
        win_norm(o);
      }
    }
  }
#undef XK
#undef YK
  free(beta);
}

/* ------------------------------------------------------------------------- */
/* Generic decoder (turbodecoder_gen.c:58-236): full length, int16 wrap.      */
/* ------------------------------------------------------------------------- */
static void gen_map(uint32_t K, const int16_t* x, const int16_t* app, const int16_t* y, int16_t* out)
{
  const uint32_t end = K + 3;
  int16_t(*beta)[8]  = malloc(sizeof(int16_t[8]) * (size_t)(end + 1));
  int16_t o[8];

  beta[end][0] = 0;
  for (int i = 1; i < 8; i++) {
    beta[end][i] = -INF;
  }
  memcpy(o, beta[end], sizeof(o));
  for (int k = (int)end - 1; k >= 0; k--) {
    int16_t xk = x[k];
    if (app && k < (int)K) {
      xk = wrap16(xk + app[k]);
    }
    int16_t yk = y[k], xy = wrap16(xk + yk), mb[8], n[8];
    mb[0] = wrap16(o[4] + xy);
    mb[1] = o[4];
    mb[2] = wrap16(o[5] + yk);
    mb[3] = wrap16(o[5] + xk);
    mb[4] = wrap16(o[6] + xk);
    mb[5] = wrap16(o[6] + yk);
    mb[6] = o[7];
    mb[7] = wrap16(o[7] + xy);
    n[0]  = o[0];
    n[1]  = wrap16(o[0] + xy);
    n[2]  = wrap16(o[1] + xk);
    n[3]  = wrap16(o[1] + yk);
    n[4]  = wrap16(o[2] + yk);
    n[5]  = wrap16(o[2] + xk);
    n[6]  = wrap16(o[3] + xy);
    n[7]  = o[3];
    for (int i = 0; i < 8; i++) {
      o[i]       = max16(mb[i], n[i]);
      beta[k][i] = o[i];
    }
    if (k % 4 == 0 && k < (int)K) {
      for (int i = 1; i < 8; i++) {
        o[i] = wrap16(o[i] - o[0]);
      }
      o[0] = 0;
    }
  }

  o[0] = 0;
  for (int i = 1; i < 8; i++) {
    o[i] = -INF;
  }
  for (uint32_t k = 1; k <= K; k++) {
    int16_t xk = x[k - 1];
    if (app) {
      xk = wrap16(xk + app[k - 1]);
    }
    int16_t yk = y[k - 1], xy = wrap16(xk + yk), c0[8], c1[8];
    c0[0] = o[0];
    c0[1] = wrap16(o[3] + yk);
    c0[2] = wrap16(o[4] + yk);
    c0[3] = o[7];
    c0[4] = o[1];
    c0[5] = wrap16(o[2] + yk);
    c0[6] = wrap16(o[5] + yk);
    c0[7] = o[6];
    c1[0] = wrap16(o[1] + xy);
    c1[1] = wrap16(o[2] + xk);
    c1[2] = wrap16(o[5] + xk);
    c1[3] = wrap16(o[6] + xy);
    c1[4] = wrap16(o[0] + xy);
    c1[5] = wrap16(o[3] + xk);
    c1[6] = wrap16(o[4] + xk);
    c1[7] = wrap16(o[7] + xy);
    int16_t m0 = wrap16(c0[0] + beta[k][0]), m1 = wrap16(c1[0] + beta[k][0]);
    for (int i = 1; i < 8; i++) {
      m0 = max16(m0, wrap16(c0[i] + beta[k][i]));
      m1 = max16(m1, wrap16(c1[i] + beta[k][i]));
    }
    for (int i = 0; i < 8; i++) {
      o[i] = max16(c0[i], c1[i]);
    }
    if (k % 4 == 0) {
      for (int i = 1; i < 8; i++) {
        o[i] = wrap16(o[i] - o[0]);
      }
      o[0] = 0;
    }
    out[k - 1] = wrap16(m1 - m0);
  }
  free(beta);
}

/* ------------------------------------------------------------------------- */
/* Half-iteration driver (turbodecoder_iter.h:72-144) and run_all.            */
/* ------------------------------------------------------------------------- */
struct oracle_tdec_state {
  uint32_t K, nsb;
  int16_t *syst, *par0, *par1, *app1, *app2, *ext1, *ext2;
  uint16_t *fwd, *rev;
};

static void state_alloc(struct oracle_tdec_state* st, uint32_t K)
{
  st->K    = K;
  st->nsb  = oracle_nof_subblocks(K);
  st->syst = calloc(K + 3, 2);
  st->par0 = calloc(K + 3, 2);
  st->par1 = calloc(K + 3, 2);
  st->app1 = calloc(K + 3, 2);
  st->app2 = calloc(K + 3, 2);
  st->ext1 = calloc(K + 3, 2);
  st->ext2 = calloc(K + 3, 2);
  st->fwd  = calloc(K, 2);
  st->rev  = calloc(K, 2);
  oracle_qpp(K, st->fwd, st->rev);
}

static void state_free(struct oracle_tdec_state* st)
{
  free(st->syst);
  free(st->par0);
  free(st->par1);
  free(st->app1);
  free(st->app2);
  free(st->ext1);
  free(st->ext2);
  free(st->fwd);
  free(st->rev);
}

/*
 * Input extraction.
 *  natural: [S0 P0_0 P1_0 S1 ...] 3K values, then tail: S,P0 x3 then app2,P1 x3
 *           (turbodecoder_gen.c:238-258, turbodecoder_win.h:880-923)
 *  SB:      [syst | pad32 | par0 | pad32 | par1 | pad32 | tail12], within each
 *           stream bit s*L+k sits at k*nsb+s (rm_turbo.c:249-273, iter.h:59-69)
 */
static void extract_input(struct oracle_tdec_state* st, const int16_t* in, int layout_sb)
{
  const uint32_t K = st->K, nsb = st->nsb;
  const int16_t* tail;
  if (layout_sb && nsb) {
    const uint32_t L = K / nsb;
    for (uint32_t s = 0; s < nsb; s++) {
      for (uint32_t k = 0; k < L; k++) {
        st->syst[s * L + k] = in[k * nsb + s];
        st->par0[s * L + k] = in[(K + 32) + k * nsb + s];
        st->par1[s * L + k] = in[2 * (K + 32) + k * nsb + s];
      }
    }
    tail = &in[3 * (K + 32)];
  } else {
    for (uint32_t i = 0; i < K; i++) {
      st->syst[i] = in[3 * i];
      st->par0[i] = in[3 * i + 1];
      st->par1[i] = in[3 * i + 2];
    }
    tail = &in[3 * K];
  }
  for (int t = 0; t < 3; t++) {
    st->syst[K + t] = tail[2 * t];
    st->par0[K + t] = tail[2 * t + 1];
    st->app2[K + t] = tail[6 + 2 * t];
    st->par1[K + t] = tail[6 + 2 * t + 1];
  }
}

static void constituent(struct oracle_tdec_state* st, const int16_t* x, const int16_t* app, const int16_t* y, int16_t* out)
{
  if (st->nsb) {
    win_map(st->nsb, st->K, x, app, y, out);
  } else {
    gen_map(st->K, x, app, y, out);
  }
}

static void half_iteration(struct oracle_tdec_state* st, int n_iter)
{
  const uint32_t K = st->K;
  if (n_iter % 2 == 0) {
    if (n_iter) {
      for (uint32_t i = 0; i < K; i++) { /* srsran_vec_sub_sss: non-saturating */
        st->app1[i] = wrap16(st->app1[i] - st->ext1[i]);
      }
    }
    constituent(st, st->syst, n_iter ? st->app1 : NULL, st->par0, st->ext1);
  } else {
    if (n_iter > 1) {
      for (uint32_t i = 0; i < K; i++) {
        st->ext1[i] = wrap16(st->ext1[i] - st->app1[i]);
      }
    }
    for (uint32_t i = 0; i < K; i++) { /* srsran_vec_lut_sss(ext1, deinter, app2) */
      st->app2[st->rev[i]] = st->ext1[i];
    }
    constituent(st, st->app2, NULL, st->par1, st->ext2);
    for (uint32_t i = 0; i < K; i++) { /* srsran_vec_lut_sss(ext2, inter, app1) */
      st->app1[st->fwd[i]] = st->ext2[i];
    }
  }
}

static void decision(const int16_t* llr, uint8_t* out, uint32_t K)
{
  for (uint32_t i = 0; i < K / 8; i++) {
    uint8_t b = 0;
    for (int j = 0; j < 8; j++) {
      b |= (uint8_t)((llr[8 * i + j] > 0) << (7 - j));
    }
    out[i] = b;
  }
}

int oracle_tdec_run(uint32_t K, const int16_t* input, int layout_sb, uint32_t nof_iterations, uint8_t* output, int16_t* trace)
{
  if (oracle_cb_index(K) < 0 || nof_iterations < 1) {
    return -1;
  }
  struct oracle_tdec_state st;
  state_alloc(&st, K);
  extract_input(&st, input, layout_sb);
  int n = 0;
  do {
    half_iteration(&st, n);
    if (trace) {
      memcpy(&trace[(size_t)n * K], n % 2 ? st.app1 : st.ext1, K * sizeof(int16_t));
    }
    n++;
  } while (n < (int)nof_iterations);
  decision(n % 2 ? st.ext1 : st.app1, output, K);
  state_free(&st);
  return 0;
}

int oracle_tdec_run_batch(uint32_t K,
                          const int16_t* input,
                          uint32_t       in_stride,
                          int            layout_sb,
                          uint32_t       nof_iterations,
                          uint8_t*       output,
                          uint32_t       nof_cb)
{
  for (uint32_t c = 0; c < nof_cb; c++) {
    if (oracle_tdec_run(K, &input[(size_t)c * in_stride], layout_sb, nof_iterations, &output[(size_t)c * (K / 8)], NULL)) {
      return -1;
    }
  }
  return 0;
}

/* ------------------------------------------------------------------------- */
/* Turbo encoder (turbocoder.c:77-185), used to synthesise test codewords.    */
/* ------------------------------------------------------------------------- */
int oracle_tcod_encode(uint32_t K, const uint8_t* bits, uint8_t* out)
{
  uint16_t* fwd = malloc(K * sizeof(uint16_t));
  if (oracle_qpp(K, fwd, NULL)) {
    free(fwd);
    return -1;
  }
  uint8_t r1[3] = {0, 0, 0}, r2[3] = {0, 0, 0};
  uint32_t k = 0;
  for (uint32_t i = 0; i < K; i++) {
    uint8_t bit = bits[i] & 1, in, p;
    out[k++]    = bit;
    in          = bit ^ (r1[2] ^ r1[1]);
    p           = r1[2] ^ (r1[0] ^ in);
    r1[2]       = r1[1];
    r1[1]       = r1[0];
    r1[0]       = in;
    out[k++]    = p;
    bit         = bits[fwd[i]] & 1;
    in          = bit ^ (r2[2] ^ r2[1]);
    p           = r2[2] ^ (r2[0] ^ in);
    r2[2]       = r2[1];
    r2[1]       = r2[0];
    r2[0]       = in;
    out[k++]    = p;
  }
  for (int e = 0; e < 2; e++) {
    uint8_t* r = e ? r2 : r1;
    for (int j = 0; j < 3; j++) {
      uint8_t bit = r[2] ^ r[1], in, p;
      out[k++]    = bit;
      in          = bit ^ (r[2] ^ r[1]);
      p           = r[2] ^ (r[0] ^ in);
      r[2]        = r[1];
      r[1]        = r[0];
      r[0]        = in;
      out[k++]    = p;
    }
  }
  free(fwd);
  return 0;
}

/* Natural (3K+12) -> sub-block layout 3(K+32)+12, as rm_turbo_rx_lut would emit. */
int oracle_natural_to_sb(uint32_t K, const int16_t* in, int16_t* out)
{
  uint32_t nsb = oracle_nof_subblocks(K);
  if (!nsb) {
    memcpy(out, in, (3 * K + 12) * sizeof(int16_t));
    return 0;
  }
  uint32_t L = K / nsb;
  memset(out, 0, (3 * (K + 32) + 12) * sizeof(int16_t));
  for (uint32_t n = 0; n < K; n++) {
    uint32_t sb = (n % L) * nsb + n / L;
    for (int j = 0; j < 3; j++) {
      out[j * (K + 32) + sb] = in[3 * n + j];
    }
  }
  memcpy(&out[3 * (K + 32)], &in[3 * K], 12 * sizeof(int16_t));
  return 0;
}

/* ======================= 8-bit window decoders (turbodecoder_win.h WINIMP_IS_SSE8 / _AVX8) =======================
 * C form of oracle/tdec8.py (the same schedule, pinned to the reference's decoders compiled into oracle/_ref by
 * tests/test_tdec8bit.py and tests/test_sch_oracle.py): int8 metrics with saturating add / sub, normalisation
 * by the state maximum at every step but k = 0, the tail trellis saturating upwards only, LLR m1 - m0 halved;
 * training windows of 40 steps over the neighbouring sub-block.  Input in the 8-bit decoder's sub-block layout
 * (rm_turbo_rx_lut_8bit): syst | 32 | parity0 | 32 | parity1 | 32 | tail. */
#define OVL8 40

/* srsran_tdec_autoimp_get_subblocks_8bit of an AVX2 build (turbodecoder.c:410-424): 32 / 16 / 8 / 0 */
uint32_t oracle_nof_subblocks_8bit(uint32_t K)
{
  if (K % 32 == 0 && K > 2048) {
    return 32;
  }
  if (K % 16 == 0 && K > 800) {
    return 16;
  }
  if (K % 8 == 0 && K > 400) {
    return 8;
  }
  return 0;
}

static int s8(int v) { return v > 127 ? 127 : (v < -128 ? -128 : v); }
static int t8(int a, int b) /* beta_trellis sadd: upper clamp, int8 wrap below */
{
  const int z = a + b;
  return z > 127 ? 127 : (int)(int8_t)z;
}
static void norm8(int k, int* o)
{
  if (k) {
    int m = o[0];
    for (int i = 1; i < 8; i++) {
      m = o[i] > m ? o[i] : m;
    }
    for (int i = 0; i < 8; i++) {
      o[i] = s8(o[i] - m);
    }
  }
}
static int max8(int a, int b) { return a > b ? a : b; }
static void beta8(int* o, int x, int y)
{
  const int xy = s8(x + y);
  int       n[8];
  n[0] = max8(s8(o[4] + xy), o[0]);
  n[1] = max8(o[4], s8(o[0] + xy));
  n[2] = max8(s8(o[5] + y), s8(o[1] + x));
  n[3] = max8(s8(o[5] + x), s8(o[1] + y));
  n[4] = max8(s8(o[6] + x), s8(o[2] + y));
  n[5] = max8(s8(o[6] + y), s8(o[2] + x));
  n[6] = max8(o[7], s8(o[3] + xy));
  n[7] = max8(s8(o[7] + xy), o[3]);
  memcpy(o, n, sizeof(n));
}
static void alpha8(const int* o, int x, int y, int* mb, int* nw)
{
  const int xy = s8(x + y);
  mb[0] = o[0], mb[1] = s8(o[3] + y), mb[2] = s8(o[4] + y), mb[3] = o[7];
  mb[4] = o[1], mb[5] = s8(o[2] + y), mb[6] = s8(o[5] + y), mb[7] = o[6];
  nw[0] = s8(o[1] + xy), nw[1] = s8(o[2] + x), nw[2] = s8(o[5] + x), nw[3] = s8(o[6] + xy);
  nw[4] = s8(o[0] + xy), nw[5] = s8(o[3] + x), nw[6] = s8(o[4] + x), nw[7] = s8(o[7] + xy);
}

/* one MAP pass: X, A (optional), P in SB order with the tail at [K, K + 3); OUT = extrinsic (K) */
static void map8(const int* X, const int* A, const int* P, int* OUT, int K, int nsb, int* beta, int* train)
{
  const int Ls = K / nsb;
#define XA(q) (A ? s8(A[q] + X[q]) : X[q])
  for (int d = 0; d < nsb; d++) { /* beta training from unknown (0) states */
    int* o = &train[8 * d];
    memset(o, 0, 8 * sizeof(int));
    for (int k = OVL8 - 1; k >= 0; k--) {
      beta8(o, XA(k * nsb + d), P[k * nsb + d]);
      norm8(k, o);
    }
  }
  for (int d = 0; d < nsb; d++) {
    int o[8];
    if (d < nsb - 1) {
      memcpy(o, &train[8 * (d + 1)], sizeof(o));
    } else { /* beta_trellis over the tail */
      int t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int k = K + 2; k >= K; k--) {
        const int x = X[k], y = P[k], xy = t8(x, y);
        int       mb[8] = {t8(t[4], xy), t[4], t8(t[5], y), t8(t[5], x), t8(t[6], x), t8(t[6], y), t[7], t8(t[7], xy)};
        int       nw[8] = {t[0], t8(t[0], xy), t8(t[1], x), t8(t[1], y), t8(t[2], y), t8(t[2], x), t8(t[3], xy), t[3]};
        for (int i = 0; i < 8; i++) {
          t[i] = max8(mb[i], nw[i]);
        }
      }
      memcpy(o, t, sizeof(o));
    }
    memcpy(&beta[((size_t)Ls * nsb + d) * 8], o, sizeof(o));
    for (int k = Ls - 1; k >= 0; k--) {
      beta8(o, XA(k * nsb + d), P[k * nsb + d]);
      memcpy(&beta[((size_t)k * nsb + d) * 8], o, sizeof(o)); /* before normalisation */
      norm8(k, o);
    }
  }
  for (int d = 0; d < nsb; d++) { /* alpha training over the sub-block's last 40 steps */
    int* o = &train[8 * d];
    memset(o, 0, 8 * sizeof(int));
    for (int k = 0; k < OVL8; k++) {
      const int q = (Ls - OVL8 + k) * nsb + d;
      int       mb[8], nw[8];
      alpha8(o, XA(q), P[q], mb, nw);
      for (int i = 0; i < 8; i++) {
        o[i] = max8(mb[i], nw[i]);
      }
      norm8(k, o);
    }
  }
  for (int d = nsb - 1; d >= 0; d--) { /* descending: sub-block d starts from d - 1's training, still intact */
    int o[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (d > 0) {
      memcpy(o, &train[8 * (d - 1)], sizeof(o));
    }
    for (int k = 0; k < Ls; k++) {
      const int q = k * nsb + d;
      int       mb[8], nw[8];
      alpha8(o, XA(q), P[q], mb, nw);
      const int* b  = &beta[((size_t)(k + 1) * nsb + d) * 8];
      int        m0 = s8(b[0] + mb[0]), m1 = s8(b[0] + nw[0]);
      for (int i = 1; i < 8; i++) {
        m0 = max8(m0, s8(b[i] + mb[i]));
        m1 = max8(m1, s8(b[i] + nw[i]));
      }
      OUT[q] = s8(m1 - m0) >> 1;
      for (int i = 0; i < 8; i++) {
        o[i] = max8(mb[i], nw[i]);
      }
      norm8(k, o);
    }
  }
#undef XA
}

/* srsran_tdec_run_all_8bit on one block of an 8-bit decoder class (nsb 16 / 32, SB layout input):
 * nof_iterations half-iterations; output = decision bytes; trace (optional, nof_iterations * K int8) = the
 * latest output after each half-iteration in natural order. */
int oracle_tdec8_run(uint32_t K, const int8_t* in, uint32_t nof_iterations, uint8_t* output, int8_t* trace)
{
  const int nsb = (int)oracle_nof_subblocks_8bit(K);
  if ((nsb != 16 && nsb != 32) || nof_iterations < 1) {
    return -1;
  }
  const int Ls = (int)K / nsb;
  uint16_t* fwd = malloc(K * sizeof(uint16_t));
  int*      SY  = calloc(K + 3, sizeof(int));
  int*      P0  = calloc(K + 3, sizeof(int));
  int*      P1  = calloc(K + 3, sizeof(int));
  int*      A1  = calloc(K, sizeof(int));
  int*      A2  = calloc(K + 3, sizeof(int));
  int*      E1  = calloc(K, sizeof(int));
  int*      E2  = calloc(K, sizeof(int));
  int*      fsb = malloc(K * sizeof(int));
  int*      beta  = malloc((size_t)(Ls + 1) * nsb * 8 * sizeof(int));
  int*      train = malloc((size_t)nsb * 8 * sizeof(int));
  oracle_qpp(K, fwd, NULL);
  for (int q = 0; q < (int)K; q++) { /* QPP forward table in SB slot order (tc_interl_lte.c:88-106, win = nsb) */
    const int n  = (q % nsb) * Ls + q / nsb;
    const int fn = fwd[n];
    fsb[q]       = (fn % Ls) * nsb + fn / Ls;
  }
  for (uint32_t q = 0; q < K; q++) {
    SY[q] = in[q];
    P0[q] = in[K + 32 + q];
    P1[q] = in[2 * (K + 32) + q];
  }
  const int8_t* tail = &in[3 * (K + 32)];
  for (int j = 0; j < 3; j++) {
    SY[K + j] = tail[2 * j];
    P0[K + j] = tail[2 * j + 1];
    A2[K + j] = tail[6 + 2 * j];
    P1[K + j] = tail[7 + 2 * j];
  }
  for (uint32_t n = 0; n < nof_iterations; n++) {
    if (n % 2 == 0) {
      if (n) {
        for (uint32_t q = 0; q < K; q++) {
          A1[q] = s8(A1[q] - E1[q]);
        }
      }
      map8(SY, n ? A1 : NULL, P0, E1, (int)K, nsb, beta, train);
    } else {
      if (n > 1) {
        for (uint32_t q = 0; q < K; q++) {
          E1[q] = s8(E1[q] - A1[q]);
        }
      }
      for (uint32_t j = 0; j < K; j++) {
        A2[j] = E1[fsb[j]];
      }
      map8(A2, NULL, P1, E2, (int)K, nsb, beta, train);
      for (uint32_t i = 0; i < K; i++) {
        A1[fsb[i]] = E2[i];
      }
    }
    if (trace) {
      const int* src = ((n + 1) % 2) ? E1 : A1;
      for (uint32_t i = 0; i < K; i++) {
        trace[(size_t)n * K + i] = (int8_t)src[(i % Ls) * nsb + i / Ls];
      }
    }
  }
  const int* src = (nof_iterations % 2) ? E1 : A1;
  for (uint32_t b = 0; b < K / 8; b++) {
    uint8_t v = 0;
    for (int t = 0; t < 8; t++) {
      const uint32_t i = 8 * b + t;
      v |= (uint8_t)((src[(i % Ls) * nsb + i / Ls] > 0) << (7 - t));
    }
    output[b] = v;
  }
  free(fwd), free(SY), free(P0), free(P1), free(A1), free(A2), free(E1), free(E2), free(fsb), free(beta), free(train);
  return 0;
}
