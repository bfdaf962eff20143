/*
 * synth/tx.c -- synthetic eNB-side transmitter for tests and bench inputs.
 *
 * NOT the product and NOT the oracle: this generates the signals the receive path decodes
 * (bench.py's workloads, tests' subframes).  Written from 3GPP TS 36.212 / 36.211 directly:
 *   CRC attachment              36.212 5.1.1 (gCRC24A, gCRC24B)
 *   code-block segmentation     36.212 5.1.2 (blocks of K- first)
 *   turbo encoding (PCCC, QPP)  36.212 5.1.3.2, Table 5.1.3-3, trellis termination 5.1.3.2.2
 *   rate matching               36.212 5.1.4.1 (sub-block interleaver, bit collection, selection;
 *                               N_cb = K_w as srsRAN's receiver assumes, rm_turbo.c:175-248)
 *   code-block concatenation    36.212 5.1.5, E per block from G' = G / (N_L Q_m)
 *   pseudo-random sequence      36.211 7.2 (Nc = 1600)
 * tests/test_synth.py checks every piece against oracle/ (itself pinned to the reference).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define CRC24A 0x1864CFBu
#define CRC24B 0x1800063u

static const uint16_t kK[188] = {
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

/* 36.212 Table 5.1.3-3 */
static const uint16_t kF1[188] = {
    3,   7,   19,  7,   7,   11,  5,   11,  7,   41,  103, 15,  9,   17,  9,   21,  101, 21,  57, 23,  13,
    27,  11,  27,  85,  29,  33,  15,  17,  33,  103, 19,  19,  37,  19,  21,  21,  115, 193, 21, 133, 81,
    45,  23,  243, 151, 155, 25,  51,  47,  91,  29,  29,  247, 29,  89,  91,  157, 55,  31,  17, 35,  227,
    65,  19,  37,  41,  39,  185, 43,  21,  155, 79,  139, 23,  217, 25,  17,  127, 25,  239, 17, 137, 215,
    29,  15,  147, 29,  59,  65,  55,  31,  17,  171, 67,  35,  19,  39,  19,  199, 21,  211, 21, 43,  149,
    45,  49,  71,  13,  17,  25,  183, 55,  127, 27,  29,  29,  57,  45,  31,  59,  185, 113, 31, 17,  171,
    209, 253, 367, 265, 181, 39,  27,  127, 143, 43,  29,  45,  157, 47,  13,  111, 443, 51,  51, 451, 257,
    57,  313, 271, 179, 331, 363, 375, 127, 31,  33,  43,  33,  477, 35,  233, 357, 337, 37,  71, 71,  37,
    39,  127, 39,  39,  31,  113, 41,  251, 43,  21,  43,  45,  45,  161, 89,  323, 47,  23,  47, 263};
static const uint16_t kF2[188] = {
    10,  12,  42,  16,  18,  20,  22,  24,  26,  84,  90,  32,  34,  108, 38,  120, 84,  44,  46,  48,  50,
    52,  36,  56,  58,  60,  62,  32,  198, 68,  210, 36,  74,  76,  78,  120, 82,  84,  86,  44,  90,  46,
    94,  48,  98,  40,  102, 52,  106, 72,  110, 168, 114, 58,  118, 180, 122, 62,  84,  64,  66,  68,  420,
    96,  74,  76,  234, 80,  82,  252, 86,  44,  120, 92,  94,  48,  98,  80,  102, 52,  106, 48,  110, 112,
    114, 58,  118, 60,  122, 124, 84,  64,  66,  204, 140, 72,  74,  76,  78,  240, 82,  252, 86,  88,  60,
    92,  846, 48,  28,  80,  102, 104, 954, 96,  110, 112, 114, 116, 354, 120, 610, 124, 420, 64,  66,  136,
    420, 216, 444, 456, 468, 80,  164, 504, 172, 88,  300, 92,  188, 96,  28,  240, 204, 104, 212, 192, 220,
    336, 228, 232, 236, 120, 244, 248, 168, 64,  130, 264, 134, 408, 138, 280, 142, 480, 146, 444, 120, 152,
    462, 234, 158, 80,  96,  902, 166, 336, 170, 86,  174, 176, 178, 120, 182, 184, 186, 94,  190, 480};

/* 36.212 Table 5.1.4-1 inter-column permutation */
static const uint8_t kPerm[32] = {0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30,
                                  1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31};

static int k_index(uint32_t K)
{
  for (int i = 0; i < 188; i++) {
    if (kK[i] == K) {
      return i;
    }
  }
  return -1;
}

/* bit-serial CRC remainder of bits[0..n) (MSB first), zero initial state */
uint32_t synth_crc(uint32_t poly, const uint8_t* bits, uint32_t n)
{
  uint32_t r = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t fb = ((r >> 23) & 1u) ^ (bits[i] & 1u);
    r                 = (r << 1) & 0xFFFFFFu;
    if (fb) {
      r ^= poly & 0xFFFFFFu;
    }
  }
  return r;
}

static void put24(uint8_t* bits, uint32_t v)
{
  for (int i = 0; i < 24; i++) {
    bits[i] = (uint8_t)((v >> (23 - i)) & 1u);
  }
}

/* 36.212 5.1.3.2: d0/d1/d2 of length K + 4 */
int synth_turbo_encode(uint32_t K, const uint8_t* c, uint8_t* d0, uint8_t* d1, uint8_t* d2)
{
  const int ki = k_index(K);
  if (ki < 0) {
    return -1;
  }
  const uint64_t f1 = kF1[ki], f2 = kF2[ki];
  uint32_t       s1 = 0, s2 = 0; /* 3-bit shift registers, bit0 = D^1 */
  uint8_t        xt[3], zt[3], xpt[3], zpt[3];
  for (uint32_t k = 0; k < K; k++) {
    const uint8_t  ck = c[k] & 1u;
    const uint32_t pi = (uint32_t)((f1 * k + f2 * (uint64_t)k * k) % K);
    const uint8_t  cp = c[pi] & 1u;
    /* RSC: feedback g0 = 1 + D^2 + D^3, parity g1 = 1 + D + D^3 */
    uint8_t a = ck ^ ((s1 >> 1) & 1u) ^ ((s1 >> 2) & 1u);
    uint8_t z = a ^ (s1 & 1u) ^ ((s1 >> 2) & 1u);
    s1        = ((s1 << 1) | a) & 7u;
    uint8_t b = cp ^ ((s2 >> 1) & 1u) ^ ((s2 >> 2) & 1u);
    uint8_t zp = b ^ (s2 & 1u) ^ ((s2 >> 2) & 1u);
    s2         = ((s2 << 1) | b) & 7u;
    d0[k]      = ck;
    d1[k]      = z;
    d2[k]      = zp;
  }
  /* trellis termination: input = feedback so the register input is 0 */
  for (int t = 0; t < 3; t++) {
    uint8_t x = ((s1 >> 1) & 1u) ^ ((s1 >> 2) & 1u);
    xt[t]     = x;
    zt[t]     = (uint8_t)(0 ^ (s1 & 1u) ^ ((s1 >> 2) & 1u));
    s1        = (s1 << 1) & 7u;
  }
  for (int t = 0; t < 3; t++) {
    uint8_t x = ((s2 >> 1) & 1u) ^ ((s2 >> 2) & 1u);
    xpt[t]    = x;
    zpt[t]    = (uint8_t)(0 ^ (s2 & 1u) ^ ((s2 >> 2) & 1u));
    s2        = (s2 << 1) & 7u;
  }
  d0[K] = xt[0], d0[K + 1] = zt[1], d0[K + 2] = xpt[0], d0[K + 3] = zpt[1];
  d1[K] = zt[0], d1[K + 1] = xt[2], d1[K + 2] = zpt[0], d1[K + 3] = xpt[2];
  d2[K] = xt[1], d2[K + 1] = zt[2], d2[K + 2] = xpt[1], d2[K + 3] = zpt[2];
  return 0;
}

/* natural srsRAN decoder-input order: [d0_i d1_i d2_i] for i < K + 4 (3K + 12 bits) */
int synth_turbo_encode_natural(uint32_t K, const uint8_t* c, uint8_t* out)
{
  uint8_t* d = malloc(3 * (K + 4));
  if (!d || synth_turbo_encode(K, c, d, d + K + 4, d + 2 * (K + 4))) {
    free(d);
    return -1;
  }
  for (uint32_t i = 0; i < K + 4; i++) {
    out[3 * i]     = d[i];
    out[3 * i + 1] = d[K + 4 + i];
    out[3 * i + 2] = d[2 * (K + 4) + i];
  }
  free(d);
  return 0;
}

/* 36.212 5.1.4.1: e[0..E) from the three streams (2 = NULL marker internally) */
static int rate_match(uint32_t K, uint32_t rv, const uint8_t* d0, const uint8_t* d1, const uint8_t* d2, uint32_t E,
                      uint8_t* e)
{
  const uint32_t D = K + 4, R = (D + 31) / 32, Kp = 32 * R, Nd = Kp - D, Ncb = 3 * Kp;
  uint8_t*       w = malloc(Ncb);
  if (!w) {
    return -1;
  }
  for (uint32_t k = 0; k < Kp; k++) {
    const uint32_t col = kPerm[k / R], row = k % R;
    const uint32_t idx = col + 32 * row;                /* position in y (streams 0, 1) */
    const uint32_t pi2 = (col + 32 * row + 1) % Kp;      /* stream 2 */
    w[k]               = idx < Nd ? 2 : d0[idx - Nd];
    w[Kp + 2 * k]      = idx < Nd ? 2 : d1[idx - Nd];
    w[Kp + 2 * k + 1]  = pi2 < Nd ? 2 : d2[pi2 - Nd];
  }
  const uint32_t k0 = R * (2 * ((Ncb + 8 * R - 1) / (8 * R)) * rv + 2);
  for (uint32_t k = 0, j = 0; k < E; j++) {
    const uint8_t v = w[(k0 + j) % Ncb];
    if (v != 2) {
      e[k++] = v;
    }
  }
  free(w);
  return 0;
}

/* segmentation: C, K+, K-, C+, C-, F (36.212 5.1.2) */
static int segment(uint32_t B, uint32_t* C, uint32_t* Kp, uint32_t* Km, uint32_t* Cp, uint32_t* Cm, uint32_t* F)
{
  const uint32_t Z = 6144;
  uint32_t       Bp;
  if (B <= Z) {
    *C = 1;
    Bp = B;
  } else {
    *C = (B + Z - 24 - 1) / (Z - 24);
    Bp = B + 24 * *C;
  }
  int ip = -1;
  for (int i = 0; i < 188; i++) {
    if ((uint64_t)*C * kK[i] >= Bp) {
      ip = i;
      break;
    }
  }
  if (ip < 0) {
    return -1;
  }
  *Kp = kK[ip];
  if (*C == 1) {
    *Cp = 1, *Km = 0, *Cm = 0;
  } else {
    *Km = ip > 0 ? kK[ip - 1] : 0;
    *Cm = (*C * *Kp - Bp) / (*Kp - *Km);
    *Cp = *C - *Cm;
  }
  *F = *Cp * *Kp + *Cm * *Km - Bp;
  return 0;
}

/* DL-SCH transport channel processing of one TB (36.212 5.3.2): returns bits written (= G) or -1.
 * tb_crc_xor != 0 corrupts the TB CRC (every CB CRC still passes). */
int synth_dlsch_encode(uint32_t tbs, uint32_t Qm, uint32_t Nl, uint32_t rv, uint32_t G, const uint8_t* tb_bytes,
                       uint32_t tb_crc_xor, uint8_t* e)
{
  const uint32_t B = tbs + 24;
  uint32_t       C, Kp, Km, Cp, Cm, F;
  if (tbs == 0 || tbs % 8 || segment(B, &C, &Kp, &Km, &Cp, &Cm, &F) || F != 0 || Qm * Nl == 0) {
    return -1;
  }
  uint8_t* b = malloc(B);
  uint8_t* c = malloc(6144);
  uint8_t* d = malloc(3 * (6144 + 4));
  if (!b || !c || !d) {
    free(b), free(c), free(d);
    return -1;
  }
  for (uint32_t i = 0; i < tbs; i++) {
    b[i] = (uint8_t)((tb_bytes[i / 8] >> (7 - i % 8)) & 1u);
  }
  put24(b + tbs, synth_crc(CRC24A, b, tbs) ^ tb_crc_xor);
  const uint32_t Gp = G / (Nl * Qm), gamma = Gp % C;
  uint32_t       rp = 0, wp = 0;
  for (uint32_t r = 0; r < C; r++) {
    const uint32_t K    = r < Cm ? Km : Kp;
    const uint32_t nsrc = C > 1 ? K - 24 : K;
    memcpy(c, b + rp, nsrc);
    if (C > 1) {
      put24(c + nsrc, synth_crc(CRC24B, c, nsrc));
    }
    rp += nsrc;
    const uint32_t E = r <= C - gamma - 1 ? Nl * Qm * (Gp / C) : Nl * Qm * ((Gp + C - 1) / C);
    if (synth_turbo_encode(K, c, d, d + K + 4, d + 2 * (K + 4)) ||
        rate_match(K, rv, d, d + K + 4, d + 2 * (K + 4), E, e + wp)) {
      free(b), free(c), free(d);
      return -1;
    }
    wp += E;
  }
  free(b), free(c), free(d);
  return (int)wp;
}

/* 36.211 7.2: c(n), n = 0..len-1, for c_init */
void synth_gold(uint32_t c_init, uint32_t len, uint8_t* out)
{
  uint32_t x1 = 1, x2 = c_init & 0x7FFFFFFFu;
  for (uint32_t n = 0; n < 1600 + len; n++) {
    if (n >= 1600) {
      out[n - 1600] = (uint8_t)((x1 ^ x2) & 1u);
    }
    const uint32_t f1 = ((x1 >> 3) ^ x1) & 1u;
    const uint32_t f2 = ((x2 >> 3) ^ (x2 >> 2) ^ (x2 >> 1) ^ x2) & 1u;
    x1                = (x1 >> 1) | (f1 << 30);
    x2                = (x2 >> 1) | (f2 << 30);
  }
}
