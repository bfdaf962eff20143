// srsran_4g_amd/csrc/llr_kernel.hip -- PDSCH soft demapping + descrambling for CDNA4.
//
// Bit-exact with the reference's x86 build (SSE/AVX2) of
//   srsran_demod_soft_demodulate_s  modem/demod_soft.c:871-894 (per modulation, see below)
//   srsran_sequence_apply_s         common/sequence.c:507-561  (Gold sequence, 36.211 7.2)
// The reference demaps 4-symbol blocks with SSE (round half-even, int16 saturation) and the
// n % 4 tail with scalar C (truncation); QPSK goes through srsran_vec_convert_fi (16-value
// AVX2 blocks: truncation + saturation; tail: truncation + wrap).  Both splits are kept
// here by the symbol's index within the call.
//
// Layout: one workgroup per LLR_THREADS * SPT symbols.  The first wave's lanes jump the Gold LFSRs
// to the block start with three byte-indexed GF(2) jump tables (a uniform address: one fetch a wave),
// then each lane to its 64-symbol slice with one per-lane stride matrix, steps them 16 bits at a time
// and stages the bits in LDS; symbols are then processed with a stride of
// LLR_THREADS (coalesced).  HBM-bound elementwise work: 8 B (+4 B CSI) in, 2*Qm B out per symbol.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "devkey.h"
#include "eq_dev.h"
#include "gmem.h"
#include "llr_kernel.h"
#include "stage_timing.h"

namespace srsran_amd {

static constexpr int GOLD_NC   = 1600;  // sequence.c:39
static constexpr int JUMP_BITS = 24;    // offsets below 2^24 bits
static constexpr int JUMP_LVLS = 3;     // offset = b0 + 256 b1 + 65536 b2
static constexpr int GOLD_LANE_SYMBOLS = 4 * LLR_SPT_CFG;  // symbols whose sequence bits one lane of the first wave steps out
static constexpr int GOLD_NMOD         = 5;   // BPSK .. 256QAM: Qm = 1, 2, 4, 6, 8

struct GoldTables {
  uint32_t        x1_nc;      // x1 after Nc steps from x1 = 1
  uint32_t        x2_nc[31];  // x2 after Nc steps from the unit seed 1 << i
  const uint32_t* jump;       // [lvl][b][lfsr][32]: columns of A_lfsr^(b * 256^lvl) (device memory)
  const uint32_t* stride;     // [MOD][lane][lfsr][32]: columns of A_lfsr^(lane * GOLD_LANE_SYMBOLS * Qm) (device)
};
__constant__ GoldTables kGold;

__host__ __device__ inline uint32_t step_x1(uint32_t s) { return (s >> 1) ^ (((s ^ (s >> 3)) & 1u) << 30); }
__host__ __device__ inline uint32_t step_x2(uint32_t s)
{
  return (s >> 1) ^ (((s ^ (s >> 1) ^ (s >> 2) ^ (s >> 3)) & 1u) << 30);
}
__host__ __device__ inline uint32_t apply(const uint32_t* cols, uint32_t v)
{
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 31; i++) {
    r ^= ((v >> i) & 1u) ? cols[i] : 0u;
  }
  return r;
}

hipError_t gold_tables_init()
{
  // built once per device (kGold is the current device's copy of the constant)
  static std::mutex                mu;
  static std::map<int, hipError_t> done;
  std::lock_guard<std::mutex>      lk(mu);
  const int                        dev = cur_dev();
  if (done.count(dev)) {
    return done[dev];
  }
  hipError_t err = hipSuccess;
  // powers A^(2^k) of both LFSR transition matrices (as columns), k < JUMP_BITS
  std::vector<uint32_t> pw(2 * JUMP_BITS * 31);
  auto P = [&](int l, int k) { return &pw[(l * JUMP_BITS + k) * 31]; };
  for (int i = 0; i < 31; i++) {
    P(0, 0)[i] = step_x1(1u << i);
    P(1, 0)[i] = step_x2(1u << i);
  }
  for (int k = 1; k < JUMP_BITS; k++) {
    for (int l = 0; l < 2; l++) {
      for (int i = 0; i < 31; i++) {
        P(l, k)[i] = apply(P(l, k - 1), P(l, k - 1)[i]);
      }
    }
  }
  std::vector<uint32_t> jt((size_t)JUMP_LVLS * 256 * 2 * 32, 0u);
  for (int lvl = 0; lvl < JUMP_LVLS; lvl++) {
    for (int l = 0; l < 2; l++) {
      const uint32_t* M = P(l, 8 * lvl);  // A^(256^lvl)
      for (int b = 0; b < 256; b++) {
        uint32_t*       dst  = &jt[(((size_t)lvl * 256 + b) * 2 + l) * 32];
        const uint32_t* prev = b ? &jt[(((size_t)lvl * 256 + b - 1) * 2 + l) * 32] : nullptr;
        for (int i = 0; i < 31; i++) {
          dst[i] = b ? apply(M, prev[i]) : (1u << i);
        }
      }
    }
  }
  // lane strides: A^(lane * 64 Qm) for the 64 lanes of each modulation
  const size_t stride_off = jt.size();
  jt.resize(stride_off + (size_t)GOLD_NMOD * 64 * 2 * 32, 0u);
  const int qms[GOLD_NMOD] = {1, 2, 4, 6, 8};
  for (int m = 0; m < GOLD_NMOD; m++) {
    const uint32_t n = (uint32_t)(GOLD_LANE_SYMBOLS * qms[m]);
    for (int l = 0; l < 2; l++) {
      uint32_t S[31];  // A^n from the binary powers
      for (int i = 0; i < 31; i++) {
        S[i] = 1u << i;
      }
      for (int k = 0; k < JUMP_BITS; k++) {
        if ((n >> k) & 1u) {
          for (int i = 0; i < 31; i++) {
            S[i] = apply(P(l, k), S[i]);
          }
        }
      }
      for (int lane = 0; lane < 64; lane++) {
        uint32_t*       dst  = &jt[stride_off + (((size_t)m * 64 + lane) * 2 + l) * 32];
        const uint32_t* prev = lane ? dst - 2 * 32 : nullptr;
        for (int i = 0; i < 31; i++) {
          dst[i] = lane ? apply(S, prev[i]) : (1u << i);
        }
      }
    }
  }
  GoldTables t;
  uint32_t   s = 1;
  for (int n = 0; n < GOLD_NC; n++) {
    s = step_x1(s);
  }
  t.x1_nc = s;
  for (int i = 0; i < 31; i++) {
    uint32_t v = 1u << i;
    for (int n = 0; n < GOLD_NC; n++) {
      v = step_x2(v);
    }
    t.x2_nc[i] = v;
  }
  uint32_t* d_jump = nullptr;
  err = hipMalloc((void**)&d_jump, jt.size() * sizeof(uint32_t));
  if (err == hipSuccess) {
    err = hipMemcpy(d_jump, jt.data(), jt.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  }
  t.jump   = d_jump;
  t.stride = d_jump ? d_jump + stride_off : nullptr;
  if (err == hipSuccess) {
    err = hipMemcpyToSymbol(HIP_SYMBOL(kGold), &t, sizeof(t));
  }
  done[dev] = err;
  return err;
}

// columns (32 dwords, 16-byte aligned) applied to v
__device__ __forceinline__ uint32_t apply_cols(const uint32_t* __restrict__ cols, uint32_t v)
{
  const uint4* c4 = reinterpret_cast<const uint4*>(cols);
  uint32_t     r  = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const uint4 c = c4[q];
    r ^= ((v >> (4 * q)) & 1u) ? c.x : 0u;
    r ^= ((v >> (4 * q + 1)) & 1u) ? c.y : 0u;
    r ^= ((v >> (4 * q + 2)) & 1u) ? c.z : 0u;
    if (q < 7) {
      r ^= ((v >> (4 * q + 3)) & 1u) ? c.w : 0u;
    }
  }
  return r;
}

// LFSR states at bit offset `off` (< 2^24) of the sequence for `seed`: three table jumps.
__device__ __forceinline__ void gold_at(uint32_t seed, uint32_t off, uint32_t& x1, uint32_t& x2)
{
  x1 = kGold.x1_nc;
  x2 = apply(kGold.x2_nc, seed & 0x7FFFFFFFu);
#pragma unroll
  for (int lvl = 0; lvl < JUMP_LVLS; lvl++) {
    const uint32_t b = (off >> (8 * lvl)) & 255u;
    if (b) {
      const uint32_t* t = kGold.jump + (((size_t)lvl * 256 + b) * 2) * 32;
      x1                = apply_cols(t, x1);
      x2                = apply_cols(t + 32, x2);
    }
  }
}

// ---- x86 conversion semantics (see oracle/phy_oracle.c) ----
// out of range or NaN -> INT32_MIN ("integer indefinite"); one |x| compare (x = -2^31 converts to INT32_MIN either
// way, so the half-open range needs no second compare)
__device__ __forceinline__ int32_t cvt_rn(float x)
{
  return __builtin_fabsf(x) < 2147483648.0f ? (int32_t)__builtin_rintf(x) : INT32_MIN;
}
__device__ __forceinline__ int32_t cvt_tz(float x)
{
  return __builtin_fabsf(x) < 2147483648.0f ? (int32_t)x : INT32_MIN;
}
__device__ __forceinline__ int32_t cvt_tz_d(double x)
{
  return __builtin_fabs(x) < 2147483648.0 ? (int32_t)x : INT32_MIN;
}
__device__ __forceinline__ int16_t sat16(int32_t v) { return (int16_t)max(-32768, min(32767, v)); }
__device__ __forceinline__ int16_t wrap16(int32_t v) { return (int16_t)(uint16_t)(uint32_t)v; }
__device__ __forceinline__ int16_t abs16(int16_t v) { return wrap16(v < 0 ? -(int32_t)v : (int32_t)v); }

template <int MOD>
struct Qm;
template <>
struct Qm<0> {
  static constexpr int v = 1;
};
template <>
struct Qm<1> {
  static constexpr int v = 2;
};
template <>
struct Qm<2> {
  static constexpr int v = 4;
};
template <>
struct Qm<3> {
  static constexpr int v = 6;
};
template <>
struct Qm<4> {
  static constexpr int v = 8;
};

// LLRs of symbol i (of n in the call), reference semantics per modulation.
template <int MOD>
__device__ __forceinline__ void demap(float re, float im, uint32_t i, uint32_t n, int16_t* o)
{
  if constexpr (MOD == 0) {  // demod_bpsk_lte_s (demod_soft.c:96-101)
    const float t = -100.0f * (re + im);
    o[0]          = wrap16(cvt_tz_d((double)t * 0.70710678118654752440));
  } else if constexpr (MOD == 1) {  // srsran_vec_convert_fi (vector_simd.c:436-472), scale -100*sqrt(2)
    const float    scale = (float)(-100.0 * 1.41421356237309504880);
    const uint32_t nblk  = 16 * ((2 * n) / 16);
    const float    v[2]  = {re, im};
#pragma unroll
    for (int c = 0; c < 2; c++) {
      const int32_t t = cvt_tz(v[c] * scale);
      o[c]            = (2 * i + c < nblk) ? sat16(t) : wrap16(t);
    }
  } else if constexpr (MOD == 2) {  // demod_16qam_lte_s_sse (demod_soft.c:250-299)
    const float v[2] = {re, im};
    if (i < 4 * (n / 4)) {
#pragma unroll
      for (int c = 0; c < 2; c++) {
        const int16_t s = sat16(cvt_rn(v[c] * -400.0f));
        o[c]            = s;
        o[2 + c]        = wrap16(abs16(s) - 252);
      }
    } else {
      const float off = 800.0f / sqrtf(10.0f);
#pragma unroll
      for (int c = 0; c < 2; c++) {
        const int16_t y = wrap16(cvt_tz(400.0f * v[c]));
        o[c]            = wrap16(-(int32_t)y);
        o[2 + c]        = wrap16(cvt_tz((float)abs((int32_t)y) - off));
      }
    }
  } else if constexpr (MOD == 3) {  // demod_64qam_lte_s_sse (demod_soft.c:569-644)
    const float v[2] = {re, im};
    if (i < 4 * (n / 4)) {
#pragma unroll
      for (int c = 0; c < 2; c++) {
        const int16_t s = sat16(cvt_rn(v[c] * -700.0f));
        const int16_t a = wrap16(abs16(s) - 432);
        o[c]            = s;
        o[2 + c]        = a;
        o[4 + c]        = wrap16(abs16(a) - 216);
      }
    } else {
#pragma unroll
      for (int c = 0; c < 2; c++) {
        const int16_t y = wrap16(cvt_tz(700.0f * v[c]));
        const int16_t a = wrap16((int32_t)wrap16(abs((int32_t)y)) - 432);
        o[c]            = wrap16(-(int32_t)y);
        o[2 + c]        = a;
        o[4 + c]        = wrap16((int32_t)wrap16(abs((int32_t)a)) - 216);
      }
    }
  } else {  // demod_256qam_lte_s (demod_soft.c:824-844)
    const float t1 = 8.0f / sqrtf(170.0f), t2 = 4.0f / sqrtf(170.0f), t3 = 2.0f / sqrtf(170.0f);
    float       a = -re, b = -im;
    o[0] = wrap16(cvt_tz(1000.0f * a));
    o[1] = wrap16(cvt_tz(1000.0f * b));
    a    = fabsf(a) - t1;
    b    = fabsf(b) - t1;
    o[2] = wrap16(cvt_tz(1000.0f * a));
    o[3] = wrap16(cvt_tz(1000.0f * b));
    a    = fabsf(a) - t2;
    b    = fabsf(b) - t2;
    o[4] = wrap16(cvt_tz(1000.0f * a));
    o[5] = wrap16(cvt_tz(1000.0f * b));
    a    = fabsf(a) - t3;
    b    = fabsf(b) - t3;
    o[6] = wrap16(cvt_tz(1000.0f * a));
    o[7] = wrap16(cvt_tz(1000.0f * b));
  }
}

static constexpr int LLR_THREADS = 256;
static constexpr int SPT         = LLR_SPT_CFG;  // symbols per thread
static_assert(LLR_THREADS * SPT == LLR_BLOCK_SYMBOLS, "llr_kernel.h block size");

__device__ __forceinline__ float2 modulate(int mod, uint32_t i);

// csi_correction (pdsch.c:523-618, SSE build) for the LLRs o[0..Q) of symbol s:
// symbols inside the SSE blocks get mulhi(e, cvtps_pi16(csi * 32767/csi_max)) -- with the
// reference's _mm_blend_ps(.., 3) swap: in a QPSK/64QAM symbol pair the middle lanes take
// the other symbol's CSI -- and the tail truncates (float)e * (csi / csi_max).
__device__ __forceinline__ int16_t cvt_pi16(float x) { return sat16(cvt_rn(x)); }
__device__ __forceinline__ int16_t mulhi16(int16_t a, int16_t b) { return (int16_t)(((int32_t)a * (int32_t)b) >> 16); }

template <int MOD>
// cs = csi[s], cso = csi[s ^ 1] (loaded by the caller; cso only read where s ^ 1 < n)
__device__ __forceinline__ void csi_correct(int16_t* o, uint32_t s, float cs, float cso, float mx, uint32_t nof_bits)
{
  constexpr int Q     = Qm<MOD>::v;
  const float   scale = 32767.0f / mx;
  uint32_t      nblk;  // symbols covered by the SSE blocks
  if constexpr (MOD == 1) {
    nblk = 2 * (nof_bits / 4);
  } else if constexpr (MOD == 2) {
    nblk = nof_bits / 4;
  } else if constexpr (MOD == 3) {
    nblk = 2 * (nof_bits / 12);
  } else if constexpr (MOD == 4) {
    nblk = nof_bits / 8;
  } else {
    nblk = 0;
  }
  if (s < nblk) {
    const int16_t c = cvt_pi16(cs * scale);
    if constexpr (MOD == 1) {  // pair (s, s^1): lanes 0,1 take the odd symbol's CSI, lanes 2,3 the even's
      const int16_t co = cvt_pi16(cso * scale);
#pragma unroll
      for (int b = 0; b < Q; b++) {
        o[b] = mulhi16(o[b], co);
      }
    } else if constexpr (MOD == 3) {  // even s: LLR 4,5 use s+1; odd s: LLR 0,1 use s-1
      const int16_t co = cvt_pi16(cso * scale);
#pragma unroll
      for (int b = 0; b < Q; b++) {
        const bool other = (s & 1u) ? (b < 2) : (b >= 4);
        o[b]             = mulhi16(o[b], other ? co : c);
      }
    } else {
#pragma unroll
      for (int b = 0; b < Q; b++) {
        o[b] = mulhi16(o[b], c);
      }
    }
  } else {  // the release build hoists 1 / csi_max (-Ofast -freciprocal-math; oracle/ref_pdsch_tx_harness.c)
    const float c = cs * (1.0f / mx);
#pragma unroll
    for (int b = 0; b < Q; b++) {
      o[b] = wrap16(cvt_tz((float)o[b] * c));
    }
  }
}

// ---- the 8-bit chain (q->llr_is_8bit, pdsch.c:691-737) ----
__device__ __forceinline__ int8_t sat8(int32_t v) { return (int8_t)max(-128, min(127, v)); }
__device__ __forceinline__ int8_t wrap8(int32_t v) { return (int8_t)(uint8_t)(uint32_t)v; }
__device__ __forceinline__ int8_t abs8(int8_t v) { return wrap8(v < 0 ? -(int32_t)v : (int32_t)v); }  // _mm_abs_epi8

// srsran_demod_soft_demodulate_b (demod_soft.c:896-919), x86 SSE build: SSE blocks of 8 symbols (QPSK: 16 values of
// srsran_vec_convert_fb_simd) round (QAM) or truncate (QPSK) and saturate to int8, their abs / offset steps wrap; the
// tails truncate and wrap (oracle_demod_soft_b)
template <int MOD>
__device__ __forceinline__ void demap8(float re, float im, uint32_t i, uint32_t n, int8_t* o)
{
  const float v[2] = {re, im};
  if constexpr (MOD == 0) {  // demod_bpsk_lte_b
    const float t = -20.0f * (re + im);
    o[0]          = wrap8(cvt_tz_d((double)t * 0.70710678118654752440));
  } else if constexpr (MOD == 1) {  // vector_simd.c:524-589, scale (float)(-20 * M_SQRT2)
    const float    scale = (float)(-20.0 * 1.41421356237309504880);
    const uint32_t nblk  = 16 * ((2 * n) / 16);
#pragma unroll
    for (int c = 0; c < 2; c++) {
      const int32_t t = cvt_tz(v[c] * scale);
      o[c]            = (2 * i + c < nblk) ? sat8(t) : wrap8(t);
    }
  } else if constexpr (MOD == 2) {  // demod_16qam_lte_b_sse (demod_soft.c:301-364)
    if (i < 8 * (n / 8)) {
#pragma unroll
      for (int c = 0; c < 2; c++) {
        const int8_t s = sat8(cvt_rn(v[c] * -30.0f));
        o[c]           = s;
        o[2 + c]       = wrap8(abs8(s) - 18);  // _mm_set1_epi8(60 / sqrtf(10))
      }
    } else {
      const float off = 60.0f / sqrtf(10.0f);
#pragma unroll
      for (int c = 0; c < 2; c++) {
        const int8_t y = wrap8(cvt_tz(30.0f * v[c]));
        o[c]           = wrap8(-(int32_t)y);
        o[2 + c]       = wrap8(cvt_tz((float)abs((int32_t)y) - off));
      }
    }
  } else if constexpr (MOD == 3) {  // demod_64qam_lte_b_sse (demod_soft.c:650-730)
    if (i < 8 * (n / 8)) {
#pragma unroll
      for (int c = 0; c < 2; c++) {
        const int8_t s = sat8(cvt_rn(v[c] * -40.0f));
        const int8_t a = wrap8(abs8(s) - 24);
        o[c]           = s;
        o[2 + c]       = a;
        o[4 + c]       = wrap8(abs8(a) - 12);
      }
    } else {
#pragma unroll
      for (int c = 0; c < 2; c++) {
        const int8_t y = wrap8(cvt_tz(40.0f * v[c]));
        const int8_t a = wrap8((int32_t)wrap8(abs((int32_t)y)) - 24);
        o[c]           = wrap8(-(int32_t)y);
        o[2 + c]       = a;
        o[4 + c]       = wrap8((int32_t)wrap8(abs((int32_t)a)) - 12);
      }
    }
  } else {  // demod_256qam_lte_b (demod_soft.c:800-822)
    const float t[3] = {8.0f / sqrtf(170.0f), 4.0f / sqrtf(170.0f), 2.0f / sqrtf(170.0f)};
    float       a = -re, b = -im;
#pragma unroll
    for (int l = 0; l < 4; l++) {
      if (l) {
        a = fabsf(a) - t[l - 1];
        b = fabsf(b) - t[l - 1];
      }
      o[2 * l]     = wrap8(cvt_tz(50.0f * a));
      o[2 * l + 1] = wrap8(cvt_tz(50.0f * b));
    }
  }
}

// csi_correction's llr_is_8bit branch (pdsch.c:538-545): (int8)((float)e * (csi * (1 / csi_max)))
template <int MOD>
__device__ __forceinline__ void csi_correct8(int8_t* o, float cs, float mx)
{
  const float c = cs * (1.0f / mx);
#pragma unroll
  for (int b = 0; b < Qm<MOD>::v; b++) {
    o[b] = wrap8(cvt_tz((float)o[b] * c));
  }
}

// advance both LFSRs by 16 bits and return c(n..n+15) (bit k = c(n+k)): the recurrences
// x1(m+31) = x1(m+3) ^ x1(m) and x2(m+31) = x2(m+3) ^ x2(m+2) ^ x2(m+1) ^ x2(m) give 28 new bits
// per shift-xor, 16 of which are used
__device__ __forceinline__ uint32_t gold16(uint32_t& x1, uint32_t& x2)
{
  const uint32_t c  = (x1 ^ x2) & 0xFFFFu;
  const uint32_t n1 = ((x1 >> 3) ^ x1) & 0xFFFFu;
  const uint32_t n2 = ((x2 >> 3) ^ (x2 >> 2) ^ (x2 >> 1) ^ x2) & 0xFFFFu;
  x1                = (x1 >> 16) | (n1 << 15);
  x2                = (x2 >> 16) | (n2 << 15);
  return c;
}

// The fused path's symbols: the NL layers of REs base + t + (r0 + u) LLR_THREADS, u < U, equalised from the received
// grid and the channel estimates with the predecoder's arithmetic (eq_dev.h: the same floats as eq_kernel.hip's
// predecode_items, which the GPU tests check bit for bit).  Lanes past nb compute RE `base` (in range, discarded).
template <int FS, int NL, int U>
__device__ __forceinline__ void fused_group(const PredArgs& a, float noise, uint32_t base, uint32_t t, int r0,
                                            uint32_t nb, float2 (&vv)[NL][U], float (&cs)[NL][U])
{
  static_assert((FS == 0 && NL == 1) || ((FS == 2 || FS == 3) && NL == 2), "PORT0 one layer, SM / CDD two");
  uint32_t kk[U], gy[U], gh[U];
  float    ys[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint32_t i = t + (uint32_t)(r0 + u) * LLR_THREADS;
    kk[u]            = base + (i < nb ? i : 0u);
    gy[u]            = kk[u];
    gh[u]            = kk[u];
    ys[u]            = 1.0f;
  }
  if (a.idx) {
    uint32_t e[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      e[u] = gptr(a.idx)[kk[u]];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      eqd::re_pos(a, e[u], gy[u], gh[u], ys[u]);
    }
  }
  auto Ys = [&](eqd::cpx v, int u) -> eqd::cpx { return ys[u] != 1.0f ? eqd::cscale(v, ys[u]) : v; };
  if constexpr (FS == 0) {
    eqd::cpx yv[U][4], hv[U][4];
#pragma unroll
    for (int u = 0; u < U; u++) {
#pragma unroll
      for (int p = 0; p < 4; p++) {
        if (p < a.nrx) {
          yv[u][p] = eqd::ld(a.y[p], gy[u]);
          hv[u][p] = eqd::ld(a.h[0][p], gh[u]);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      eqd::cpx y[4];
#pragma unroll
      for (int p = 0; p < 4; p++) {
        y[p] = Ys(yv[u][p], u);
      }
      eqd::cpx x;
      eqd::port0(y, hv[u], a.nrx, noise, a.norm, x, cs[0][u]);
      vv[0][u] = make_float2(x.r, x.i);
    }
  } else {
    eqd::cpx y0[U], y1[U], p0[U], p1[U], q0[U], q1[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      p0[u] = eqd::ld(a.h[0][0], gh[u]);
      p1[u] = eqd::ld(a.h[0][1], gh[u]);
      q0[u] = eqd::ld(a.h[1][0], gh[u]);
      q1[u] = eqd::ld(a.h[1][1], gh[u]);
      y0[u] = eqd::ld(a.y[0], gy[u]);
      y1[u] = eqd::ld(a.y[1], gy[u]);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      eqd::cpx h00, h01, h10, h11;
      eqd::effective_h<FS>(a.codebook, kk[u], p0[u], p1[u], q0[u], q1[u], h00, h01, h10, h11);
      eqd::cpx x0, x1;
      eqd::mmse_csi(Ys(y0[u], u), Ys(y1[u], u), h00, h01, h10, h11, x0, x1, cs[0][u], cs[NL - 1][u], noise, a.norm);
      vv[0][u]      = make_float2(x0.r, x0.i);
      vv[NL - 1][u] = make_float2(x1.r, x1.i);
    }
  }
}

// Phase 1 of a block: the first wave's lanes jump the Gold LFSRs of `seed` to the block's first bit (bit0 + base Q)
// and then to their 64-symbol slices and write the block's sequence bits to cbits (the caller synchronises)
template <int MOD>
__device__ __forceinline__ void gold_stage(uint32_t seed, uint32_t bit0, uint32_t base, uint32_t nb, uint16_t* cbits)
{
  constexpr int  Q = Qm<MOD>::v;
  const uint32_t t = threadIdx.x;
  static_assert(64 * GOLD_LANE_SYMBOLS == LLR_THREADS * SPT, "the first wave covers the block");
  if (t < 64 && t * GOLD_LANE_SYMBOLS < nb) {
    uint32_t x1, x2;
    gold_at(seed, bit0 + base * Q, x1, x2);  // the block start (uniform over the wave)
    if (t) {
      const uint32_t* m = kGold.stride + ((size_t)MOD * 64 + t) * 2 * 32;
      x1                = apply_cols(m, x1);
      x2                = apply_cols(m + 32, x2);
    }
#pragma unroll 4
    for (int j = 0; j < GOLD_LANE_SYMBOLS * Q / 16; j++) {
      cbits[t * (GOLD_LANE_SYMBOLS * Q / 16) + j] = (uint16_t)gold16(x1, x2);
    }
  }
}

// Phase 2 of one symbol, int16 LLRs: demap symbol s (index i of the block), the EVM error (s < evm_n), descramble
// from the block's sequence bits, CSI correction (cso: the CSI of symbol s ^ 1), store
template <int MOD>
__device__ __forceinline__ void llr16_symbol(float2 v, uint32_t s, uint32_t i, uint32_t n, int scramble,
                                             const uint16_t* cbits, bool csi, float cs, float cso, float mx,
                                             gptr_t<int16_t> llr, bool a4, bool a16, uint32_t evm_n, float& err)
{
  constexpr int Q = Qm<MOD>::v;
  int16_t o[Q];
  demap<MOD>(v.x, v.y, s, n, o);
  if constexpr (MOD >= 1) {
    if (s < evm_n) {  // hard decision (bit = !sign, evm.h HARD_DECISION), remodulated, error power
      uint32_t idx = 0;
#pragma unroll
      for (int k = 0; k < Q; k++) {
        idx = (idx << 1) | (o[k] >= 0 ? 1u : 0u);
      }
      const float2 m  = modulate(MOD, idx);
      const float  dr = v.x - m.x, di = v.y - m.y;
      err += dr * dr + di * di;
    }
  }
  if (scramble) {
    const uint32_t b  = i * Q;
    const uint32_t w0 = cbits[b >> 4];
    const uint32_t w  = ((b & 15) + Q > 16) ? (w0 | ((uint32_t)cbits[(b >> 4) + 1] << 16)) : w0;
    const uint32_t cb = w >> (b & 15);
#pragma unroll
    for (int k = 0; k < Q; k++) {
      o[k] = ((cb >> k) & 1u) ? wrap16(-(int32_t)o[k]) : o[k];
    }
  }
  if (csi) {  // after descrambling, as pdsch.c:735-737 orders it
    csi_correct<MOD>(o, s, cs, cso, mx, n * Q);
  }
  const gptr_t<int16_t> dst = llr + (size_t)s * Q;
  if (Q == 1 || !a4) {
#pragma unroll
    for (int k = 0; k < Q; k++) {
      dst[k] = o[k];
    }
  } else if constexpr (Q == 2) {
    *reinterpret_cast<gptr_t<uint32_t>>(dst) = (uint32_t)(uint16_t)o[0] | ((uint32_t)(uint16_t)o[1] << 16);
  } else if constexpr (Q == 8) {
    uint4 u;
    u.x = (uint32_t)(uint16_t)o[0] | ((uint32_t)(uint16_t)o[1] << 16);
    u.y = (uint32_t)(uint16_t)o[2] | ((uint32_t)(uint16_t)o[3] << 16);
    u.z = (uint32_t)(uint16_t)o[4] | ((uint32_t)(uint16_t)o[5] << 16);
    u.w = (uint32_t)(uint16_t)o[6] | ((uint32_t)(uint16_t)o[7] << 16);
    if (a16) {
      *reinterpret_cast<gptr_t<uint4>>(dst) = u;
    } else {
      const gptr_t<uint32_t> d = reinterpret_cast<gptr_t<uint32_t>>(dst);
      d[0] = u.x, d[1] = u.y, d[2] = u.z, d[3] = u.w;
    }
  } else {  // Q = 4, 6: 4-byte aligned words (int16 buffers are 4-byte aligned)
    const gptr_t<uint32_t> d = reinterpret_cast<gptr_t<uint32_t>>(dst);
#pragma unroll
    for (int k = 0; k < Q / 2; k++) {
      d[k] = (uint32_t)(uint16_t)o[2 * k] | ((uint32_t)(uint16_t)o[2 * k + 1] << 16);
    }
  }
}

// One block = LLR_THREADS * SPT consecutive symbols.  Phase 1 (gold_stage): thread t < 64 jumps the Gold LFSRs to
// the block's bit t * GOLD_LANE_SYMBOLS * Q and writes its sequence bits to LDS.  Phase 2: thread t handles symbols
// t, t + 256, ... -- coalesced loads and stores -- demapping, descrambling from the LDS bits and CSI correction in
// registers.
template <int MOD, bool B8 = false>
__device__ __forceinline__ void llr_block(const float2* __restrict__ sym_p, uint32_t n, int scramble, uint32_t seed,
                                          uint32_t bit0, const float* __restrict__ csi_p,
                                          const float* __restrict__ csi_max, int16_t* __restrict__ llr_p, uint32_t blk,
                                          float* __restrict__ evm_part = nullptr, uint32_t evm_n = 0,
                                          int8_t* __restrict__ llr8_p = nullptr)
{
  const gptr_t<const float2> sym  = gptr(sym_p);  // global-space views (gmem.h)
  const gptr_t<const float>  csi  = gptr(csi_p);
  const gptr_t<int16_t>      llr  = gptr(llr_p);
  const gptr_t<int8_t>       llr8 = gptr(llr8_p);
  constexpr int       Q = Qm<MOD>::v;
  __shared__ uint16_t cbits[LLR_THREADS * 8 + 2];  // SPT * Q / 16 = Q chunks per thread
  const uint32_t      base = blk * (uint32_t)(LLR_THREADS * SPT);
  if (base >= n) {
    return;  // uniform per block
  }
  const uint32_t nb = min((uint32_t)(LLR_THREADS * SPT), n - base);
  const uint32_t t  = threadIdx.x;
  if (scramble) {
    gold_stage<MOD>(seed, bit0, base, nb, cbits);
    __syncthreads();
  }
  const float mx  = csi ? *gptr(csi_max) : 1.0f;
  const uintptr_t ob  = B8 ? (uintptr_t)llr8 : (uintptr_t)llr;
  const bool      a16 = (ob & 15) == 0;
  const bool      a8  = (ob & 7) == 0;
  const bool      a4  = (ob & 3) == 0;
  const bool      a2  = (ob & 1) == 0;
  float       err = 0.0f;  // EVM: this thread's sum of squared symbol errors
  // the thread's symbols (and CSI) in groups of LLR_U, each group's loads issued before the first is used: one
  // HBM round trip a group instead of one a symbol
  constexpr int LLR_U = SPT < 8 ? SPT : 8;
  static_assert(SPT % LLR_U == 0, "whole groups");
  for (int r0 = 0; r0 < SPT; r0 += LLR_U) {
    if (t + (uint32_t)r0 * LLR_THREADS >= nb) {
      break;
    }
    float2 vv[LLR_U];
    float  cs[LLR_U], cso[LLR_U];
#pragma unroll
    for (int u = 0; u < LLR_U; u++) {
      const uint32_t i = t + (uint32_t)(r0 + u) * LLR_THREADS;
      if (i < nb) {
        vv[u] = sym[base + i];
        if (csi) {
          cs[u] = csi[base + i];
          if (!B8 && (MOD == 1 || MOD == 3) && ((base + i) ^ 1u) < n) {
            cso[u] = csi[(base + i) ^ 1u];
          }
        }
      }
    }
#pragma unroll
  for (int u = 0; u < LLR_U; u++) {
    const uint32_t i = t + (uint32_t)(r0 + u) * LLR_THREADS;
    if (i >= nb) {
      break;
    }
    const uint32_t s = base + i;
    const float2   v = vv[u];
    if constexpr (B8) {  // int8 LLRs: demod_b, sequence_apply_c, the 8-bit CSI correction
      int8_t o[Q];
      demap8<MOD>(v.x, v.y, s, n, o);
      if constexpr (MOD >= 1) {
        if (s < evm_n) {  // srsran_evm_run_b: the same hard decision on the int8 LLRs
          uint32_t idx = 0;
#pragma unroll
          for (int k = 0; k < Q; k++) {
            idx = (idx << 1) | (o[k] >= 0 ? 1u : 0u);
          }
          const float2 m  = modulate(MOD, idx);
          const float  dr = v.x - m.x, di = v.y - m.y;
          err += dr * dr + di * di;
        }
      }
      if (scramble) {
        const uint32_t b  = i * Q;
        const uint32_t w0 = cbits[b >> 4];
        const uint32_t w  = ((b & 15) + Q > 16) ? (w0 | ((uint32_t)cbits[(b >> 4) + 1] << 16)) : w0;
        const uint32_t cb = w >> (b & 15);
#pragma unroll
        for (int k = 0; k < Q; k++) {
          o[k] = ((cb >> k) & 1u) ? wrap8(-(int32_t)o[k]) : o[k];
        }
      }
      if (csi) {
        csi_correct8<MOD>(o, cs[u], mx);
      }
      const gptr_t<int8_t> dst = llr8 + (size_t)s * Q;
      if constexpr (Q == 8) {
        uint2 u;
        u.x = (uint32_t)(uint8_t)o[0] | ((uint32_t)(uint8_t)o[1] << 8) | ((uint32_t)(uint8_t)o[2] << 16) |
              ((uint32_t)(uint8_t)o[3] << 24);
        u.y = (uint32_t)(uint8_t)o[4] | ((uint32_t)(uint8_t)o[5] << 8) | ((uint32_t)(uint8_t)o[6] << 16) |
              ((uint32_t)(uint8_t)o[7] << 24);
        if (a8) {
          *reinterpret_cast<gptr_t<uint2>>(dst) = u;
          continue;
        }
      } else if constexpr (Q == 4) {
        if (a4) {
          *reinterpret_cast<gptr_t<uint32_t>>(dst) = (uint32_t)(uint8_t)o[0] | ((uint32_t)(uint8_t)o[1] << 8) |
                                              ((uint32_t)(uint8_t)o[2] << 16) | ((uint32_t)(uint8_t)o[3] << 24);
          continue;
        }
      } else if constexpr (Q == 2 || Q == 6) {
        if (a2) {  // Q = 6: the symbol's 6 bytes start 2-byte aligned
#pragma unroll
          for (int k = 0; k < Q / 2; k++) {
            reinterpret_cast<gptr_t<uint16_t>>(dst)[k] = (uint16_t)((uint8_t)o[2 * k] | ((uint32_t)(uint8_t)o[2 * k + 1] << 8));
          }
          continue;
        }
      }
#pragma unroll
      for (int k = 0; k < Q; k++) {
        dst[k] = o[k];
      }
      continue;
    }
    llr16_symbol<MOD>(v, s, i, n, scramble, cbits, csi, cs[u], cso[u], mx, llr, a4, a16, evm_n, err);
  }
  }
  if (evm_part && base < evm_n) {  // block sum in a fixed order: wave butterflies, then the 4 waves
    __shared__ float wsum[LLR_THREADS / 64];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      err += __shfl_xor(err, off, 64);
    }
    if ((t & 63) == 0) {
      wsum[t >> 6] = err;
    }
    __syncthreads();
    if (t == 0) {
      gptr(evm_part)[blk] = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
    }
  }
}

template <int MOD>
__global__ __launch_bounds__(LLR_THREADS) void llr_kernel(const float2* __restrict__ sym, uint32_t n, int scramble,
                                                          uint32_t seed, uint32_t bit0, const float* __restrict__ csi,
                                                          const float* __restrict__ csi_max, int16_t* __restrict__ llr)
{
  llr_block<MOD>(sym, n, scramble, seed, bit0, csi, csi_max, llr, blockIdx.x);
}

template <int MOD, bool B8>
__global__ __launch_bounds__(LLR_THREADS) void llr_batch_kernel(const LlrItem* __restrict__ items)
{
  const LlrItem& it = items[blockIdx.y];
  llr_block<MOD, B8>(reinterpret_cast<const float2*>(it.sym), it.n, it.scramble, it.seed, it.bit0, it.csi, it.csi_max,
                     it.llr, blockIdx.x, it.evm_part, it.evm_n, it.llr8);
}

// One block = LLR_THREADS * SPT REs of one subframe: each RE equalised once (fused_group), then the symbol of every
// layer demapped, descrambled with that codeword's sequence and CSI-corrected into that codeword's LLRs
template <int MOD, int FS, int U, int FSPT>
__global__ __launch_bounds__(LLR_THREADS) void fused_llr_batch_kernel(const FusedItem* __restrict__ items)
{
  constexpr int       NL = FS == 0 ? 1 : 2;  // U: REs a group, each carrying up to 8 complex loads
  static_assert(FSPT % U == 0 && FSPT <= SPT, "whole groups, blocks within gold_stage's reach");
  __shared__ uint16_t cbits[NL][LLR_THREADS * 8 + 2];
  const FusedItem&    f    = items[blockIdx.y];
  const uint32_t      n    = f.n;
  const uint32_t      base = blockIdx.x * (uint32_t)(LLR_THREADS * FSPT);
  if (base >= n) {
    return;  // uniform per block
  }
  const uint32_t nb = min((uint32_t)(LLR_THREADS * FSPT), n - base);
  const uint32_t t  = threadIdx.x;
#pragma unroll
  for (int l = 0; l < NL; l++) {
    gold_stage<MOD>(f.seed[l], 0, base, nb, cbits[l]);
  }
  __syncthreads();
  const PredArgs& a   = *f.pa;
  const bool      csi = f.csi_max != nullptr;
  const float     noise = a.noise_ptr ? *gptr(a.noise_ptr) : a.noise;
  float           mx[NL];
  bool            a4[NL], a16[NL];
#pragma unroll
  for (int l = 0; l < NL; l++) {
    mx[l]  = csi ? gptr(f.csi_max)[l] : 1.0f;
    a4[l]  = ((uintptr_t)f.llr[l] & 3) == 0;
    a16[l] = ((uintptr_t)f.llr[l] & 15) == 0;
  }
  float err = 0.0f;  // (no EVM on this path)
  for (int r0 = 0; r0 < FSPT; r0 += U) {
    if (t + (uint32_t)r0 * LLR_THREADS >= nb) {
      break;
    }
    float2 vv[NL][U];
    float  cs[NL][U], cso[NL][U];
    fused_group<FS, NL, U>(a, noise, base, t, r0, nb, vv, cs);
    if (MOD == 1 || MOD == 3) {
      // the CSI of RE s ^ 1 sits in lane t ^ 1 of the same group; that lane has left the loop only when s ^ 1 >= n,
      // where csi_correct does not read it
#pragma unroll
      for (int l = 0; l < NL; l++) {
#pragma unroll
        for (int u = 0; u < U; u++) {
          cso[l][u] = __shfl_xor(cs[l][u], 1, 64);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t i = t + (uint32_t)(r0 + u) * LLR_THREADS;
      if (i >= nb) {
        break;
      }
#pragma unroll
      for (int l = 0; l < NL; l++) {
        llr16_symbol<MOD>(vv[l][u], base + i, i, n, 1, cbits[l], csi, cs[l][u], cso[l][u], mx[l], gptr(f.llr[l]),
                          a4[l], a16[l], 0, err);
      }
    }
  }
}

__global__ void evm_finalize_kernel(const EvmItem* __restrict__ items, uint32_t nitems)
{
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nitems) {
    return;
  }
  const EvmItem& e = items[k];
  float          s = 0.0f;
  for (uint32_t j = 0; j < e.nparts; j++) {
    s += e.part[j];
  }
  *e.out = e.nsym ? sqrtf(s / (float)e.nsym) : NAN;  // srsran_vec_avg_power_cf + sqrtf
}

hipError_t evm_finalize_launch(const EvmItem* d_items, uint32_t nitems, hipStream_t stream)
{
  if (nitems == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(evm_finalize_kernel, dim3((nitems + 63) / 64), dim3(64), 0, stream, d_items, nitems);
  return hipGetLastError();
}

hipError_t llr_batch_launch(int mod, const LlrItem* d_items, uint32_t nitems, uint32_t max_n, int any_scramble,
                            hipStream_t stream, bool llr8)
{
  StageScope timing_scope(ST_LLR, stream);
  if (nitems == 0 || max_n == 0) {
    return hipSuccess;
  }
  if (any_scramble && (uint64_t)max_n * 8 > (1ull << JUMP_BITS)) {
    return hipErrorInvalidValue;
  }
  if (any_scramble) {
    hipError_t e = gold_tables_init();
    if (e != hipSuccess) {
      return e;
    }
  }
  const dim3 grid((max_n + LLR_THREADS * SPT - 1) / (LLR_THREADS * SPT), nitems);
#define LLR_CASE(M)                                                                                 \
  case M:                                                                                           \
    if (llr8) {                                                                                     \
      hipLaunchKernelGGL((llr_batch_kernel<M, true>), grid, dim3(LLR_THREADS), 0, stream, d_items);  \
    } else {                                                                                        \
      hipLaunchKernelGGL((llr_batch_kernel<M, false>), grid, dim3(LLR_THREADS), 0, stream, d_items); \
    }                                                                                               \
    break;
  switch (mod) {
    LLR_CASE(0)
    LLR_CASE(1)
    LLR_CASE(2)
    LLR_CASE(3)
    LLR_CASE(4)
    default:
      return hipErrorInvalidValue;
  }
#undef LLR_CASE
  return hipGetLastError();
}

hipError_t fused_llr_batch_launch(int mod, int scheme, const FusedItem* d_items, uint32_t nitems, uint32_t max_n,
                                  hipStream_t stream)
{
  StageScope timing_scope(ST_LLR, stream);
  if (nitems == 0 || max_n == 0) {
    return hipSuccess;
  }
  if ((uint64_t)max_n * 8 > (1ull << JUMP_BITS)) {
    return hipErrorInvalidValue;
  }
  hipError_t e = gold_tables_init();
  if (e != hipSuccess) {
    return e;
  }
  // 4 REs a thread in 2 load groups: 2 x the blocks of llr_batch_launch's 2048-symbol ones, at 83 VGPRs (5 waves a
  // SIMD); r05m A/B of 2x2 / 4x2 / 4x4 / 8x2: 4x2 the fastest, by < 10 %
  constexpr int FSPT = 4;
  const dim3    grid((max_n + LLR_THREADS * FSPT - 1) / (LLR_THREADS * FSPT), nitems);
#define FUSED_CASE(M, S)                                                                                        \
  case M * 8 + S:                                                                                               \
    hipLaunchKernelGGL((fused_llr_batch_kernel<M, S, 2, FSPT>), grid, dim3(LLR_THREADS), 0, stream, d_items); \
    break;
#define FUSED_MOD(M) FUSED_CASE(M, 0) FUSED_CASE(M, 2) FUSED_CASE(M, 3)
  switch (mod * 8 + scheme) {
    FUSED_MOD(0)
    FUSED_MOD(1)
    FUSED_MOD(2)
    FUSED_MOD(3)
    FUSED_MOD(4)
    default:
      return hipErrorInvalidValue;
  }
#undef FUSED_MOD
#undef FUSED_CASE
  return hipGetLastError();
}

hipError_t llr_launch(int mod, const float* d_sym, uint32_t nsym, int scramble, uint32_t seed, uint32_t bit0,
                      const float* d_csi, const float* d_csi_max, int16_t* d_llr, hipStream_t stream)
{
  StageScope timing_scope(ST_LLR, stream);
  if (nsym == 0) {
    return hipSuccess;
  }
  if (scramble && (uint64_t)bit0 + (uint64_t)nsym * 8 > (1ull << JUMP_BITS)) {
    return hipErrorInvalidValue;  // jump tables cover offsets below 2^24
  }
  if (scramble) {
    hipError_t e = gold_tables_init();
    if (e != hipSuccess) {
      return e;
    }
  }
  const dim3    grid((nsym + LLR_THREADS * SPT - 1) / (LLR_THREADS * SPT));
  const float2* s = reinterpret_cast<const float2*>(d_sym);
  switch (mod) {
    case 0:
      hipLaunchKernelGGL(llr_kernel<0>, grid, dim3(LLR_THREADS), 0, stream, s, nsym, scramble, seed, bit0, d_csi,
                         d_csi_max, d_llr);
      break;
    case 1:
      hipLaunchKernelGGL(llr_kernel<1>, grid, dim3(LLR_THREADS), 0, stream, s, nsym, scramble, seed, bit0, d_csi,
                         d_csi_max, d_llr);
      break;
    case 2:
      hipLaunchKernelGGL(llr_kernel<2>, grid, dim3(LLR_THREADS), 0, stream, s, nsym, scramble, seed, bit0, d_csi,
                         d_csi_max, d_llr);
      break;
    case 3:
      hipLaunchKernelGGL(llr_kernel<3>, grid, dim3(LLR_THREADS), 0, stream, s, nsym, scramble, seed, bit0, d_csi,
                         d_csi_max, d_llr);
      break;
    case 4:
      hipLaunchKernelGGL(llr_kernel<4>, grid, dim3(LLR_THREADS), 0, stream, s, nsym, scramble, seed, bit0, d_csi,
                         d_csi_max, d_llr);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

static constexpr int SEQ_PER_THREAD = 64;

__global__ __launch_bounds__(LLR_THREADS) void seq_apply_kernel(const int16_t* __restrict__ in,
                                                                int16_t* __restrict__ out, uint32_t len,
                                                                uint32_t seed)
{
  const uint32_t i0 = (blockIdx.x * LLR_THREADS + threadIdx.x) * SEQ_PER_THREAD;
  if (i0 >= len) {
    return;
  }
  uint32_t x1, x2;
  gold_at(seed, i0, x1, x2);
  const uint32_t n = min((uint32_t)SEQ_PER_THREAD, len - i0);
#pragma unroll
  for (int c = 0; c < SEQ_PER_THREAD / 16; c++) {
    const uint32_t bits = gold16(x1, x2);
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t i = (uint32_t)(16 * c + k);
      if (i < n) {
        const int16_t v = in[i0 + i];
        out[i0 + i]     = ((bits >> k) & 1u) ? wrap16(-(int32_t)v) : v;
      }
    }
  }
}

hipError_t seq_apply_launch(const int16_t* d_in, int16_t* d_out, uint32_t len, uint32_t seed, hipStream_t stream)
{
  StageScope timing_scope(ST_LLR, stream);
  if (len == 0) {
    return hipSuccess;
  }
  if (len > (1u << JUMP_BITS)) {
    return hipErrorInvalidValue;
  }
  hipError_t e = gold_tables_init();
  if (e != hipSuccess) {
    return e;
  }
  const dim3 grid((len + LLR_THREADS * SEQ_PER_THREAD - 1) / (LLR_THREADS * SEQ_PER_THREAD));
  hipLaunchKernelGGL(seq_apply_kernel, grid, dim3(LLR_THREADS), 0, stream, d_in, d_out, len, seed);
  return hipGetLastError();
}

// c(i) as one byte per bit (srsran_sequence_pusch_gen_unpack, sequences.c:95-102): the UCI
// decoder's scrambling sequence, 16 bits written as 4 dwords
__global__ __launch_bounds__(LLR_THREADS) void seq_unpack_kernel(uint8_t* __restrict__ out, uint32_t len,
                                                                 uint32_t seed)
{
  const uint32_t i0 = (blockIdx.x * LLR_THREADS + threadIdx.x) * SEQ_PER_THREAD;
  if (i0 >= len) {
    return;
  }
  uint32_t x1, x2;
  gold_at(seed, i0, x1, x2);
  const uint32_t n = min((uint32_t)SEQ_PER_THREAD, len - i0);
#pragma unroll
  for (int c = 0; c < SEQ_PER_THREAD / 16; c++) {
    const uint32_t bits = gold16(x1, x2);
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t i = (uint32_t)(16 * c + k);
      if (i < n) {
        out[i0 + i] = (uint8_t)((bits >> k) & 1u);
      }
    }
  }
}

hipError_t seq_unpack_launch(uint8_t* d_out, uint32_t len, uint32_t seed, hipStream_t stream)
{
  if (len == 0) {
    return hipSuccess;
  }
  if (len > (1u << JUMP_BITS)) {
    return hipErrorInvalidValue;
  }
  hipError_t e = gold_tables_init();
  if (e != hipSuccess) {
    return e;
  }
  const dim3 grid((len + LLR_THREADS * SEQ_PER_THREAD - 1) / (LLR_THREADS * SEQ_PER_THREAD));
  hipLaunchKernelGGL(seq_unpack_kernel, grid, dim3(LLR_THREADS), 0, stream, d_out, len, seed);
  return hipGetLastError();
}

// ---------------------------------------------------------------- transmitter
// modulation tables of lte_tables.c:45-160, as the same float expressions
__device__ __forceinline__ float qam64_level(uint32_t hi, uint32_t lo)  // (b2, b4) -> 3, 1, 5, 7 / sqrt(42)
{
  const uint32_t m = hi * 2 + lo;
  return m == 0 ? 3.0f / sqrtf(42.0f) : m == 1 ? 1.0f / sqrtf(42.0f) : m == 2 ? 5.0f / sqrtf(42.0f) : 7.0f / sqrtf(42.0f);
}

// symbol of modulation `mod` (1 QPSK, 2 16QAM, 3 64QAM, 4 256QAM) from its Qm bits, b0 first (MSB)
__device__ __forceinline__ float2 modulate(int mod, uint32_t i)
{
  if (mod == 1) {
    const float l = (float)0.70710678118654752440;  // M_SQRT1_2
    return make_float2((i & 2u) ? -l : l, (i & 1u) ? -l : l);
  }
  if (mod == 2) {
    const float l1 = 1.0f / sqrtf(10.0f), l2 = 3.0f / sqrtf(10.0f);
    const float re = (i & 2u) ? l2 : l1, im = (i & 1u) ? l2 : l1;
    return make_float2((i & 8u) ? -re : re, (i & 4u) ? -im : im);
  }
  if (mod == 3) {
    const float re = qam64_level((i >> 3) & 1u, (i >> 1) & 1u), im = qam64_level((i >> 2) & 1u, i & 1u);
    return make_float2((i & 32u) ? -re : re, (i & 16u) ? -im : im);
  }
  float offset = -1, re = 0, im = 0;  // set_256QAMtable's loop
  for (uint32_t j = 0; j < 4; j++) {
    re += offset;
    im += offset;
    offset *= 2;
    re *= (i & (1u << (2 * j + 1))) ? +1 : -1;
    im *= (i & (1u << (2 * j + 0))) ? +1 : -1;
  }
  return make_float2(re / sqrtf(170), im / sqrtf(170));
}

static constexpr int TX_SPT = 16;  // symbols a thread (a whole number of bytes of e bits for every Qm)

// bits of TX_SPT symbols of one codeword starting at symbol k0: scrambled (sequences.c pdsch seed,
// srsran_sequence_pdsch_apply_pack) and mapped (srsran_mod_modulate_bytes)
__device__ __forceinline__ void tx_symbols(const uint8_t* __restrict__ e, uint32_t seed, int mod, uint32_t k0,
                                           uint32_t n, float2 (&x)[TX_SPT])
{
  const uint32_t Q = mod == 1 ? 2u : mod == 2 ? 4u : mod == 3 ? 6u : 8u;
  uint32_t       c[8];
  uint32_t       x1, x2;
  gold_at(seed, k0 * Q, x1, x2);
#pragma unroll
  for (int w = 0; w < 8; w++) {
    const uint32_t lo = gold16(x1, x2), hi = gold16(x1, x2);
    c[w]                = lo | (hi << 16);
  }
  const uint8_t* b = e + (k0 * Q) / 8;
#pragma unroll
  for (int s = 0; s < TX_SPT; s++) {
    uint32_t idx = 0;
    if (k0 + s < n) {
      for (uint32_t j = 0; j < Q; j++) {
        const uint32_t pos = s * Q + j;
        const uint32_t bit = ((b[pos >> 3] >> (7 - (pos & 7))) ^ (c[pos >> 5] >> (pos & 31))) & 1u;
        idx                = (idx << 1) | bit;
      }
    }
    x[s] = modulate(mod, idx);
  }
}

// one workgroup per LLR_THREADS * TX_SPT PDSCH REs of one subframe (grid.y = subframe)
__global__ __launch_bounds__(LLR_THREADS) void pdsch_tx_kernel(const PdschTx* __restrict__ items)
{
  const PdschTx& t  = items[blockIdx.y];
  const uint32_t k0 = (blockIdx.x * LLR_THREADS + threadIdx.x) * TX_SPT;
  if (k0 >= t.nre) {
    return;
  }
  float2 a[TX_SPT], b[TX_SPT];
  tx_symbols(t.e[0], t.seed[0], t.mod[0], k0, t.nre, a);
  if (t.scheme == 3) {
    tx_symbols(t.e[1], t.seed[1], t.mod[1], k0, t.nre, b);
  }
  const float sc = t.scaling;
#pragma unroll
  for (int s = 0; s < TX_SPT; s++) {
    const uint32_t k = k0 + s;
    if (k >= t.nre) {
      break;
    }
    const uint32_t g = t.idx[k] & 0x7fffffffu;
    if (t.scheme == 0) {  // srsran_precoding_single / 1 port
      t.grid[0][g] = sc == 1.0f ? a[s] : make_float2(a[s].x * sc, a[s].y * sc);
    } else if (t.scheme == 3) {  // srsran_precoding_cdd_2x2 (precoding.c:1996-2055)
      const float  nm = 0.5f * sc;
      const float2 y0 = make_float2((a[s].x + b[s].x) * nm, (a[s].y + b[s].y) * nm);
      const float2 y1 = (k & 1u) ? make_float2((-a[s].x + b[s].x) * nm, (-a[s].y + b[s].y) * nm)
                                 : make_float2((a[s].x - b[s].x) * nm, (a[s].y - b[s].y) * nm);
      t.grid[0][g] = y0;
      t.grid[1][g] = y1;
    } else if (t.scheme == 4) {  // transmit diversity, 4 ports (layermap.c:38-47 + precoding.c:1961-1988):
                                 // groups (4i .. 4i+3) of the codeword, SFBC on ports (0, 2) then (1, 3)
      const float  h  = t.div_scale;
      const float2 z  = make_float2(0.f, 0.f);
      const uint32_t b = (uint32_t)s & ~3u;  // k0 is a multiple of 4: the group is inside the thread
      const float2 x0 = a[b], x1 = a[b + 1], x2 = a[b + 2], x3 = a[b + 3];
      if (4 * (k / 4) + 3 >= t.nre) {
        break;  // a trailing half group is not transmitted (m_ap = 4 * (nre / 4))
      }
      switch (k & 3u) {
        case 0:
          t.grid[0][g] = make_float2(x0.x * h, x0.y * h);
          t.grid[1][g] = z;
          t.grid[2][g] = make_float2(-x1.x * h, x1.y * h);
          t.grid[3][g] = z;
          break;
        case 1:
          t.grid[0][g] = make_float2(x1.x * h, x1.y * h);
          t.grid[1][g] = z;
          t.grid[2][g] = make_float2(x0.x * h, -x0.y * h);
          t.grid[3][g] = z;
          break;
        case 2:
          t.grid[0][g] = z;
          t.grid[1][g] = make_float2(x2.x * h, x2.y * h);
          t.grid[2][g] = z;
          t.grid[3][g] = make_float2(-x3.x * h, x3.y * h);
          break;
        default:
          t.grid[0][g] = z;
          t.grid[1][g] = make_float2(x3.x * h, x3.y * h);
          t.grid[2][g] = z;
          t.grid[3][g] = make_float2(x2.x * h, -x2.y * h);
          break;
      }
    } else {  // transmit diversity, 2 ports (layermap.c + precoding.c:1943-1960): pairs (2i, 2i+1)
      const float  h  = t.div_scale;
      const bool   ev = (k & 1u) == 0;
      const float2 x0 = a[s & ~1], x1 = a[s | 1];  // k0 even: the pair (2i, 2i+1) is inside the thread
      if (ev) {
        t.grid[0][g] = make_float2(x0.x * h, x0.y * h);
        t.grid[1][g] = make_float2(-x1.x * h, x1.y * h);
      } else {
        t.grid[0][g] = make_float2(x1.x * h, x1.y * h);
        t.grid[1][g] = make_float2(x0.x * h, -x0.y * h);
      }
    }
  }
}

hipError_t pdsch_tx_launch(const PdschTx* d_items, uint32_t nitems, uint32_t max_nre, hipStream_t stream)
{
  if (nitems == 0 || max_nre == 0) {
    return hipSuccess;
  }
  hipError_t e = gold_tables_init();
  if (e != hipSuccess) {
    return e;
  }
  const dim3 grid((max_nre + LLR_THREADS * TX_SPT - 1) / (LLR_THREADS * TX_SPT), nitems);
  hipLaunchKernelGGL(pdsch_tx_kernel, grid, dim3(LLR_THREADS), 0, stream, d_items);
  return hipGetLastError();
}

// cell-specific reference signals of 1, 2 or 4 ports (refsignal_dl.c, 36.211 6.10.1): grid (CRS symbol of
// the subframe, port, subframe); 2 * nof_prb pilots a symbol
__global__ __launch_bounds__(256) void crs_put_kernel(float2* __restrict__ grids, uint32_t nof_prb, uint32_t cell_id,
                                                      uint32_t nports, uint32_t nsymb,
                                                      const uint32_t* __restrict__ sf_idx)
{
  // sym: 0..3 -> (slot, l in {0, nsymb - 3}); N_cp = 1 normal, 0 extended CP (refsignal_dl.c:81-97)
  const uint32_t sym = blockIdx.x, port = blockIdx.y, sf = blockIdx.z;
  const uint32_t slot = sym >> 1, l = (sym & 1) ? nsymb - 3 : 0u;
  const uint32_t ns   = 2 * sf_idx[sf] + slot;
  const uint32_t v    = port == 0 ? (l == 0 ? 0u : 3u) : (l == 0 ? 3u : 0u);
  if (port >= 2) {  // ports 2 / 3: one CRS symbol a slot, l = 1, v = 3 (ns mod 2) (+ 3 for port 3)
    if (sym & 1) {
      return;
    }
    const uint32_t l1 = 1, v1 = (3 * (ns & 1u) + (port == 3 ? 3u : 0u)) % 6;
    const uint32_t s1 = (1u << 10) * (7 * (ns + 1) + l1 + 1) * (2 * cell_id + 1) + 2 * cell_id + (nsymb == 7 ? 1u : 0u);
    float2* row1 = grids + (((size_t)sf * nports + port) * 2 * nsymb + nsymb * slot + l1) * (12 * nof_prb);
    for (uint32_t m = threadIdx.x; m < 2 * nof_prb; m += 256) {
      const uint32_t mp = m + 110 - nof_prb;
      uint32_t       x1, x2;
      gold_at(s1, 2 * mp, x1, x2);
      const uint32_t c = gold16(x1, x2);
      const float    r = (float)0.70710678118654752440;
      row1[6 * m + (v1 + cell_id % 6) % 6] = make_float2((c & 1u) ? -r : r, (c & 2u) ? -r : r);
    }
    return;
  }
  const uint32_t seed = (1u << 10) * (7 * (ns + 1) + l + 1) * (2 * cell_id + 1) + 2 * cell_id + (nsymb == 7 ? 1u : 0u);
  const uint32_t nre  = 12 * nof_prb;
  float2*        row  = grids + (((size_t)sf * nports + port) * 2 * nsymb + nsymb * slot + l) * nre;
  for (uint32_t m = threadIdx.x; m < 2 * nof_prb; m += 256) {
    const uint32_t mp = m + 110 - nof_prb;
    uint32_t       x1, x2;
    gold_at(seed, 2 * mp, x1, x2);
    const uint32_t c  = gold16(x1, x2);
    const float    r  = (float)0.70710678118654752440;
    row[6 * m + (v + cell_id % 6) % 6] = make_float2((c & 1u) ? -r : r, (c & 2u) ? -r : r);
  }
}

hipError_t crs_put_launch(float2* d_grids, uint32_t nof_prb, uint32_t cell_id, uint32_t nports, uint32_t nsymb,
                          const uint32_t* d_sf_idx, uint32_t nsf, hipStream_t stream)
{
  if (nsf == 0) {
    return hipSuccess;
  }
  if (nports == 0 || nports == 3 || nports > 4 || (nsymb != 7 && nsymb != 6)) {
    return hipErrorInvalidValue;
  }
  hipError_t e = gold_tables_init();
  if (e != hipSuccess) {
    return e;
  }
  hipLaunchKernelGGL(crs_put_kernel, dim3(4, nports, nsf), dim3(256), 0, stream, d_grids, nof_prb, cell_id, nports,
                     nsymb, d_sf_idx);
  return hipGetLastError();
}

// ---------------- control channels (enb_dl.c:333-420; pdcch.c:528-660, pcfich.c:185-235, pbch.c) ----------------
static constexpr int CC_NCOLS = 32;
__constant__ uint8_t kCcPerm[CC_NCOLS] = {1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
                                          0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30};

// bit k of the rate-matched tail-biting code of data[0..F) (rm_conv.c:40-90 bit collection over the
// sub-block interleaver, convcoder.c with polynomials 0x6D, 0x4F, 0x57 and K = 7)
__device__ __forceinline__ uint32_t cc_rm_bit(const uint8_t* data, int F, int k)
{
  const int nrows = (F - 1) / CC_NCOLS + 1, Kp = nrows * CC_NCOLS, nd = Kp - F, nv = 3 * F;
  int       r = k % nv;
  const int st = r / F;
  r -= st * F;
  int col = 0;
  for (; col < CC_NCOLS; col++) {  // the rank r among the column-ordered non-dummy entries
    const int cnt = nrows - (kCcPerm[col] < nd ? 1 : 0);
    if (r < cnt) {
      break;
    }
    r -= cnt;
  }
  const int row = r + (kCcPerm[col] < nd ? 1 : 0);
  const int bi  = row * CC_NCOLS + kCcPerm[col] - nd;  // encoder input bit
  uint32_t  sr  = 0;
  for (int t = bi - 6; t <= bi; t++) {
    sr = (sr << 1) | data[(t + F) % F];
  }
  const uint32_t poly = st == 0 ? 0x6Du : st == 1 ? 0x4Fu : 0x57u;
  return (uint32_t)__popc(sr & poly) & 1u;
}

// One 64-lane workgroup per job; a lane writes one transmit-diversity group (nports symbols) at a time.
__global__ __launch_bounds__(64) void ctrl_tx_kernel(const CtrlTxJob* __restrict__ jobs)
{
  const CtrlTxJob& j    = jobs[blockIdx.x];
  const int        lane = threadIdx.x;
  const uint32_t   P    = j.nports;
  if (j.kind == 2) {
    for (uint32_t s = lane; s < j.nsym; s += 64) {
      const float2   v   = j.seq[s];
      const uint32_t idx = j.re ? j.re[s] : j.re0 + s;
      for (uint32_t p = 0; p < P; p++) {
        j.grid[p][idx] = v;
      }
    }
    return;
  }
  __shared__ uint8_t data[128 + 16];
  const int          F = (int)j.nof_bits + 16;
  if (j.kind == 0) {
    for (uint32_t i = lane; i < j.nof_bits; i += 64) {
      data[i] = j.payload[i] & 1u;
    }
    if (lane == 0) {  // CRC16 (0x1021) of the payload, MSB first, masked (srsran_crc_attach + mask)
      uint32_t crc = 0;
      for (uint32_t i = 0; i < j.nof_bits; i++) {
        const uint32_t fb = ((crc >> 15) ^ j.payload[i]) & 1u;
        crc               = (crc << 1) & 0xffffu;
        crc ^= fb ? 0x1021u : 0u;
      }
      crc ^= j.crc_mask;
      for (int i = 0; i < 16; i++) {
        data[j.nof_bits + i] = (uint8_t)((crc >> (15 - i)) & 1u);
      }
    }
    __syncthreads();
  }
  const float h = P == 4 ? (float)(1.0f / 1.41421356237309504880) : (float)(1.0 * 0.70710678118654752440);
  const float a = (float)0.70710678118654752440;  // QPSK (lte_tables.c)
  for (uint32_t g = lane; g * P < j.nsym; g += 64) {
    const uint32_t s0 = g * P;
    if (j.kind == 0 && ((j.skip >> (s0 / 36)) & 1u)) {
      continue;
    }
    uint32_t x1, x2;
    gold_at(j.seed, j.seq_off + 2 * s0, x1, x2);
    const uint32_t c = gold16(x1, x2);
    float2         d[4];
    for (uint32_t q = 0; q < P; q++) {
      uint32_t b[2];
      for (int hb = 0; hb < 2; hb++) {
        const uint32_t i = 2 * (s0 + q) + hb;
        const uint32_t e = j.kind == 1 ? (uint32_t)((i % 3) != j.nof_bits - 1) : cc_rm_bit(data, F, (int)(j.bit0 + i));
        b[hb]            = e ^ ((c >> (2 * q + hb)) & 1u);
      }
      d[q] = make_float2(b[0] ? -a : a, b[1] ? -a : a);
    }
    uint32_t idx[4];
    for (uint32_t q = 0; q < P; q++) {
      idx[q] = j.re ? j.re[s0 + q] : j.re0 + s0 + q;
    }
    if (P == 1) {
      j.grid[0][idx[0]] = d[0];
    } else if (P == 2) {  // layermap_diversity + precoding_diversity, 2 ports (precoding.c:1943-1960)
      j.grid[0][idx[0]] = make_float2(d[0].x * h, d[0].y * h);
      j.grid[1][idx[0]] = make_float2(-d[1].x * h, d[1].y * h);
      j.grid[0][idx[1]] = make_float2(d[1].x * h, d[1].y * h);
      j.grid[1][idx[1]] = make_float2(d[0].x * h, -d[0].y * h);
    } else {  // 4 ports (precoding.c:1961-1988): SFBC on ports (0, 2) then (1, 3)
      const float2 z = make_float2(0.f, 0.f);
      j.grid[0][idx[0]] = make_float2(d[0].x * h, d[0].y * h);
      j.grid[1][idx[0]] = z;
      j.grid[2][idx[0]] = make_float2(-d[1].x * h, d[1].y * h);
      j.grid[3][idx[0]] = z;
      j.grid[0][idx[1]] = make_float2(d[1].x * h, d[1].y * h);
      j.grid[1][idx[1]] = z;
      j.grid[2][idx[1]] = make_float2(d[0].x * h, -d[0].y * h);
      j.grid[3][idx[1]] = z;
      j.grid[0][idx[2]] = z;
      j.grid[1][idx[2]] = make_float2(d[2].x * h, d[2].y * h);
      j.grid[2][idx[2]] = z;
      j.grid[3][idx[2]] = make_float2(-d[3].x * h, d[3].y * h);
      j.grid[0][idx[3]] = z;
      j.grid[1][idx[3]] = make_float2(d[3].x * h, d[3].y * h);
      j.grid[2][idx[3]] = z;
      j.grid[3][idx[3]] = make_float2(d[2].x * h, -d[2].y * h);
    }
  }
}

hipError_t ctrl_tx_launch(const CtrlTxJob* d_jobs, uint32_t njobs, hipStream_t stream)
{
  if (njobs == 0) {
    return hipSuccess;
  }
  hipError_t e = gold_tables_init();
  if (e != hipSuccess) {
    return e;
  }
  hipLaunchKernelGGL(ctrl_tx_kernel, dim3(njobs), dim3(64), 0, stream, d_jobs);
  return hipGetLastError();
}

}  // namespace srsran_amd
