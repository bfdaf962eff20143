// srsran_4g_amd/csrc/tdecs_kernel.hip -- LTE turbo decoder of the window classes (16 sub-blocks for
// K >= 816, 8 sub-blocks for 408 <= K <= 800), ONE LANE PER SUB-BLOCK: the throughput mapping on CDNA4.
// Compiled once per class (Makefile: -DTDECS_NSB=16 -> namespace tdecs16, kernels tdec16s_*;
// -DTDECS_NSB=8 -> tdecs8, tdec8s_*).
//
// Same arithmetic, schedule and LDS bookkeeping as tdec16_kernel.hip (bit-exact with srsRAN_4G's AVX2
// 16-bit window decoder, turbodecoder_win.h:480-832, driven by turbodecoder_iter.h:72-144 on the
// rm_turbo sub-block input layout); only the mapping of the trellis differs:
//
//   * the 8 states of a sub-block live in ONE lane as four packed int16 registers.  A trellis step
//     (forward or backward) is two "s" butterflies  (max(u, v + s), max(v, u + s))  and two "xy"
//     butterflies  (max(u + y, v + x), max(v + y, u + x))  on the four registers (u, v), with
//     s = sat(x + y):  2 + 2 + 3 + 3 = 10 v_pk_add_i16 clamp / v_pk_max_i16 whose operand halves are
//     chosen by op_sel, then 4 v_perm_b32 that re-pair the outputs for the next step.  No lane
//     exchange, no DPP, 4 independent chains per step (the VALU hazard slots fill themselves).
//     The pairings that make the forward and the backward trellis the SAME instruction sequence
//     (only two perm selectors differ):
//         alpha:  (a0,a1) (a7,a6) (a3,a2) (a4,a5)    beta:  (b0,b4) (b7,b3) (b2,b6) (b5,b1)
//     and the forward step's candidates pair with the betas of the LLR in the same registers
//     (derivation in DESIGN.md section 4.1).
//   * per code block NSB lanes a side: a wave holds the forward (alpha) side of 64 / NSB code blocks,
//     its partner wave their backward (beta) side: 128-thread workgroups of 64 / NSB blocks of one K.
//     Half the lanes of the lane-pair kernel per block and none of its duplicated loads, LDS writes and
//     LLR work.  The 8-sub-block class is the SSE 8-block window decoder (turbodecoder_win.h with
//     WINIMP sse16): the same arithmetic on half as many sub-blocks.
//   * LDS per code block exactly as tdec16_kernel.hip: the in-place a-priori / extrinsic array S over
//     the soft-buffer slots, beta / alpha checkpoints (one state = 16 B per sub-block and window) and
//     the decision bitmap.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc24_dev.h"
#include "stage_timing.h"
#include "tdec_kernel.h"

#ifndef TDECS_NSB
#define TDECS_NSB 16
#endif
#ifndef TDECS_W
#define TDECS_W 16
#endif
#if TDECS_NSB == 16 && TDECS_W == 16
#define TDECS_NS tdecs16
#define TDECS_K(n) tdec16s_##n
#define TDECS_NAME "tdec16s_"
#elif TDECS_NSB == 8 && TDECS_W == 16
#define TDECS_NS tdecs8
#define TDECS_K(n) tdec8s_##n
#define TDECS_NAME "tdec8s_"
#elif TDECS_NSB == 16 && TDECS_W == 8
#define TDECS_NS tdecs16w8
#define TDECS_K(n) tdec16sw8_##n
#define TDECS_NAME "tdec16sw8_"
#elif TDECS_NSB == 8 && TDECS_W == 8
#define TDECS_NS tdecs8w8
#define TDECS_K(n) tdec8sw8_##n
#define TDECS_NAME "tdec8sw8_"
#else
#error "TDECS_NSB must be 16 or 8, TDECS_W 16 or 8"
#endif

namespace srsran_amd {
namespace TDECS_NS {
namespace {

typedef short v2s __attribute__((ext_vector_type(2)));

constexpr int   W    = TDECS_W;       // window: steps between checkpoints (16; 8 for fewer registers)
constexpr int   OVL  = TDEC_OVERLAP;  // win_overlap_len (turbodecoder_win.h:54)
constexpr int   NTR  = (OVL + W - 1) / W;  // training windows (the last one partial when W does not divide 40)
constexpr int   NSB  = TDECS_NSB;     // nof_blocks of the window decoder (avx16: 16, sse16: 8)
constexpr short NEG  = -10000;        // -INF (turbodecoder_win.h:56)
constexpr int   CPWG = 64 / NSB;      // code blocks per workgroup (one wave a side)
constexpr int   ROWB = 2 * NSB;       // bytes of one position row of the SB input (all sub-blocks)

#ifdef TDECS_STAMPS
// Diagnostic build only (Makefile `stamps`, tools/tdec_stamps.py; never the product library): lane 0 of
// every wave writes the shader clock at the phase boundaries of every half-iteration into a debug
// buffer, [workgroup][wave][64 stamps], with an ordinary vector store.
__device__ unsigned long long* g_stamps = nullptr;
#define TDECS_STAMP(k)                                                                               \
  do {                                                                                               \
    if ((threadIdx.x & 63) == 0 && g_stamps && (k) < 64) {                                          \
      g_stamps[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64 + (k)] = clock64(); \
    }                                                                                                \
  } while (0)
#else
#define TDECS_STAMP(k) \
  do {                 \
  } while (0)
#endif

__device__ __forceinline__ v2s u2v(uint32_t u) { return __builtin_bit_cast(v2s, u); }
__device__ __forceinline__ uint32_t v2u(v2s v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ v2s padd(v2s a, v2s b) { return __builtin_elementwise_add_sat(a, b); }
__device__ __forceinline__ v2s psub(v2s a, v2s b) { return __builtin_elementwise_sub_sat(a, b); }
__device__ __forceinline__ v2s pmax(v2s a, v2s b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ v2s lo2(v2s a) { return __builtin_shufflevector(a, a, 0, 0); }
__device__ __forceinline__ v2s hi2(v2s a) { return __builtin_shufflevector(a, a, 1, 1); }
__device__ __forceinline__ v2s swp(v2s a) { return __builtin_shufflevector(a, a, 1, 0); }
// v_perm_b32: selector bytes 0-3 pick bytes of lo_src, 4-7 bytes of hi_src
__device__ __forceinline__ v2s perm(v2s hi_src, v2s lo_src, uint32_t sel)
{
  return u2v(__builtin_amdgcn_perm(v2u(hi_src), v2u(lo_src), sel));
}

// Trellis state of one sub-block (four packed int16 registers, layouts in the header comment).
struct St {
  v2s a, b, c, d;
};

// Re-pairing selectors of the two registers whose pairing differs between the directions:
//   alpha: c = (o2.lo, o4.lo), d = (o1.hi, o3.hi);   beta: c = (o4.lo, o2.lo), d = (o3.hi, o1.hi)
template <bool BETA>
struct Sel {
  static constexpr uint32_t c = BETA ? 0x01000504u : 0x05040100u;  // perm(o4, o2, .)
  static constexpr uint32_t d = BETA ? 0x03020706u : 0x07060302u;  // perm(o3, o1, .)
};

// Branch metrics of a position: xy = (x lo, y hi); s = sat(x + y) in both halves.
struct Bm {
  v2s s, x, y;
};
__device__ __forceinline__ Bm bm(uint32_t xyw)
{
  const v2s xy = u2v(xyw);
  return Bm{padd(xy, swp(xy)), lo2(xy), hi2(xy)};
}

// The two candidates of each output pair (c0: bit-0 branch, c1: bit-1 branch), before the max.
// Output pairs: alpha (n0,n4) (n3,n7) (n1,n5) (n2,n6); beta (n0,n1) (n6,n7) (n4,n5) (n2,n3).
struct Cand {
  v2s c01, c11, c02, c12, c03, c13, c04, c14;
};
__device__ __forceinline__ Cand cand(const St& p, const Bm& m)
{
  Cand c;
  c.c01 = p.a;
  c.c11 = padd(swp(p.a), m.s);
  c.c02 = p.b;
  c.c12 = padd(swp(p.b), m.s);
  c.c03 = padd(p.c, m.y);
  c.c13 = padd(swp(p.c), m.x);
  c.c04 = padd(p.d, m.y);
  c.c14 = padd(swp(p.d), m.x);
  return c;
}
template <bool BETA>
__device__ __forceinline__ St next(const Cand& c)
{
  const v2s o1 = pmax(c.c01, c.c11);
  const v2s o2 = pmax(c.c02, c.c12);
  const v2s o3 = pmax(c.c03, c.c13);
  const v2s o4 = pmax(c.c04, c.c14);
  return St{perm(o3, o1, 0x05040100u), perm(o4, o2, 0x07060302u), perm(o4, o2, Sel<BETA>::c), perm(o3, o1, Sel<BETA>::d)};
}
// Forward (turbodecoder_win.h:767-787) or backward (win.h:641-664) trellis step.
template <bool BETA>
__device__ __forceinline__ St step(const St& p, uint32_t xyw)
{
  return next<BETA>(cand(p, bm(xyw)));
}

// LLR of a position from the forward candidates of alpha_k and beta_{k+1} (win.h:788-815):
// max_s(beta + c1) - max_s(beta + c0).  The beta pairs line up with the candidate pairs:
// (b0,b4) = B.a, (b3,b7) = swp(B.b), (b1,b5) = swp(B.d), (b2,b6) = B.c.
__device__ __forceinline__ short llr(const Cand& c, const St& B)
{
  const v2s b1 = B.a, b2 = swp(B.b), b3 = swp(B.d), b4 = B.c;
  const v2s m0 = pmax(pmax(padd(b1, c.c01), padd(b2, c.c02)), pmax(padd(b3, c.c03), padd(b4, c.c04)));
  const v2s m1 = pmax(pmax(padd(b1, c.c11), padd(b2, c.c12)), pmax(padd(b3, c.c13), padd(b4, c.c14)));
  return psub(pmax(m1, swp(m1)), pmax(m0, swp(m0))).x;
}

// normalize() (turbodecoder_win.h:480-498): subtract state 0 (the low half of register a in both
// layouts), saturating.
__device__ __forceinline__ St norm(const St& p)
{
  const v2s z = lo2(p.a);
  return St{psub(p.a, z), psub(p.b, z), psub(p.c, z), psub(p.d, z)};
}
__device__ __forceinline__ bool norm_at(int k) { return (k & 1) == 0 && k != 0; }  // normalize_period 2
__device__ __forceinline__ bool nrm(int t0, int i) { return (i & 1) == 0 && (i != 0 || t0 != 0); }

__device__ __forceinline__ St neg_state() { return St{v2s{NEG, NEG}, v2s{NEG, NEG}, v2s{NEG, NEG}, v2s{NEG, NEG}}; }
__device__ __forceinline__ St alpha_known() { return St{v2s{0, NEG}, v2s{NEG, NEG}, v2s{NEG, NEG}, v2s{NEG, NEG}}; }

// beta_trellis (turbodecoder_win.h:500-548): the tail steps K+2..K of the last sub-block,
// non-saturating (sadd without use_saturated_add), in the beta layout.
__device__ __forceinline__ St trellis(const short* xt, const short* yt)
{
  short o[8] = {0, NEG, NEG, NEG, NEG, NEG, NEG, NEG};
#pragma unroll
  for (int t = 2; t >= 0; t--) {
    const short x = xt[t], y = yt[t], xy = (short)(x + y);
    short       n[8];
    n[0] = max(o[0], (short)(o[4] + xy));
    n[1] = max((short)(o[0] + xy), o[4]);
    n[2] = max((short)(o[1] + x), (short)(o[5] + y));
    n[3] = max((short)(o[1] + y), (short)(o[5] + x));
    n[4] = max((short)(o[2] + y), (short)(o[6] + x));
    n[5] = max((short)(o[2] + x), (short)(o[6] + y));
    n[6] = max((short)(o[3] + xy), o[7]);
    n[7] = max(o[3], (short)(o[7] + xy));
#pragma unroll
    for (int i = 0; i < 8; i++) {
      o[i] = n[i];
    }
  }
  return St{v2s{o[0], o[4]}, v2s{o[7], o[3]}, v2s{o[2], o[6]}, v2s{o[5], o[1]}};
}

// LDS of one code block (dwords): S [NSB*Ls int16] | CK [M windows][NSB lanes][16 B] | BITS | RED [2].  BITS holds
// the hard decisions (emit): plain launches in natural order, K/8 bytes; DL-SCH batches (slot) by soft-buffer slot,
// as S: bit `slot` (dword slot / 32, bit slot % 32) is natural position j L + r for slot = j Ls + r -- a DEC1 lane's
// window is a run of consecutive bits, a DEC2 position's bit is its slot's (no division, no multiply); nat_byte()
// reads natural-order bytes out of it -- NSB*Ls bits + a guard dword.
struct Geo {
  int s_dw, ck_dw, bits_dw, cb_dw;
};
__host__ __device__ __forceinline__ Geo geo(int K, int Ls, int M, bool slot)
{
  Geo g;
  g.s_dw    = (NSB * Ls + 1) / 2;
  g.ck_dw   = M * NSB * 4;
  g.bits_dw = slot ? (NSB * Ls + 31) / 32 + 1 : (K / 8 + 3) / 4;
  g.cb_dw   = g.s_dw + g.ck_dw + g.bits_dw + 2;
  return g;
}

struct Raw {
  uint32_t a[W];  // systematic LLR (DEC1) / slot of pi(position) (DEC2)
  uint32_t b[W];  // parity0 / parity1
};

typedef short __attribute__((address_space(3)))* lshort;
typedef __amdgpu_buffer_rsrc_t                   rsrc_t;
__device__ __forceinline__ uint32_t ldb(rsrc_t r, uint32_t voff, uint32_t soff, int imm)
{
  return __builtin_amdgcn_raw_buffer_load_b16(r, voff + imm, soff, 0);
}
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes)
{
  const size_t   u  = (size_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((size_t)hi << 32) | lo), 0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

struct Lane {
  int       s, K, L, Ls, M, KP;
  uint32_t  magicLs;
  rsrc_t    rin;   // the workgroup's blocks' inputs, from the lowest of them
  uint32_t  voff;  // bytes from rin's base to this lane's first position (q = s) of its block
  rsrc_t    rtf;   // tfwd (q order, SB input: slot of pi(n(q))), K entries
  lshort    S;     // this block's S (LDS)
  lshort    Ssb;   // S + s * Ls: this lane's sub-block
  uint4*    CK;    // this block's checkpoints (LDS), [M][NSB]
  uint32_t* BITS;  // this block's decision bitmap (LDS)
};

__device__ __forceinline__ void ck_put(const Lane& c, int m, const St& p)
{
  c.CK[m * NSB + c.s] = make_uint4(v2u(p.a), v2u(p.b), v2u(p.c), v2u(p.d));
}
__device__ __forceinline__ St ck_get(const Lane& c, int m)
{
  const uint4 v = c.CK[m * NSB + c.s];
  return St{u2v(v.x), u2v(v.y), u2v(v.z), u2v(v.w)};
}

template <bool D2>
__device__ __forceinline__ void issue(const Lane& c, Raw& r, int t0)
{
  const uint32_t soff = (uint32_t)ROWB * (uint32_t)t0;
  const uint32_t poff = soff + (D2 ? 4u : 2u) * (uint32_t)c.KP;  // parity stream, bytes
#ifdef TDECS_FAKELOAD  // diagnostic timing build only: no global loads (results are garbage)
#pragma unroll
  for (int i = 0; i < W; i++) {
    r.a[i] = D2 ? (uint32_t)((c.s * 37 + t0 + i) & 511) : (soff + i) & 0xff;  // slots < 512 <= K
    r.b[i] = (poff + 3 * i) & 0xff;
  }
#else
#pragma unroll
  for (int i = 0; i < W; i++) {
    r.a[i] = D2 ? ldb(c.rtf, 2u * (uint32_t)c.s, soff, ROWB * i) : ldb(c.rin, c.voff, soff, ROWB * i);
    r.b[i] = ldb(c.rin, c.voff, poff, ROWB * i);
  }
#endif
}

__device__ __forceinline__ uint32_t pin(uint32_t v)
{
  asm volatile("" : "+v"(v));
  return v;
}

// The LLR o of position k: S update (vec_sub, wraps) and, when the half-iteration's decision is
// needed, its bit (turbodecoder.c:370-378: the sign of ext1 after DEC1, of app1 after DEC2).  Two bit layouts:
//  * BITS == 1 (plain launches): natural order, srsran_bit_pack's bytes (MSB first) -- the output copies bytes;
//  * BITS == 2 (DL-SCH batches, CRC every half-iteration): by soft-buffer slot (Geo) -- DEC1 returns the bit (the
//    caller gathers a window's bits and stores them once, flush_bits), DEC2 sets its slot's bit (no division).
// The plain launches keep the natural layout: their code (the all-188 step's) measured faster with it.
__device__ __forceinline__ void set_nat(const Lane& c, int n, short o)
{
  atomicOr(&c.BITS[n >> 5], (uint32_t)(o > 0) << (((n >> 3) & 3) * 8 + 7 - (n & 7)));
}

template <bool D2, int BITS>
__device__ __forceinline__ uint32_t emit(const Lane& c, int k, short o, uint32_t aux, uint32_t xw)
{
  if (D2) {
    const lshort p = (lshort)(size_t)aux;
    *p             = (short)(o - (short)(xw & 0xffffu));
    if (BITS == 2) {
      const uint32_t slot = (uint32_t)(p - c.S);
      atomicOr(&c.BITS[slot >> 5], (uint32_t)(o > 0) << (slot & 31));
    } else if (BITS == 1) {
      const int slot = (int)(p - c.S);
      const int sb   = (int)__umulhi((uint32_t)slot, c.magicLs);
      set_nat(c, slot - sb * (c.Ls - c.L), o);
    }
    return 0;
  }
  c.Ssb[k] = (short)(o - (short)aux);
  if (BITS == 1) {
    set_nat(c, c.s * c.L + k, o);
  }
  return BITS == 2 ? (uint32_t)(o > 0) : 0u;
}

// DEC1: the decisions of a window t0 .. t0 + W - 1 of this lane's sub-block (bit i = position t0 + i), slots
// s Ls + t0 .. + W - 1: one or two dwords (shared with the other wave's windows and the neighbouring sub-blocks: OR)
__device__ __forceinline__ void flush_bits(const Lane& c, int t0, uint32_t wbits)
{
  if (wbits) {
    const uint32_t pos = (uint32_t)(c.s * c.Ls + t0);
    const uint64_t v   = (uint64_t)wbits << (pos & 31);
    atomicOr(&c.BITS[pos >> 5], (uint32_t)v);
    if ((uint32_t)(v >> 32)) {
      atomicOr(&c.BITS[(pos >> 5) + 1], (uint32_t)(v >> 32));
    }
  }
}

// Natural-order byte b of the decisions (8 positions MSB first, as srsran_bit_pack): positions n = 8b .. 8b + 7 of
// sub-block j = n / L (magicL = ceil(2^32 / L): exact for n < 2^16) are slots n + j (Ls - L): nine bits from there,
// the padding slot between sub-blocks j and j + 1 (Ls - L = 1 for even L, never set) squeezed out
__device__ __forceinline__ uint32_t nat_byte(const uint32_t* bits, int L, int Ls, uint32_t magicL, int b)
{
  const int      n0  = 8 * b;
  const int      j   = (int)__umulhi((uint32_t)n0, magicL);
  const int      cnt = (j + 1) * L - n0;  // positions left in sub-block j
  const uint32_t s0  = (uint32_t)(n0 + j * (Ls - L));
  const uint64_t v   = (uint64_t)bits[s0 >> 5] | (uint64_t)bits[(s0 >> 5) + 1] << 32;
  uint32_t       x   = (uint32_t)(v >> (s0 & 31)) & 0x1ffu;
  if (cnt < 8) {
    x = (x & ((1u << cnt) - 1u)) | ((x >> (cnt + Ls - L)) << cnt);
  }
  return __builtin_bitreverse32(x & 0xffu) >> 24;
}

// Phase-2 alpha side, window at t0 >= W: beta[t0+1 .. cc] recomputed from the stored beta at
// cc = min(t0 + W, L) (checkpoint), then alpha + LLR of t0 .. cc-1.
template <bool D2, int BITS, bool FULL>
__device__ __forceinline__ St alpha_llr_window(const Lane& c, St P, int t0, St Pb, const uint32_t* xw,
                                               const uint32_t* aux)
{
  const int L  = c.L;
  const int cc = FULL ? t0 + W : L;
  const int ic = cc - t0 - 1;
  St        bw[W];
#pragma unroll
  for (int i = W - 1; i >= 0; i--) {
    if (FULL ? i == W - 1 : i == ic) {
      bw[i] = Pb;
      if (cc < L && norm_at(cc)) Pb = norm(Pb);
    } else if (FULL || i < ic) {
      Pb    = step<true>(Pb, xw[i + 1]);
      bw[i] = Pb;
      if (FULL ? (i & 1) : norm_at(t0 + 1 + i)) Pb = norm(Pb);
    }
  }
  uint32_t wbits = 0;
#pragma unroll
  for (int i = 0; i < W; i++) {
    if (FULL || t0 + i < L) {
      const Cand  cd = cand(P, bm(xw[i]));
      const short o  = llr(cd, bw[i]);
      P              = next<false>(cd);
      if ((i & 1) == 0) P = norm(P);  // t0 >= W: every even position
      wbits |= emit<D2, BITS>(c, t0 + i, o, aux[i], xw[i]) << i;
    }
  }
  if (BITS == 2 && !D2) {
    flush_bits(c, t0, wbits);
  }
  return P;
}

// Phase-1 beta side, window at t0 >= W: backward over t0+W-1 .. t0 (FULL) or L-1 .. t0; Bst = the
// stored beta at t0, which is the checkpoint of window t0/W - 1 when `store`.
template <bool FULL>
__device__ __forceinline__ St beta_window(const Lane& c, St P, int t0, bool store, St& Bst, const uint32_t* xw)
{
#pragma unroll
  for (int i = W - 1; i >= 0; i--) {
    if (FULL || t0 + i < c.L) {
      P = step<true>(P, xw[i]);
      if (i == 0) {
        Bst = P;
        if (store) {
          ck_put(c, t0 / W - 1, P);
        }
      }
      if ((i & 1) == 0) P = norm(P);
    }
  }
  return P;
}

// Window inputs of one side, prefetched along the side's window sequence (as tdec16_kernel.hip):
//   alpha side: training [L-40, L-24), [L-24, L-8), [L-8, L); then windows 0, 1, ..., Ma-1
//   beta side:  training [32, 40), [16, 32), [0, 16);       then windows Ma-1, ..., 1, 0
template <bool D2>
struct Pipe {
  Raw      g;
  uint32_t dv[W];
  int      nwin, Ma;
  bool     beta;

  __device__ __forceinline__ int t0_of(int idx, int L) const
  {
    if (beta) {
      return idx < NTR ? (NTR - 1 - idx) * W : (Ma - 1 - (idx - NTR)) * W;
    }
    return idx < NTR ? L - OVL + W * idx : (idx - NTR) * W;
  }

  __device__ __forceinline__ void load(const Lane& c, int idx)
  {
    if (idx < nwin) {
      const int t0 = t0_of(idx, c.L);
      issue<D2>(c, g, t0);
      if (!D2) {
#pragma unroll
        for (int i = 0; i < W; i++) {
          dv[i] = (uint16_t)c.Ssb[t0 + i];
        }
      }
    }
  }
  __device__ __forceinline__ void start(const Lane& c) { load(c, 0); }
  __device__ __forceinline__ void next(const Lane& c, int idx, uint32_t* xw, uint32_t* aux)
  {
    if (D2) {
      uint32_t d[W], hi[W];
#pragma unroll
      for (int i = 0; i < W; i++) {
        aux[i] = (uint32_t)(size_t)(c.S + g.a[i]);
        d[i]   = (uint16_t)*(lshort)(size_t)aux[i];
        hi[i]  = g.b[i] << 16;
      }
      load(c, idx + 1);
#pragma unroll
      for (int i = 0; i < W; i++) {
        xw[i] = pin(hi[i] | d[i]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < W; i++) {
        xw[i]  = pin(v2u(padd(u2v(__builtin_amdgcn_perm(g.b[i], g.a[i], 0x05040100u)), u2v(dv[i]))));
        aux[i] = dv[i];
      }
      load(c, idx + 1);
    }
  }
};

// One constituent MAP decode of this lane's sub-block; wave 0 = alpha side, wave 1 = beta side.
template <bool D2, int BITS>
__device__ __forceinline__ void map16s(const Lane& cin, int wave, int st0)
{
  (void)st0;  // first stamp index of this half-iteration (TDECS_STAMPS builds)
  Lane c = cin;
  asm volatile("" : "+v"(c.s));
  asm volatile("" : "+v"(c.voff));
  {
    uint32_t ssb = (uint32_t)(size_t)c.Ssb;
    asm volatile("" : "+v"(ssb));
    c.Ssb = (lshort)(size_t)ssb;
  }
  const int L     = c.L;
  const int Mfull = L / W;
  const int Ma    = (L + W - 1) / W;
  const int h     = max(1, min((L + W) / (2 * W), L / W));
  Pipe<D2>  pp;
  pp.nwin = NTR + Ma;
  pp.Ma   = Ma;
  pp.beta = __builtin_amdgcn_readfirstlane(wave) != 0;
  uint32_t xw[W];
  uint32_t aux[W];
  pp.start(c);
  if (wave == 0) {
    // ================= alpha side =================
    St P = neg_state();
    TDECS_STAMP(st0);
    // training over the last 40 steps of the own sub-block (win.h:747-756)
#pragma unroll
    for (int w = 0; w < NTR; w++) {
      pp.next(c, w, xw, aux);
#pragma unroll
      for (int i = 0; i < (W < OVL - w * W ? W : OVL - w * W); i++) {
        P = step<false>(P, xw[i]);
        if (norm_at(w * W + i)) P = norm(P);
      }
    }
    TDECS_STAMP(st0 + 1);
    {  // move_left: sub-block s starts from the training state of s - 1; s = 0 is known
      St q;
      q.a = u2v((uint32_t)__shfl_up((int)v2u(P.a), 1, NSB));
      q.b = u2v((uint32_t)__shfl_up((int)v2u(P.b), 1, NSB));
      q.c = u2v((uint32_t)__shfl_up((int)v2u(P.c), 1, NSB));
      q.d = u2v((uint32_t)__shfl_up((int)v2u(P.d), 1, NSB));
      P   = c.s == 0 ? alpha_known() : q;
    }
    // phase 1: windows [0, h) (all full), entry checkpoints in slots 0..h-1
#pragma unroll 1
    for (int ma = 0; ma < h; ma++) {
      const int t0 = ma * W;
      pp.next(c, NTR + ma, xw, aux);
      ck_put(c, ma, P);
#pragma unroll
      for (int i = 0; i < W; i++) {
        P = step<false>(P, xw[i]);
        if (nrm(t0, i)) P = norm(P);
      }
    }
    TDECS_STAMP(st0 + 2);
    __syncthreads();
    TDECS_STAMP(st0 + 3);
    // phase 2: windows [h, Ma): beta recomputed from the checkpoint above the window, then alpha + LLR
#pragma unroll 1
    for (int ma = h; ma < Mfull; ma++) {
      pp.next(c, NTR + ma, xw, aux);
      P = alpha_llr_window<D2, BITS, true>(c, P, ma * W, ck_get(c, ma), xw, aux);
    }
    if (Ma > Mfull) {
      pp.next(c, NTR + Mfull, xw, aux);
      alpha_llr_window<D2, BITS, false>(c, P, Mfull * W, ck_get(c, Mfull), xw, aux);
    }
    TDECS_STAMP(st0 + 4);
  } else {
    // ================= beta side =================
    St P = neg_state();
    TDECS_STAMP(st0);
    // training over the first 40 steps of the own sub-block, backwards (win.h:622-630)
#pragma unroll
    for (int w = 0; w < NTR; w++) {  // the top (maybe partial) training window first
      pp.next(c, w, xw, aux);
      const int t0 = (NTR - 1 - w) * W;
#pragma unroll
      for (int i = (W < OVL - t0 ? W : OVL - t0) - 1; i >= 0; i--) {
        P = step<true>(P, xw[i]);
        if (norm_at(t0 + i)) P = norm(P);
      }
    }
    TDECS_STAMP(st0 + 1);
    {  // move_right: sub-block s starts from the training state of s + 1; the last from the tail
      St q;
      q.a = u2v((uint32_t)__shfl_down((int)v2u(P.a), 1, NSB));
      q.b = u2v((uint32_t)__shfl_down((int)v2u(P.b), 1, NSB));
      q.c = u2v((uint32_t)__shfl_down((int)v2u(P.c), 1, NSB));
      q.d = u2v((uint32_t)__shfl_down((int)v2u(P.d), 1, NSB));
      if (c.s == NSB - 1) {  // trellis termination: systematic / parity0 (DEC1), app2 / parity1 (DEC2)
        const int tail = 6 * c.KP + (D2 ? 12 : 0);  // bytes
        short     xt[3], yt[3];
#pragma unroll
        for (int t = 0; t < 3; t++) {
          xt[t] = (short)ldb(c.rin, c.voff - 2 * c.s, tail, 4 * t);
          yt[t] = (short)ldb(c.rin, c.voff - 2 * c.s, tail, 4 * t + 2);
        }
        P = trellis(xt, yt);
      } else {
        P = q;
      }
    }
    const int mtop = Ma - 1;
    ck_put(c, mtop, P);  // beta[L]
    St Bst = P;  // stored (pre-normalisation) beta of the position above the current window
    // phase 1: windows [h, Ma) from the top (the top one maybe partial)
    if (Ma > Mfull) {
      pp.next(c, NTR, xw, aux);
      P = beta_window<false>(c, P, mtop * W, mtop > h, Bst, xw);
    }
#pragma unroll 1
    for (int mb = Mfull - 1; mb >= h; mb--) {
      pp.next(c, NTR + mtop - mb, xw, aux);
      P = beta_window<true>(c, P, mb * W, mb > h, Bst, xw);
    }
    TDECS_STAMP(st0 + 2);
    __syncthreads();
    TDECS_STAMP(st0 + 3);
    // phase 2: windows [0, h) from the top: alpha recomputed from the entry checkpoint, then
    // beta backwards with the LLR of every position
#pragma unroll 1
    for (int mb = h - 1; mb >= 0; mb--) {
      const int t0 = mb * W;
      pp.next(c, NTR + mtop - mb, xw, aux);
      St Pa = ck_get(c, mb);
      St aw[W];  // alpha entering each position (candidates rebuilt at LLR time)
#pragma unroll
      for (int i = 0; i < W; i++) {
        aw[i] = Pa;
        if (i < W - 1) {
          Pa = step<false>(Pa, xw[i]);
          if (nrm(t0, i)) Pa = norm(Pa);
        }
      }
      uint32_t wbits = 0;
#pragma unroll
      for (int i = W - 1; i >= 0; i--) {
        const short o = llr(cand(aw[i], bm(xw[i])), Bst);
        P             = step<true>(P, xw[i]);
        Bst           = P;
        if (nrm(t0, i)) P = norm(P);
        wbits |= emit<D2, BITS>(c, t0 + i, o, aux[i], xw[i]) << i;
      }
      if (BITS == 2 && !D2) {
        flush_bits(c, t0, wbits);
      }
    }
    TDECS_STAMP(st0 + 4);
  }
}

}  // namespace

template <bool ES>
__device__ __forceinline__ void body(const TdecArgs& a, int bid)
{
  constexpr int NT = 128;  // threads: the alpha and the beta wave
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int cbw  = lane / NSB;        // block of the workgroup
  const int s    = lane % NSB;        // sub-block
  const int t2   = wave * NSB + s;    // thread within the block (both sides), 0..2 NSB - 1
  const int K    = (int)a.K;
  const int L    = (int)a.L;
  const int Ls   = (int)a.Ls;
  const int M    = (L + W - 1) / W;
  const Geo g    = geo(K, Ls, M, ES);
  const int cb   = bid * CPWG + cbw;
  const int cbl  = cb < (int)a.ncb ? cb : (int)a.ncb - 1;
  const bool live = cb < (int)a.ncb && (!ES || a.cbs[cbl].slot != TDEC_PAD_SLOT);
  bool done      = ES && (!live || *a.cbs[cbl].skip);

  uint32_t* base = smem + cbw * g.cb_dw;
  Lane      c;
  c.s       = s;
  c.K       = K;
  c.L       = L;
  c.Ls      = Ls;
  c.M       = M;
  c.KP      = K + 32;  // SB stream stride (rm_turbo.c:260-273)
  c.magicLs = a.magicLs;
  const uint32_t magicL = 0xffffffffu / (uint32_t)L + 1u;  // ceil(2^32 / L) (2^32 / L for a power of two)
  // the workgroup's blocks read through one uniform base: the lowest of their inputs (plain launches:
  // in_stride apart; DL-SCH: the host keeps every group of CPWG descriptors within TDEC_PAIR_SPAN)
  const int cb0 = bid * CPWG;
  size_t    in_lane, in_lo = SIZE_MAX, in_hi = 0;
#pragma unroll
  for (int i = 0; i < CPWG; i++) {
    const int    j = min(cb0 + i, (int)a.ncb - 1);
    const size_t p = ES ? (size_t)a.cbs[j].in : (size_t)(a.in + (size_t)j * a.in_stride);
    in_lo          = min(in_lo, p);
    in_hi          = max(in_hi, p);
  }
  in_lane                 = ES ? (size_t)a.cbs[cbl].in : (size_t)(a.in + (size_t)cbl * a.in_stride);
  const uint32_t cb_bytes = (uint32_t)(3 * c.KP + 12) * 2;  // one block's soft-buffer input
  c.rin  = make_rsrc((const void*)in_lo, (uint32_t)(in_hi - in_lo) + cb_bytes);
  c.voff = (uint32_t)(in_lane - in_lo) + 2 * c.s;
  c.rtf  = make_rsrc(a.tfwd, 2u * (uint32_t)K);
  c.S    = (lshort)(short*)base;
  c.Ssb  = c.S + c.s * Ls;
  c.CK   = reinterpret_cast<uint4*>(base + g.s_dw);
  c.BITS = base + g.s_dw + g.ck_dw;
  uint32_t* RED = c.BITS + g.bits_dw;

  if constexpr (ES) {
    if (live && done && t2 == 0) {  // skipped block (sch.c:392, 476-480)
      const uint32_t slot = a.cbs[cbl].slot;
      a.noi_out[slot]     = 0;
      a.crc_ok[slot]      = 1;
    }
  }
  // S = 0: no a-priori information before the first half-iteration
  for (int i = threadIdx.x; i < CPWG * g.s_dw; i += NT) {
    smem[(i / g.s_dw) * g.cb_dw + i % g.s_dw] = 0u;
  }
  const int h_end = (ES && __syncthreads_or(!done) == 0) ? 0 : a.n_end;
#ifdef TDECS_STAMPS
  int passed_at = 0, ran = 0;  // diagnostic: the half-iteration count at which this block passed; the group's count
#endif

#pragma unroll 1
  for (int hi = 0; hi < h_end; hi++) {
    const bool crc_now = ES && hi + 1 >= a.min_iters;  // early-stop check (sch.c:433: from the 2nd)
    for (int i = threadIdx.x; i < CPWG * g.bits_dw; i += NT) {
      smem[(i / g.bits_dw) * g.cb_dw + g.s_dw + g.ck_dw + i % g.bits_dw] = 0u;
    }
    __syncthreads();
    const bool    bits = ES ? crc_now : hi + 1 == h_end;
    constexpr int BM   = ES ? 2 : 1;  // the bit layout (emit)
    if (hi & 1) {
      if (bits) {
        map16s<true, BM>(c, wave, 5 * hi);
      } else {
        map16s<true, 0>(c, wave, 5 * hi);
      }
    } else {
      if (bits) {
        map16s<false, BM>(c, wave, 5 * hi);
      } else {
        map16s<false, 0>(c, wave, 5 * hi);
      }
    }
    __syncthreads();

    // ---------------- DL-SCH early stop: CRC of the hard decision (sch.c:426-456) ----------------
    if constexpr (ES) {
      if (crc_now) {
        const int      nbytes = K / 8;
        const int      bpt    = (nbytes + 2 * NSB - 1) / (2 * NSB);
        const int      b0     = t2 * bpt;
        const int      b1     = min(b0 + bpt, nbytes);
        const bool     crc_a  = a.cbs[cbl].crc_a;
        const uint32_t poly   = crc_a ? LTE_CRC24A : LTE_CRC24B;
        uint32_t       crc    = 0;
#pragma unroll 1
        for (int b = b0; b < b1; b++) {
          crc = crc24_byte(crc, nat_byte(c.BITS, L, Ls, magicL, b), poly);
        }
        uint32_t part = b0 < nbytes ? clmul_mod24(crc, (crc_a ? a.xpow_a : a.xpow_b)[nbytes - b1], poly) : 0;
#pragma unroll
        for (int off = 1; off < NSB; off <<= 1) {
          part ^= (uint32_t)__shfl_xor((int)part, off, 64);
        }
        if (s == 0) {
          RED[wave] = part;
        }
        __syncthreads();
        const bool ok = (RED[0] ^ RED[1]) == 0;
        if (ok && !done && live) {
          const uint32_t slot = a.cbs[cbl].slot;
          uint8_t*       out  = a.out + (size_t)slot * a.out_stride;
          for (int b = t2; b < nbytes; b += 2 * NSB) {
            out[b] = (uint8_t)nat_byte(c.BITS, L, Ls, magicL, b);
          }
          if (t2 == 0) {
            a.noi_out[slot] = (uint8_t)(hi + 1);
            a.crc_ok[slot]  = 1;
          }
        }
#ifdef TDECS_STAMPS
        if (ok && !done) {
          passed_at = hi + 1;
        }
#endif
        done = done || ok;
      }
#ifdef TDECS_STAMPS
      ran = hi + 1;
#endif
      if (__syncthreads_or(!done) == 0) {
        break;  // every block of the workgroup passed its CRC
      }
    }
  }
#ifdef TDECS_STAMPS
  // diagnostic (DL-SCH batches): stamps 56 + block = the half-iterations that block needed (its CRC passed; the limit
  // when it never did), stamp 63 = the half-iterations the workgroup ran (tools/chain_stamps.py)
  if (ES && g_stamps && t2 == 0 && wave == 0) {
    unsigned long long* st = g_stamps + (size_t)blockIdx.x * (blockDim.x >> 6) * 64;
    st[56 + cbw]           = live ? (unsigned long long)(passed_at ? passed_at : h_end) : 0ull;
    if (cbw == 0) {
      st[63] = (unsigned long long)ran;
    }
  }
#endif

  // ---------------- hard decision of the last half-iteration (turbodecoder.c:370-378) ----------------
  if (live && !done && h_end > 0) {
    const int      cbm   = ES ? (int)a.cbs[cbl].slot : cbl;
    uint8_t*       out   = a.out + (size_t)cbm * (ES ? a.out_stride : K / 8);
    for (int b = t2; b < K / 8; b += 2 * NSB) {
      out[b] = ES ? (uint8_t)nat_byte(c.BITS, L, Ls, magicL, b) : reinterpret_cast<const uint8_t*>(c.BITS)[b];
    }
    if (ES && t2 == 0) {
      a.noi_out[cbm] = (uint8_t)a.n_end;
      a.crc_ok[cbm]  = 0;
    }
  }
}

template <bool ES>
__global__ __launch_bounds__(128, 1) void TDECS_K(kernel)(TdecArgs a)
{
  body<ES>(a, blockIdx.x);
}

__global__ __launch_bounds__(128, 1) void TDECS_K(multi_kernel)(const TdecArgs* __restrict__ groups,
                                                            const uint32_t* __restrict__ first, int ngroups)
{
  if constexpr (NSB == 16 && W == 16) {
    // the large sizes of a cut all-188 class are the step's critical path: their waves win the VALU
    // arbitration against the 8-step part and the other classes' waves that share their SIMDs
    // (all-188 step, alternating runs on one box: 11.47-11.53 ms without, 11.16-11.22 ms with; priority 1
    // for the 8-step part as well: 11.24-11.28 ms, gpurun_out r03ad / r03ae)
    __builtin_amdgcn_s_setprio(2);
  }
  const uint32_t b  = blockIdx.x;
  int            lo = 0, hi = ngroups - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (first[mid] <= b) {
      lo = mid;
    } else {
      hi = mid - 1;
    }
  }
  const TdecArgs a = groups[lo];
  body<false>(a, (int)(b - first[lo]));
}

size_t lds_bytes(const TdecArgs& a)
{
  const Geo g = geo((int)a.K, (int)a.Ls, (int)((a.L + W - 1) / W), a.cbs != nullptr);
  return (size_t)CPWG * g.cb_dw * 4;
}

int cpw() { return CPWG; }

hipError_t launch(const TdecArgs& a, hipStream_t stream)
{
  StageScope timing_scope(ST_TDEC, stream);
  const int    grid = (a.ncb + CPWG - 1) / CPWG;
  const size_t lds  = lds_bytes(a);
  tdec_set_last_kernel(a.cbs ? TDECS_NAME "kernel<true>" : TDECS_NAME "kernel<false>");
  if (a.cbs) {
    hipLaunchKernelGGL((TDECS_K(kernel)<true>), dim3(grid), dim3(128), lds, stream, a);
  } else {
    hipLaunchKernelGGL((TDECS_K(kernel)<false>), dim3(grid), dim3(128), lds, stream, a);
  }
  return hipGetLastError();
}

hipError_t multi_launch(const TdecArgs* d_groups, const uint32_t* d_first, int ngroups, uint32_t nblocks, size_t lds,
                        hipStream_t stream)
{
  StageScope timing_scope(ST_TDEC, stream);
  if (ngroups == 0 || nblocks == 0) {
    return hipSuccess;
  }
  tdec_set_last_kernel(TDECS_NAME "multi_kernel");
  hipLaunchKernelGGL(TDECS_K(multi_kernel), dim3(nblocks), dim3(128), lds, stream, d_groups, d_first, ngroups);
  return hipGetLastError();
}

#ifdef TDECS_STAMPS
hipError_t set_stamps(void* d_buf)
{
  unsigned long long* p = (unsigned long long*)d_buf;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &p, sizeof(p));
}
#endif

}  // namespace TDECS_NS
}  // namespace srsran_amd
