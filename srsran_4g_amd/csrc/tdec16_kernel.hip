// srsran_4g_amd/csrc/tdec16_kernel.hip -- LTE turbo decoder for K >= 816 (16 sub-blocks) on CDNA4.
//
// Bit-exact with srsRAN_4G's AVX2 16-bit window decoder (turbodecoder_win.h, WINIMP avx16:
// saturating int16, 16 sub-blocks, 40-step overlap training, normalisation every 2 steps) driven
// by the half-iteration loop of turbodecoder_iter.h:72-144, on the rm_turbo sub-block (SB) input
// layout (rm_turbo.c:260-273).  This is the hot class of the all-188 workload and of every
// DL-SCH / PDSCH code block of K >= 816; tdec_kernel.hip keeps the 8-sub-block and generic
// decoders, the natural input layout and the srsran_tdec_iteration state save/restore.
//
// Mapping -- a LANE PAIR per sub-block:
//   * the 8 trellis states of a sub-block live in two lanes, 4 states each as two packed int16
//     VGPRs.  A step is 9 VALU a lane: 3 v_pk_add_i16 clamp + 2 v_pk_max_i16 on register pairs
//     whose halves are picked by op_sel (the butterflies need no data movement inside a lane),
//     one DPP swap between the two lanes and 2 v_perm_b32 with per-lane selectors.  The state
//     pairing (beta: (0,4)(1,5) | (7,3)(6,2); alpha: (0,1)(2,3) | (6,7)(4,5)) is chosen so both
//     lanes run the same instruction stream and the alpha candidates line up with the betas for
//     the LLR (derivation in DESIGN.md section 4.1).  18 lane-instructions per step and sub-block
//     against 36 for a quad of lanes holding 2 states each (tdec_kernel.hip).
//   * workgroup = 2 waves x 2 code blocks of the same K: wave 0 runs the alpha side, wave 1 the
//     beta side of both blocks (32 lanes per block and side), in the crossover schedule of
//     tdec_kernel.hip (phase 1: alpha over windows [0,h) || beta over [h,M); phase 2: each side
//     recomputes the other direction from LDS checkpoints, W = 16 steps a window, and emits LLRs).
//   * LDS per code block is ONE int16 array S over the soft-buffer slots plus the checkpoints and
//     a decision bitmap (~19 KB at K = 6144, half of tdec_kernel.hip's 40 KB).  S carries the
//     a-priori / extrinsic bookkeeping of the reference's app1/ext1/ext2 buffers in place:
//       DEC1 (even half-iteration) at slot a:  x = sat(syst + S[a]),  y = parity0
//            S[a] <- out1 - S[a]                   (ext1 -= app1, vec_sub: wraps)
//       DEC2 (odd)  at slot a, b = pi-slot(a): x = S[b],  y = parity1
//            S[b] <- out2 - S[b]                   (app1 = ext2 de-interleaved; app1 -= ext1)
//     The hard decision of the half-iteration (ext1 after DEC1, app1 after DEC2:
//     turbodecoder.c:370-378) is the sign of out, ORed into the bitmap as it is produced.
//   * systematic / parity LLRs are not staged: every window loads its W positions straight from
//     the input (L2) one window ahead of use.  Everything runs in one launch for all
//     half-iterations; the DL-SCH variant (ES) adds the CRC early stop of decode_tb_cb
//     (sch.c:426-456) on the bitmap.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc24_dev.h"
#include "stage_timing.h"
#include "tdec_kernel.h"

namespace srsran_amd {
namespace {

typedef short v2s __attribute__((ext_vector_type(2)));

constexpr int   W    = 16;            // window: steps between checkpoints
constexpr int   OVL  = TDEC_OVERLAP;  // win_overlap_len (turbodecoder_win.h:54)
constexpr int   NSB  = 16;            // nof_blocks of the avx16 window decoder
constexpr short NEG  = -10000;        // -INF (turbodecoder_win.h:56)
constexpr int   CPWG = 2;             // code blocks per workgroup

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
#define QP(a, b, c, d) ((a) | ((b) << 2) | ((c) << 4) | ((d) << 6))
template <int CTRL>
__device__ __forceinline__ v2s dpp(v2s a)
{
  return u2v((uint32_t)__builtin_amdgcn_mov_dpp((int)v2u(a), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ v2s pswap(v2s a) { return dpp<QP(1, 0, 3, 2)>(a); }  // the other lane of the pair


// Per-lane v_perm selectors (j = lane & 1).
struct PairSel {
  uint32_t b0, b1;   // beta: new V0 / V1 from (O0, R)
  uint32_t as, ak;   // alpha: the half sent to the other lane / the half kept, from (O0, O1)
};
__device__ __forceinline__ PairSel pair_sel(int j)
{
  PairSel p;
  p.b0 = j ? 0x03020706u : 0x01000504u;  // a: (O0.lo, R.lo)   b: (O0.hi, R.hi)
  p.b1 = j ? 0x01000504u : 0x03020706u;  // a: (O0.hi, R.hi)   b: (O0.lo, R.lo)
  p.as = j ? 0x03020706u : 0x07060302u;  // a: (O0.hi, O1.hi)  b: (O1.hi, O0.hi)
  p.ak = j ? 0x01000504u : 0x05040100u;  // a: (O0.lo, O1.lo)  b: (O1.lo, O0.lo)
  return p;
}

// Trellis state of one sub-block in a lane pair.
struct St {
  v2s v0, v1;
};

// Backward step (turbodecoder_win.h:641-664).  Beta pairing: lane a (b0,b4)(b1,b5), lane b
// (b7,b3)(b6,b2).  O0 = max(V0, swap(V0 + xy)) gives (n0,n1) | (n6,n7); O1 = max(V1 + x,
// swap(V1 + y)) gives (n2,n3) | (n4,n5); the lanes trade O1 and re-pair.
__device__ __forceinline__ St beta_step(St p, v2s xy, const PairSel& ps)
{
  const v2s xys = padd(xy, swp(xy));
  const v2s O0  = pmax(p.v0, swp(padd(p.v0, xys)));
  const v2s O1  = pmax(padd(p.v1, lo2(xy)), swp(padd(p.v1, hi2(xy))));
  const v2s R   = pswap(O1);
  return St{perm(O0, R, ps.b0), perm(O0, R, ps.b1)};
}

// Forward candidates (turbodecoder_win.h:767-785): c0 = bit-0 (m_b), c1 = bit-1 (new) metrics
// of the destination states, paired as the betas.  Alpha pairing: lane a (a0,a1)(a2,a3),
// lane b (a6,a7)(a4,a5).
struct Cand {
  v2s c00, c10, c01, c11;  // c0 / c1 of pair 0 and pair 1
};
__device__ __forceinline__ Cand alpha_cand(St p, v2s xy)
{
  const v2s xys = padd(xy, swp(xy));
  Cand      c;
  c.c00 = p.v0;
  c.c10 = padd(swp(p.v0), xys);
  c.c01 = padd(swp(p.v1), hi2(xy));
  c.c11 = padd(p.v1, lo2(xy));
  return c;
}
__device__ __forceinline__ St alpha_next(const Cand& c, const PairSel& ps)
{
  const v2s O0 = pmax(c.c00, c.c10);  // a: (s0,s4)  b: (s7,s3)
  const v2s O1 = pmax(c.c01, c.c11);  // a: (s1,s5)  b: (s6,s2)
  return St{perm(O1, O0, ps.ak), pswap(perm(O1, O0, ps.as))};
}

// LLR = max_s(beta + c1) - max_s(beta + c0) over the 8 states (turbodecoder_win.h:788-815).
__device__ __forceinline__ short llr_out(St b, const Cand& c)
{
  const v2s m0 = pmax(padd(b.v0, c.c00), padd(b.v1, c.c01));
  const v2s m1 = pmax(padd(b.v0, c.c10), padd(b.v1, c.c11));
  v2s       r  = pmax(perm(m1, m0, 0x05040100u), perm(m1, m0, 0x07060302u));  // (max0, max1) of the lane
  r            = pmax(r, pswap(r));
  return psub(swp(r), r).x;
}

// normalize() (turbodecoder_win.h:480-498): subtract state 0 (lane a, V0.lo in both pairings).
__device__ __forceinline__ St norm(St p)
{
  const v2s z = lo2(dpp<QP(0, 0, 2, 2)>(p.v0));
  return St{psub(p.v0, z), psub(p.v1, z)};
}
__device__ __forceinline__ bool norm_at(int k) { return (k & 1) == 0 && k != 0; }  // normalize_period 2

__device__ __forceinline__ St neg_state() { return St{v2s{NEG, NEG}, v2s{NEG, NEG}}; }
__device__ __forceinline__ St alpha_known(int j) { return j ? neg_state() : St{v2s{0, NEG}, v2s{NEG, NEG}}; }

// beta_trellis (turbodecoder_win.h:500-548): the tail steps K+2..K of the last sub-block,
// non-saturating (sadd without use_saturated_add).
__device__ __forceinline__ St trellis_pair(const short* xt, const short* yt, int j)
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
  return j ? St{v2s{o[7], o[3]}, v2s{o[6], o[2]}} : St{v2s{o[0], o[4]}, v2s{o[1], o[5]}};
}

__device__ __forceinline__ uint32_t ck_word(int m, int l32) { return (uint32_t)(m * 32 + l32) * 2; }

// LDS of one code block (dwords): S [16*Ls int16] | CK [M*32 lanes*8 B] | BITS [K/8 B] | RED [2]
struct Geo16 {
  int s_dw, ck_dw, bits_dw, cb_dw;
};
__host__ __device__ __forceinline__ Geo16 geo16(int K, int Ls, int M)
{
  Geo16 g;
  g.s_dw    = (NSB * Ls + 1) / 2;
  g.ck_dw   = M * 64;
  g.bits_dw = (K / 8 + 3) / 4;
  g.cb_dw   = g.s_dw + g.ck_dw + g.bits_dw + 2;
  return g;
}

// One window of W inputs of this lane's sub-block, as loaded from global memory (zero-extended:
// the packing into (x, y) happens when the window starts, so the loads of the next window can be
// in flight meanwhile).
struct Raw {
  uint32_t a[W];  // systematic LLR (DEC1) / slot of pi(position) (DEC2)
  uint32_t b[W];  // parity0 / parity1
};

// Global loads through buffer resources: (uniform descriptor) + (per-lane 32-bit offset) +
// (uniform window offset) + immediate, so a window costs no address arithmetic; the range check of
// the descriptor turns reads past the block's buffer (the last, partial window) into zeros.
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

// Per-lane context of one half-iteration.
struct Lane16 {
  int      wave, l32, s, j, K, L, Ls, M, KP;
  uint32_t magicLs;
  rsrc_t   rin;   // the workgroup's blocks' inputs, from the lower of the two
  uint32_t voff;  // bytes from rin's base to this lane's first position (q = s) of its block
  rsrc_t   rtf;   // tfwd (q order, SB input: slot of pi(n(q))), K entries
  lshort   S;     // this block's S (LDS)
  lshort   Ssb;   // S + s * Ls: this lane's sub-block
  uint32_t* CK;   // this block's checkpoints (LDS)
  uint32_t* BITS; // this block's decision bitmap (LDS)
  PairSel  ps;
};

// Inputs of the window at t0 of this lane's sub-block (q = k*16 + s in the SB layout): DEC1 loads
// systematic + parity0, DEC2 the pi slot + parity1.  Positions past the sub-block (the last,
// partial window) load a neighbour's value or, past the buffer, zero; they are never used.
template <bool D2>
__device__ __forceinline__ void issue(const Lane16& c, Raw& r, int t0)
{
  const uint32_t soff = 32u * (uint32_t)t0;
  const uint32_t poff = soff + (D2 ? 4u : 2u) * (uint32_t)c.KP;  // parity stream, bytes
#pragma unroll
  for (int i = 0; i < W; i++) {
    r.a[i] = D2 ? ldb(c.rtf, 2u * (uint32_t)c.s, soff, 32 * i) : ldb(c.rin, c.voff, soff, 32 * i);
    r.b[i] = ldb(c.rin, c.voff, poff, 32 * i);
  }
}

// The packed branch input of a position stays one register: an opaque move after packing keeps
// the compiler from re-deriving it from the two halves at every use.
__device__ __forceinline__ uint32_t pin(uint32_t v)
{
  asm volatile("" : "+v"(v));
  return v;
}

// The LLR o of position k: S update (vec_sub, wraps) and, when the half-iteration's decision is
// needed, its bit (turbodecoder.c:370-378: the sign of ext1 after DEC1, of app1 after DEC2).
// DEC1 writes slot s*Ls + k and decides bit n = s*L + k; DEC2 writes the pi slot b (aux = its LDS
// address, x = the ext1 read there) and decides the natural position of b.
template <bool D2, bool BITS>
__device__ __forceinline__ void emit(const Lane16& c, int k, short o, uint32_t aux, uint32_t xw)
{
  int n;
  if (D2) {
    const lshort p = (lshort)(size_t)aux;
    *p             = (short)(o - (short)(xw & 0xffffu));
    if (BITS) {
      const int slot = (int)(p - c.S);
      const int sb   = (int)__umulhi((uint32_t)slot, c.magicLs);
      n              = slot - sb * (c.Ls - c.L);
    }
  } else {
    c.Ssb[k] = (short)(o - (short)aux);
    n        = c.s * c.L + k;
  }
  if (BITS) {
    atomicOr(&c.BITS[n >> 5], (uint32_t)(o > 0) << (((n >> 3) & 3) * 8 + 7 - (n & 7)));
  }
}

// normalize_period 2 on the absolute position k = t0 + i of a window (t0 a multiple of W): every
// even position except k = 0; only i = 0 depends on the window.
__device__ __forceinline__ bool nrm(int t0, int i) { return (i & 1) == 0 && (i != 0 || t0 != 0); }

// Phase-2 alpha side, window at t0 >= W (alpha_window of tdec_kernel.hip): beta[t0+1 .. cc]
// recomputed from the stored beta at cc = min(t0 + W, L) (checkpoint), then alpha + LLR of
// t0 .. cc-1.
template <bool D2, bool BITS, bool FULL>
__device__ __forceinline__ St alpha_llr_window(const Lane16& c, St P, int t0, St Pb, const uint32_t* xw,
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
      Pb    = beta_step(Pb, u2v(xw[i + 1]), c.ps);
      bw[i] = Pb;
      if (FULL ? (i & 1) : norm_at(t0 + 1 + i)) Pb = norm(Pb);
    }
  }
#pragma unroll
  for (int i = 0; i < W; i++) {
    if (FULL || t0 + i < L) {
      const Cand  cd = alpha_cand(P, u2v(xw[i]));
      const short o  = llr_out(bw[i], cd);
      P              = alpha_next(cd, c.ps);
      if ((i & 1) == 0) P = norm(P);  // t0 >= W: every even position
      emit<D2, BITS>(c, t0 + i, o, aux[i], xw[i]);
    }
  }
  return P;
}

// Phase-1 beta side, window at t0 >= W: backward over t0+W-1 .. t0 (FULL) or L-1 .. t0; Bst = the
// stored beta at t0, which is the checkpoint of window t0/W - 1 when `store`.
template <bool FULL>
__device__ __forceinline__ St beta_window(const Lane16& c, St P, int t0, bool store, St& Bst, const uint32_t* xw)
{
#pragma unroll
  for (int i = W - 1; i >= 0; i--) {
    if (FULL || t0 + i < c.L) {
      P = beta_step(P, u2v(xw[i]), c.ps);
      if (i == 0) {
        Bst = P;
        if (store) {
          *reinterpret_cast<uint2*>(&c.CK[ck_word(t0 / W - 1, c.l32)]) = make_uint2(v2u(P.v0), v2u(P.v1));
        }
      }
      if ((i & 1) == 0) P = norm(P);
    }
  }
  return P;
}

// The window inputs of one side, prefetched along the side's window sequence:
//   alpha side: training [L-40, L-24), [L-24, L-8), [L-8, L); then windows 0, 1, ..., Ma-1
//   beta side:  training [32, 40), [16, 32), [0, 16);       then windows Ma-1, ..., 1, 0
// The global loads of window idx + 1 are issued when window idx starts (a whole window of compute
// to arrive); DEC1's LDS reads of S (addresses known in advance) go with them.  DEC2's S gathers
// need the pi slots of the window itself: they are issued when it starts, just before the next
// window's global loads, which cover their latency.  Reading S ahead of use is safe: within a
// half-iteration a position's S is written only by the side that emits its LLR, after that side
// has read it, and no position is read again later.
template <bool D2>
struct Pipe16 {
  Raw      g;      // global loads of the next window (in flight)
  uint32_t dv[W];  // DEC1: its S values (in flight)
  int      nwin, Ma;
  bool     beta;

  __device__ __forceinline__ int t0_of(int idx, int L) const
  {
    if (beta) {
      return idx < 3 ? 2 * W - W * idx : (Ma - 1 - (idx - 3)) * W;
    }
    return idx < 3 ? L - OVL + W * idx : (idx - 3) * W;
  }

  __device__ __forceinline__ void load(const Lane16& c, int idx)
  {
    if (idx < nwin) {
      const int t0 = t0_of(idx, c.L);
      issue<D2>(c, g, t0);
      if (!D2) {  // S of the window's positions; past the sub-block: a neighbour's slot (unused)
#pragma unroll
        for (int i = 0; i < W; i++) {
          dv[i] = (uint16_t)c.Ssb[t0 + i];
        }
      }
    }
  }
  __device__ __forceinline__ void start(const Lane16& c) { load(c, 0); }
  // window idx begins: its packed (x, y) and output aux; the loads of idx + 1 are issued.
  //   DEC1: xw = (sat(syst + S[a]), parity0), aux = S[a]
  //   DEC2: xw = (S[b], parity1), aux = LDS address of S[b]
  __device__ __forceinline__ void next(const Lane16& c, int idx, uint32_t* xw, uint32_t* aux)
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
// BITS: the half-iteration's hard decision is recorded (early stop / the last half-iteration).
template <bool D2, bool BITS>
__device__ __forceinline__ void map16(const Lane16& cin)
{
  // Opaque copy of the per-lane sub-block index: every window address derives from it, so none
  // can be hoisted out of the half-iteration loop (LICM would keep hundreds of addresses live
  // across it and spill).
  Lane16 c = cin;
  asm volatile("" : "+v"(c.s));
  asm volatile("" : "+v"(c.voff));
  {
    uint32_t ssb = (uint32_t)(size_t)c.Ssb;
    asm volatile("" : "+v"(ssb));
    c.Ssb = (lshort)(size_t)ssb;
  }
  const int L     = c.L;
  const int Mfull = L / W;            // windows entirely below L
  const int Ma    = (L + W - 1) / W;  // = c.M
  const int h     = max(1, min((L + W) / (2 * W), L / W));
  const PairSel& ps = c.ps;
  Pipe16<D2> pp;
  pp.nwin = 3 + Ma;
  pp.Ma   = Ma;
  pp.beta = __builtin_amdgcn_readfirstlane(c.wave) != 0;  // wave-uniform: window offsets stay scalar
  uint32_t xw[W];
  uint32_t aux[W];
  pp.start(c);
  if (c.wave == 0) {
    // ================= alpha side =================
    St P = neg_state();
    // training over the last 40 steps of the own sub-block (win.h:747-756)
    pp.next(c, 0, xw, aux);
#pragma unroll
    for (int i = 0; i < W; i++) {
      P = alpha_next(alpha_cand(P, u2v(xw[i])), ps);
      if (norm_at(i)) P = norm(P);
    }
    pp.next(c, 1, xw, aux);
#pragma unroll
    for (int i = 0; i < W; i++) {
      P = alpha_next(alpha_cand(P, u2v(xw[i])), ps);
      if (norm_at(W + i)) P = norm(P);
    }
    pp.next(c, 2, xw, aux);
#pragma unroll
    for (int i = 0; i < OVL - 2 * W; i++) {
      P = alpha_next(alpha_cand(P, u2v(xw[i])), ps);
      if (norm_at(2 * W + i)) P = norm(P);
    }
    {  // move_left: sub-block s starts from the training state of s - 1; s = 0 is known
      St q;
      q.v0 = u2v((uint32_t)__shfl_up((int)v2u(P.v0), 2, 64));
      q.v1 = u2v((uint32_t)__shfl_up((int)v2u(P.v1), 2, 64));
      P    = c.s == 0 ? alpha_known(c.j) : q;
    }
    // phase 1: windows [0, h) (all full), entry checkpoints in slots 0..h-1
#pragma unroll 1
    for (int ma = 0; ma < h; ma++) {
      const int t0 = ma * W;
      pp.next(c, 3 + ma, xw, aux);
      *reinterpret_cast<uint2*>(&c.CK[ck_word(ma, c.l32)]) = make_uint2(v2u(P.v0), v2u(P.v1));
#pragma unroll
      for (int i = 0; i < W; i++) {
        P = alpha_next(alpha_cand(P, u2v(xw[i])), ps);
        if (nrm(t0, i)) P = norm(P);
      }
    }
    __syncthreads();
    // phase 2: windows [h, Ma): beta recomputed from the checkpoint above the window, then
    // alpha + LLR; the last window may be partial
    // (the partial window is peeled so the loop body stays one straight-line block)
#pragma unroll 1
    for (int ma = h; ma < Mfull; ma++) {
      pp.next(c, 3 + ma, xw, aux);
      const uint2 ckv = *reinterpret_cast<const uint2*>(&c.CK[ck_word(ma, c.l32)]);
      P = alpha_llr_window<D2, BITS, true>(c, P, ma * W, St{u2v(ckv.x), u2v(ckv.y)}, xw, aux);
    }
    if (Ma > Mfull) {
      pp.next(c, 3 + Mfull, xw, aux);
      const uint2 ckv = *reinterpret_cast<const uint2*>(&c.CK[ck_word(Mfull, c.l32)]);
      alpha_llr_window<D2, BITS, false>(c, P, Mfull * W, St{u2v(ckv.x), u2v(ckv.y)}, xw, aux);
    }
  } else {
    // ================= beta side =================
    St P = neg_state();
    // training over the first 40 steps of the own sub-block, backwards (win.h:622-630)
    pp.next(c, 0, xw, aux);
#pragma unroll
    for (int i = OVL - 2 * W - 1; i >= 0; i--) {
      P = beta_step(P, u2v(xw[i]), ps);
      if (norm_at(2 * W + i)) P = norm(P);
    }
    pp.next(c, 1, xw, aux);
#pragma unroll
    for (int i = W - 1; i >= 0; i--) {
      P = beta_step(P, u2v(xw[i]), ps);
      if (norm_at(W + i)) P = norm(P);
    }
    pp.next(c, 2, xw, aux);
#pragma unroll
    for (int i = W - 1; i >= 0; i--) {
      P = beta_step(P, u2v(xw[i]), ps);
      if (norm_at(i)) P = norm(P);
    }
    {  // move_right: sub-block s starts from the training state of s + 1; the last from the tail
      St q;
      q.v0 = u2v((uint32_t)__shfl_down((int)v2u(P.v0), 2, 64));
      q.v1 = u2v((uint32_t)__shfl_down((int)v2u(P.v1), 2, 64));
      if (c.s == NSB - 1) {  // trellis termination: systematic / parity0 (DEC1), app2 / parity1 (DEC2)
        const int tail = 6 * c.KP + (D2 ? 12 : 0);  // bytes
        short     xt[3], yt[3];
#pragma unroll
        for (int t = 0; t < 3; t++) {
          xt[t] = (short)ldb(c.rin, c.voff - 2 * c.s, tail, 4 * t);
          yt[t] = (short)ldb(c.rin, c.voff - 2 * c.s, tail, 4 * t + 2);
        }
        P = trellis_pair(xt, yt, c.j);
      } else {
        P = q;
      }
    }
    const int mtop = Ma - 1;
    *reinterpret_cast<uint2*>(&c.CK[ck_word(mtop, c.l32)]) = make_uint2(v2u(P.v0), v2u(P.v1));  // beta[L]
    St Bst = P;  // stored (pre-normalisation) beta of the position above the current window
    // phase 1: windows [h, Ma) from the top (the top one maybe partial); the stored beta at the
    // start of window mb is the checkpoint of window mb - 1 (slot mb - 1) for mb > h
    // (the partial top window is peeled so the loop body stays one straight-line block)
    if (Ma > Mfull) {
      pp.next(c, 3, xw, aux);
      P = beta_window<false>(c, P, mtop * W, mtop > h, Bst, xw);
    }
#pragma unroll 1
    for (int mb = Mfull - 1; mb >= h; mb--) {
      pp.next(c, 3 + mtop - mb, xw, aux);
      P = beta_window<true>(c, P, mb * W, mb > h, Bst, xw);
    }
    __syncthreads();
    // phase 2: windows [0, h) from the top: alpha recomputed from the entry checkpoint, then
    // beta backwards with the LLR of every position (beta_llr_window of tdec_kernel.hip)
#pragma unroll 1
    for (int mb = h - 1; mb >= 0; mb--) {
      const int t0 = mb * W;
      pp.next(c, 3 + mtop - mb, xw, aux);
      const uint2 cka = *reinterpret_cast<const uint2*>(&c.CK[ck_word(mb, c.l32)]);
      St          Pa{u2v(cka.x), u2v(cka.y)};
      St          aw[W];  // alpha entering each position (candidates rebuilt at LLR time)
#pragma unroll
      for (int i = 0; i < W; i++) {
        aw[i] = Pa;
        if (i < W - 1) {
          Pa = alpha_next(alpha_cand(Pa, u2v(xw[i])), ps);
          if (nrm(t0, i)) Pa = norm(Pa);
        }
      }
#pragma unroll
      for (int i = W - 1; i >= 0; i--) {
        const short o = llr_out(Bst, alpha_cand(aw[i], u2v(xw[i])));
        P             = beta_step(P, u2v(xw[i]), ps);
        Bst           = P;
        if (nrm(t0, i)) P = norm(P);
        emit<D2, BITS>(c, t0 + i, o, aux[i], xw[i]);
      }
    }
  }
}

}  // namespace

template <bool ES>
__device__ __forceinline__ void tdec16_body(const TdecArgs& a, int bid)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int cbw  = lane >> 5;         // block of the workgroup
  const int l32  = lane & 31;         // lane within the block's side
  const int t2   = wave * 32 + l32;   // thread within the block (both sides), 0..63
  const int K    = (int)a.K;
  const int L    = (int)a.L;
  const int Ls   = (int)a.Ls;
  const int M    = (L + W - 1) / W;
  const Geo16 g  = geo16(K, Ls, M);
  const int cb   = bid * CPWG + cbw;
  const int cbl  = cb < (int)a.ncb ? cb : (int)a.ncb - 1;
  const bool live = cb < (int)a.ncb && (!ES || a.cbs[cbl].slot != TDEC_PAD_SLOT);
  bool done      = ES && (!live || *a.cbs[cbl].skip);

  uint32_t* base = smem + cbw * g.cb_dw;
  Lane16    c;
  c.wave    = wave;
  c.l32     = l32;
  c.s       = l32 >> 1;
  c.j       = l32 & 1;
  c.K       = K;
  c.L       = L;
  c.Ls      = Ls;
  c.M       = M;
  c.KP      = K + 32;  // SB stream stride (rm_turbo.c:260-273)
  c.magicLs = a.magicLs;
  // the workgroup's two blocks read through one uniform base: the lower of their inputs (plain
  // launches: in_stride apart; DL-SCH: the host pads the descriptor list so that the two blocks of
  // every workgroup lie within TDEC_PAIR_SPAN, tdec_pair_cbs)
  const int cb0 = bid * CPWG;
  size_t    in_lane, in_base, in_hi;
  if (ES) {
    const size_t p0 = (size_t)a.cbs[min(cb0, (int)a.ncb - 1)].in;
    const size_t p1 = (size_t)a.cbs[min(cb0 + 1, (int)a.ncb - 1)].in;
    in_base         = min(p0, p1);
    in_hi           = max(p0, p1);
    in_lane         = (size_t)a.cbs[cbl].in;
  } else {
    in_base = (size_t)(a.in + (size_t)min(cb0, (int)a.ncb - 1) * a.in_stride);
    in_hi   = (size_t)(a.in + (size_t)min(cb0 + 1, (int)a.ncb - 1) * a.in_stride);
    in_lane = (size_t)(a.in + (size_t)cbl * a.in_stride);
  }
  const uint32_t cb_bytes = (uint32_t)(3 * c.KP + 12) * 2;  // one block's soft-buffer input
  c.rin  = make_rsrc((const void*)in_base, (uint32_t)(in_hi - in_base) + cb_bytes);
  c.voff = (uint32_t)(in_lane - in_base) + 2 * c.s;
  c.rtf  = make_rsrc(a.tfwd, 2u * (uint32_t)K);
  c.S    = (lshort)(short*)base;
  c.Ssb  = c.S + c.s * Ls;
  c.CK   = base + g.s_dw;
  c.BITS = c.CK + g.ck_dw;
  c.ps   = pair_sel(c.j);
  uint32_t* RED = c.BITS + g.bits_dw;

  if constexpr (ES) {
    if (live && done && t2 == 0) {  // skipped block (sch.c:392, 476-480)
      const uint32_t slot = a.cbs[cbl].slot;
      a.noi_out[slot]     = 0;
      a.crc_ok[slot]      = 1;
    }
  }
  // S = 0: no a-priori information before the first half-iteration
  for (int i = threadIdx.x; i < CPWG * g.s_dw; i += 128) {
    smem[(i / g.s_dw) * g.cb_dw + i % g.s_dw] = 0u;
  }
  const int h_end = (ES && __syncthreads_or(!done) == 0) ? 0 : a.n_end;

#pragma unroll 1
  for (int hi = 0; hi < h_end; hi++) {
    const bool crc_now = ES && hi + 1 >= a.min_iters;  // early-stop check (sch.c:433: from the 2nd)
    for (int i = threadIdx.x; i < CPWG * g.bits_dw; i += 128) {
      smem[(i / g.bits_dw) * g.cb_dw + g.s_dw + g.ck_dw + i % g.bits_dw] = 0u;
    }
    __syncthreads();
    // decisions: every half-iteration the early stop checks, else only the last one
    const bool bits = ES ? crc_now : hi + 1 == h_end;
    if (hi & 1) {
      if (bits) {
        map16<true, true>(c);
      } else {
        map16<true, false>(c);
      }
    } else {
      if (bits) {
        map16<false, true>(c);
      } else {
        map16<false, false>(c);
      }
    }
    __syncthreads();

    // ---------------- DL-SCH early stop: CRC of the hard decision (sch.c:426-456) ----------------
    if constexpr (ES) {
      if (crc_now) {
        const uint8_t* bytes  = reinterpret_cast<const uint8_t*>(c.BITS);
        const int      nbytes = K / 8;
        const int      bpt    = (nbytes + 63) / 64;
        const int      b0     = t2 * bpt;
        const int      b1     = min(b0 + bpt, nbytes);
        const bool     crc_a  = a.cbs[cbl].crc_a;
        const uint32_t poly   = crc_a ? LTE_CRC24A : LTE_CRC24B;
        uint32_t       crc    = 0;
#pragma unroll 1
        for (int b = b0; b < b1; b++) {
          crc = crc24_byte(crc, bytes[b], poly);
        }
        uint32_t part = b0 < nbytes ? clmul_mod24(crc, (crc_a ? a.xpow_a : a.xpow_b)[nbytes - b1], poly) : 0;
#pragma unroll
        for (int off = 1; off < 32; off <<= 1) {
          part ^= (uint32_t)__shfl_xor((int)part, off, 64);
        }
        if (l32 == 0) {
          RED[wave] = part;
        }
        __syncthreads();
        const bool ok = (RED[0] ^ RED[1]) == 0;
        if (ok && !done && live) {
          const uint32_t slot = a.cbs[cbl].slot;
          uint8_t*       out  = a.out + (size_t)slot * a.out_stride;
          for (int b = t2; b < nbytes; b += 64) {
            out[b] = bytes[b];
          }
          if (t2 == 0) {
            a.noi_out[slot] = (uint8_t)(hi + 1);
            a.crc_ok[slot]  = 1;
          }
        }
        done = done || ok;
      }
      if (__syncthreads_or(!done) == 0) {
        break;  // both blocks of the workgroup passed their CRC
      }
    }
  }

  // ---------------- hard decision of the last half-iteration (turbodecoder.c:370-378) ----------------
  if (live && !done && h_end > 0) {
    const int      cbm   = ES ? (int)a.cbs[cbl].slot : cbl;
    uint8_t*       out   = a.out + (size_t)cbm * (ES ? a.out_stride : K / 8);
    const uint8_t* bytes = reinterpret_cast<const uint8_t*>(c.BITS);
    for (int b = t2; b < K / 8; b += 64) {
      out[b] = bytes[b];
    }
    if (ES && t2 == 0) {
      a.noi_out[cbm] = (uint8_t)a.n_end;
      a.crc_ok[cbm]  = 0;
    }
  }
}

template <bool ES>
__global__ __launch_bounds__(128, 2) void tdec16_kernel(TdecArgs a)
{
  tdec16_body<ES>(a, blockIdx.x);
}

// Several sizes of the class in one launch (tdec_multi_kernel of tdec_kernel.hip): workgroup b
// belongs to the group g with first[g] <= b < first[g + 1].
__global__ __launch_bounds__(128, 2) void tdec16_multi_kernel(const TdecArgs* __restrict__ groups,
                                                           const uint32_t* __restrict__ first, int ngroups)
{
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
  tdec16_body<false>(a, (int)(b - first[lo]));
}

// Which 16-sub-block decoder a launch of n blocks gets (K = 6144, 8 half-iterations, ms per launch,
// gpurun_out r03d -> profiles/r03_tdec_kernels.jsonl):
//      n      quad (tdec_kernel<16>)   lane pair (tdec16_kernel)   single lane (tdec16s_kernel)
//    256            0.258                    0.275                        0.344
//    512            0.339                    0.282                        0.348
//   1024            0.403                    0.394                        0.362
//   2048            0.766                    0.457                        0.382
// The quad decoder (one block a workgroup) fills the chip best below ~512 blocks, the lane pair between,
// and the single-lane decoder (64 lanes a wave on 4 blocks, the densest mapping) from 1024 on.
// srsran_tdec_gpu_set_pair_threshold() / _single_threshold() move the thresholds (tests force each
// kernel onto small batches with 0).
static uint32_t g_pair_min_cb = 512u;
void     tdec16_set_min_cb(uint32_t n) { __atomic_store_n(&g_pair_min_cb, n, __ATOMIC_RELAXED); }
uint32_t tdec16_min_cb() { return __atomic_load_n(&g_pair_min_cb, __ATOMIC_RELAXED); }
bool     tdec16_pays(uint32_t ncb) { return ncb >= tdec16_min_cb(); }
// srsran_tdec_gpu_set_single_threshold(): blocks a launch from which the single-lane decoders
// (tdecs_kernel.hip, 16-sub-block class) replaces the lane pair.  Between 512 and 1024 blocks
// (K = 6144, gpurun_out r03af): single lane / lane pair 0.345 / 0.385 ms at 640, 0.349 / 0.390 at 768,
// 0.359 / 0.394 at 896, 0.361 / 0.397 at 1014 (the PUSCH batch of 78 UEs x 13 blocks: 0.108 vs 0.113 ms
// with early stop); the lane pair is ahead at 512 (0.282 vs 0.348): from 576 blocks.
static uint32_t g_single_min_cb = 576u;
void     tdec16s_set_min_cb(uint32_t n) { __atomic_store_n(&g_single_min_cb, n, __ATOMIC_RELAXED); }
uint32_t tdec16s_min_cb() { return __atomic_load_n(&g_single_min_cb, __ATOMIC_RELAXED); }
// The 8-sub-block class: its quad decoder (one block a workgroup) stays ahead up to ~1024 blocks a launch
// (K = 512: 0.060 vs 0.085 ms at 512, 0.081 vs 0.086 ms at 1024) and the single-lane decoder is ahead on
// the fused class launch (32 sizes x 256 = 8192 blocks: 0.30 vs 0.53 ms): from 4096 blocks by default.
static uint32_t g_single8_min_cb = 4096u;
// srsran_tdec_gpu_set_w8_max_k(): single-lane launches whose block sizes are all <= this K use the build
// with 8-step windows (tdecs_kernel.hip, TDECS_W = 8: 164-191 VGPRs, two waves a SIMD where LDS allows).
// Default 800 = the whole 8-sub-block class (408 <= K <= 800), where it wins: the fused class launch of
// 32 sizes x 1024 blocks 0.71 vs 0.91 ms, x 4096 blocks 2.30 vs 3.39 ms (gpurun_out r03l).  The 16-sub-block
// class keeps 16-step windows: its 8-step build is slower at every K measured (2048 blocks, K = 1024 / 2048
// / 4096 / 6144: 0.129 / 0.219 / 0.395 / 0.738 ms against 0.096 / 0.153 / 0.268 / 0.380 ms): twice the
// windows a sub-block for the same training overlap, and at 19 KB of LDS a block the second wave a
// SIMD does not fit at large K anyway.
static uint32_t g_w8_max_k = 800u;
// srsran_tdec_gpu_set_w8_fused_max_k(): in a fused multi-size launch of the 16-sub-block single-lane class,
// the sizes up to this K form their own launch on the 8-step-window build (their workgroups, at 164-191
// registers and little LDS, share SIMDs with the large sizes' workgroups).  All-188 step, one box,
// alternating runs (gpurun_out r03z): cut at 800 (none) 12.22 ms, 1536 11.65 ms, 2368 11.71-11.73 ms,
// 3136 12.37 ms.  With the 16-step part cut again at SRSRAN_AMD_TDEC_MIDCUT = 3072 (r06v, one box, alternating):
// 1024 10.95 ms, 1536 10.615 / 10.621 ms, 1792 10.68 ms, 2048 10.686 / 10.71 ms, 2560 11.34 ms.
static uint32_t g_w8_fused_max_k = 1536u;
void     tdecs_set_w8_fused_max_k(uint32_t k) { __atomic_store_n(&g_w8_fused_max_k, k, __ATOMIC_RELAXED); }
uint32_t tdecs_w8_fused_max_k() { return __atomic_load_n(&g_w8_fused_max_k, __ATOMIC_RELAXED); }
void     tdecs_set_w8_max_k(uint32_t k) { __atomic_store_n(&g_w8_max_k, k, __ATOMIC_RELAXED); }
uint32_t tdecs_w8_max_k() { return __atomic_load_n(&g_w8_max_k, __ATOMIC_RELAXED); }
void     tdec8s_set_min_cb(uint32_t n) { __atomic_store_n(&g_single8_min_cb, n, __ATOMIC_RELAXED); }
uint32_t tdec8s_min_cb() { return __atomic_load_n(&g_single8_min_cb, __ATOMIC_RELAXED); }
// srsran_tdec_gpu_set_generic_single_threshold(): the generic class (K <= 400) keeps tdec_kernel.hip's
// quad decoder by default: one lane per block and direction runs the whole K-step recursion serially, and
// at 1024 blocks per size (47104 blocks) tdec1s_kernel takes 1.47 ms against the quad decoder's 0.78 ms
// (profiles/r03_tdec_kernels.jsonl), so tdec1s is selected only when a caller lowers this threshold.
static uint32_t g_single1_min_cb = 0xffffffffu;
void     tdec1s_set_min_cb(uint32_t n) { __atomic_store_n(&g_single1_min_cb, n, __ATOMIC_RELAXED); }
uint32_t tdec1s_min_cb() { return __atomic_load_n(&g_single1_min_cb, __ATOMIC_RELAXED); }
int      tdec16_choice(uint32_t ncb) { return ncb >= tdec16s_min_cb() ? 2 : tdec16_pays(ncb) ? 1 : 0; }

bool tdec16_eligible(int nsb, const TdecArgs& a)
{
  return nsb == 16 && a.layout_sb && a.n_start == 0 && a.state == nullptr && a.L >= (uint32_t)OVL &&
         tdec16_choice(a.ncb) > 0;
}

bool tdec8s_eligible(int nsb, const TdecArgs& a)
{
  return nsb == 8 && a.layout_sb && a.n_start == 0 && a.state == nullptr && a.L >= (uint32_t)OVL &&
         a.ncb >= tdec8s_min_cb();
}

bool tdec1s_eligible(int nsb, const TdecArgs& a)
{
  return nsb == 1 && a.n_start == 0 && a.state == nullptr && a.ncb >= tdec1s_min_cb();
}

size_t tdec16_lds_bytes(const TdecArgs& a)
{
  const Geo16 g = geo16((int)a.K, (int)a.Ls, (int)((a.L + W - 1) / W));
  return (size_t)CPWG * g.cb_dw * 4;
}

int tdec16_cpw() { return CPWG; }

hipError_t tdec16_launch(const TdecArgs& a, hipStream_t stream)
{
  StageScope timing_scope(ST_TDEC, stream);
  const int    grid = (a.ncb + CPWG - 1) / CPWG;
  const size_t lds  = tdec16_lds_bytes(a);
  tdec_set_last_kernel(a.cbs ? "tdec16_kernel<true>" : "tdec16_kernel<false>");
  if (a.cbs) {
    hipLaunchKernelGGL((tdec16_kernel<true>), dim3(grid), dim3(128), lds, stream, a);
  } else {
    hipLaunchKernelGGL((tdec16_kernel<false>), dim3(grid), dim3(128), lds, stream, a);
  }
  return hipGetLastError();
}

hipError_t tdec16_multi_launch(const TdecArgs* d_groups, const uint32_t* d_first, int ngroups, uint32_t nblocks,
                               size_t lds, hipStream_t stream)
{
  StageScope timing_scope(ST_TDEC, stream);
  if (ngroups == 0 || nblocks == 0) {
    return hipSuccess;
  }
  tdec_set_last_kernel("tdec16_multi_kernel");
  hipLaunchKernelGGL(tdec16_multi_kernel, dim3(nblocks), dim3(128), lds, stream, d_groups, d_first, ngroups);
  return hipGetLastError();
}

}  // namespace srsran_amd
