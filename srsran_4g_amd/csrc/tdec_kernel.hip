// srsran_4g_amd/csrc/tdec_kernel.hip -- LTE turbo decoder for CDNA4 (gfx950).
//
// Bit-exact with srsRAN_4G's AUTO 16-bit turbo decoder (AVX2 build):
//   K <= 400           generic max-log-MAP, int16 wrap        (turbodecoder_gen.c:58-236)
//   408 <= K <= 800    8-sub-block sliding window, saturating (turbodecoder_win.h, SSE16)
//   K >= 816           16-sub-block sliding window, saturating (turbodecoder_win.h, AVX16)
// dispatch: turbodecoder.c:381-408; half-iteration driver: turbodecoder_iter.h:72-144.
//
// Mapping (two wave64 per workgroup, wave 0 = alpha side, wave 1 = beta side):
//   * a code block's sub-block s is served by a QUAD of lanes; lane j of the quad
//     holds trellis states (2j, 2j+1) packed as two int16 in one VGPR.  Each trellis
//     step is ~6 packed VALU ops per lane: two DPP quad_perm reads fetch the source
//     states, v_perm_b32 (per-lane selector) arranges them, v_pk_add_i16 (clamp)
//     adds the branch metrics, v_pk_max_i16 selects.
//   * NSB=16: one CB per wave (16 quads); NSB=8: two CBs; generic (NSB=1): 16 CBs.
//   * per CB, LDS holds XY[slot] = (x, y) branch inputs of the current constituent
//     decoder and AUX[slot] (ext1 / app1 bookkeeping of turbodecoder_iter.h); after a
//     constituent decode XY.lo is overwritten with its output LLR.  The QPP
//     interleave between half-iterations is an LDS gather.
//   * beta is not stored per step: the backward pass keeps a checkpoint every W
//     steps, the forward pass recomputes W betas into registers before consuming
//     them.  Integer recursion => the recomputed values are bit-identical.
//   * everything runs inside one launch for all half-iterations; HBM traffic is the
//     input LLRs once per half-iteration read + K/8 output bytes.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <vector>
#include <stdint.h>

#include "crc24_dev.h"
#include "tdec_kernel.h"
#include "stage_timing.h"

namespace srsran_amd {

typedef short v2s __attribute__((ext_vector_type(2)));

static constexpr int W        = TDEC_W;        // beta checkpoint / recompute window
static constexpr int OVERLAP  = TDEC_OVERLAP;  // win_overlap_len (turbodecoder_win.h:54,149)
static constexpr short NEGINF = -10000;

__device__ __forceinline__ v2s u2v(uint32_t u) { return __builtin_bit_cast(v2s, u); }
__device__ __forceinline__ uint32_t v2u(v2s v) { return __builtin_bit_cast(uint32_t, v); }

template <bool SAT>
__device__ __forceinline__ v2s padd(v2s a, v2s b)
{
  if constexpr (SAT) {
    return __builtin_elementwise_add_sat(a, b);
  } else {
    return a + b;
  }
}
template <bool SAT>
__device__ __forceinline__ v2s psub(v2s a, v2s b)
{
  if constexpr (SAT) {
    return __builtin_elementwise_sub_sat(a, b);
  } else {
    return a - b;
  }
}
__device__ __forceinline__ v2s pmax(v2s a, v2s b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ v2s lo2(v2s a) { return __builtin_shufflevector(a, a, 0, 0); }
__device__ __forceinline__ v2s hi2(v2s a) { return __builtin_shufflevector(a, a, 1, 1); }
__device__ __forceinline__ v2s swp(v2s a) { return __builtin_shufflevector(a, a, 1, 0); }
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

// Per-lane constants (quad position j = lane & 3).
struct LaneSel {
  uint32_t rb;     // beta: (o_j, o_{j+4}) from the two DPP reads
  uint32_t c0, c1; // alpha: bit-0 / bit-1 source pairs
  uint32_t gb1, gb2, ga0, ga1;  // branch-metric selectors over {x, y, xy, 0}
};

__device__ __forceinline__ LaneSel lane_sel(int j)
{
  LaneSel s;
  const int h = j & 1;
  s.rb        = h ? 0x07060302u : 0x05040100u;
  s.c0        = j < 2 ? 0x07060100u : 0x05040302u;
  s.c1        = j < 2 ? 0x05040302u : 0x07060100u;
  // bytes of {XYS=(xy,xy) : XY=(x,y)}: x=0,1 y=2,3 xy=4,5 zero=0x0c
  const uint32_t b1[4] = {0x05040c0cu, 0x03020100u, 0x01000302u, 0x0c0c0504u};
  const uint32_t b2[4] = {0x0c0c0504u, 0x01000302u, 0x03020100u, 0x05040c0cu};
  s.gb1                = j == 0 ? b1[0] : (j == 1 ? b1[1] : (j == 2 ? b1[2] : b1[3]));
  s.gb2                = j == 0 ? b2[0] : (j == 1 ? b2[1] : (j == 2 ? b2[2] : b2[3]));
  s.ga0                = h ? 0x0c0c0302u : 0x03020c0cu;
  s.ga1                = h ? 0x05040100u : 0x01000504u;
  return s;
}

// Backward step (turbodecoder_win.h:641-664 / turbodecoder_gen.c:78-100).
template <bool SAT>
__device__ __forceinline__ v2s beta_step(v2s P, v2s xy_in, const LaneSel& ls)
{
  const v2s xys = padd<SAT>(xy_in, swp(xy_in));
  const v2s g1  = perm(xys, xy_in, ls.gb1);  // the second metric pair is always swap(g1)
  const v2s t1  = dpp<QP(0, 0, 1, 1)>(P);
  const v2s t2  = dpp<QP(2, 2, 3, 3)>(P);
  const v2s r   = perm(t2, t1, ls.rb);
  return pmax(padd<SAT>(lo2(r), g1), padd<SAT>(hi2(r), swp(g1)));
}

// Forward candidates (turbodecoder_win.h:767-785 / turbodecoder_gen.c:133-149).
template <bool SAT>
__device__ __forceinline__ void alpha_cand(v2s P, v2s xy_in, const LaneSel& ls, v2s& c0, v2s& c1)
{
  const v2s xys = padd<SAT>(xy_in, swp(xy_in));
  const v2s ga  = perm(xys, xy_in, ls.ga0);
  const v2s gb  = perm(xys, xy_in, ls.ga1);
  const v2s u   = dpp<QP(0, 2, 0, 2)>(P);
  const v2s v   = dpp<QP(1, 3, 1, 3)>(P);
  c0            = padd<SAT>(perm(v, u, ls.c0), ga);
  c1            = padd<SAT>(perm(v, u, ls.c1), gb);
}

// LLR = max_i(beta_i + c1_i) - max_i(beta_i + c0_i) over the quad (win.h:788-815).
template <bool SAT>
__device__ __forceinline__ short llr_out(v2s B, v2s c0, v2s c1)
{
  const v2s m0 = padd<SAT>(B, c0);
  const v2s m1 = padd<SAT>(B, c1);
  v2s q        = pmax(perm(m1, m0, 0x05040100u), perm(m1, m0, 0x07060302u));  // (max0, max1)
  q            = pmax(q, dpp<QP(1, 0, 3, 2)>(q));
  q            = pmax(q, dpp<QP(2, 3, 0, 1)>(q));
  const v2s d  = psub<SAT>(swp(q), q);  // .x = max1 - max0
  return d.x;
}

// normalize(): subtract state 0 from all states (win.h:480-498, gen.c:105-110).
template <bool SAT>
__device__ __forceinline__ v2s norm(v2s P)
{
  return psub<SAT>(P, lo2(dpp<QP(0, 0, 0, 0)>(P)));
}

__device__ __forceinline__ v2s init_known(int j) { return j == 0 ? v2s{0, NEGINF} : v2s{NEGINF, NEGINF}; }

// beta_trellis (win.h:500-548): tail steps K+2..K for the last sub-block, int16 wrap.
__device__ __forceinline__ v2s trellis_pair(const short* xt, const short* yt, int j)
{
  short o[8] = {0, NEGINF, NEGINF, NEGINF, NEGINF, NEGINF, NEGINF, NEGINF};
#pragma unroll
  for (int t = 2; t >= 0; t--) {
    const short x = xt[t], y = yt[t], xy = (short)(x + y);
    short n[8];
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
  v2s r;
  r.x = j == 0 ? o[0] : (j == 1 ? o[2] : (j == 2 ? o[4] : o[6]));
  r.y = j == 0 ? o[1] : (j == 1 ? o[3] : (j == 2 ? o[5] : o[7]));
  return r;
}

// Per-NSB compile-time geometry.
template <int NSB>
struct Geo {
  static constexpr bool SAT   = NSB > 1;         // window decoders saturate, generic wraps
  static constexpr int  G     = 4 * NSB;         // lanes per code block
  static constexpr int  CPW   = 64 / G;          // code blocks per wave
  static constexpr int  KMAX  = NSB == 16 ? 6144 : (NSB == 8 ? 800 : 400);
  static constexpr int  NPL   = (KMAX + G - 1) / G;  // prepare positions per lane
};

struct Smem {
  uint32_t* xy;   // [CPW][XYW] (x,y) / output LLR in .lo
  short*    aux;  // [CPW][XYW]
  uint32_t* ck;   // [M][64]
};

// Normalisation predicates.
template <int NSB>
__device__ __forceinline__ bool beta_norm_at(int p, int K)
{
  if constexpr (NSB > 1) {
    return (p % 2) == 0 && p != 0;
  } else {
    return (p % 4) == 0 && p < K;
  }
}
template <int NSB>
__device__ __forceinline__ bool alpha_norm_at(int t)
{
  if constexpr (NSB > 1) {
    return (t % 2) == 0 && t != 0;
  } else {
    return ((t + 1) % 4) == 0;
  }
}

// Schedule of one constituent decode ("crossover"): with Mb = ceil(Nb/W) beta
// windows and Ma = ceil(La/W) alpha windows and split h,
//   phase 1: alpha forward over windows [0, h)      || beta backward over [h, Mb)
//            (alpha checkpoints ckA[m] = state entering window m, slots 0..h-1;
//             beta checkpoints ckB[m] = stored beta[mW] for m > h, slots m-1)
//   phase 2: alpha forward over windows [h, Ma)      || beta backward over [0, h)
//            each side recomputes the other direction's metrics for the window
//            from a checkpoint and emits the LLRs of its positions.
// The two directions are independent dependency chains, interleaved in one
// instruction stream.  Every (position, state) value is computed with the
// reference's arithmetic, so the output is bit-identical to the sequential
// beta-then-alpha order of turbodecoder_win.h / turbodecoder_gen.c.

// Backward window over positions p1-1 .. p0 (FULL => p1 = p0 + W).  Stores the
// stored (pre-normalisation) beta[p0] into slot m-1 when store_ck, and returns it
// in `stored`.
template <int NSB, bool FULL>
__device__ __forceinline__ v2s beta_window(v2s P, const uint32_t* xy, int p0, int p1, int m, bool store_ck, int K,
                                           uint32_t* ck, int lane, const LaneSel& ls, v2s& stored)
{
  constexpr bool SAT = Geo<NSB>::SAT;
  v2s            xw[W];
#pragma unroll
  for (int i = 0; i < W; i++) {
    if (FULL || p0 + i < p1) {
      xw[i] = u2v(xy[p0 + i]);
    }
  }
#pragma unroll
  for (int i = W - 1; i >= 0; i--) {
    if (FULL || p0 + i < p1) {
      P = beta_step<SAT>(P, xw[i], ls);
      if (i == 0) {
        stored = P;
        if (store_ck) {
          ck[(m - 1) * 64 + lane] = v2u(P);
        }
      }
      if (beta_norm_at<NSB>(p0 + i, K)) {
        P = norm<SAT>(P);
      }
    }
  }
  return P;
}

// Phase-1 alpha-only window (entry checkpoint in slot ma).
template <int NSB>
__device__ __forceinline__ v2s alpha_fw_window(v2s P, const uint32_t* xy, int t0, int ma, uint32_t* ck, int lane,
                                               const LaneSel& ls)
{
  constexpr bool SAT = Geo<NSB>::SAT;
  v2s            xw[W];
#pragma unroll
  for (int i = 0; i < W; i++) {
    xw[i] = u2v(xy[t0 + i]);
  }
  ck[ma * 64 + lane] = v2u(P);
#pragma unroll
  for (int i = 0; i < W; i++) {
    v2s c0, c1;
    alpha_cand<SAT>(P, xw[i], ls, c0, c1);
    P = pmax(c0, c1);
    if (alpha_norm_at<NSB>(t0 + i)) {
      P = norm<SAT>(P);
    }
  }
  return P;
}

// Phase-2 alpha side, window at t0: recompute beta[t0+1 .. c] from checkpoint c
// into registers, then alpha + LLR for t0 .. ta-1 (FULL => c = ta = t0 + W).
template <int NSB, bool FULL>
__device__ __forceinline__ v2s alpha_window(v2s P, const uint32_t* xy, short* xyo, int t0, int c, int ta, int Nb,
                                            int K, v2s ckv, const LaneSel& ls)
{
  constexpr bool SAT = Geo<NSB>::SAT;
  v2s            xw[W];
  v2s            bw[W];
#pragma unroll
  for (int i = 0; i < W; i++) {
    if (FULL || t0 + i < c) {
      xw[i] = u2v(xy[t0 + i]);
    }
  }
  v2s       Pb = ckv;
  const int ic = FULL ? W - 1 : c - t0 - 1;
#pragma unroll
  for (int i = W - 1; i >= 0; i--) {
    if (i == ic) {
      bw[i] = Pb;
      if (c < Nb && beta_norm_at<NSB>(c, K)) {
        Pb = norm<SAT>(Pb);
      }
    } else if (i < ic) {
      Pb    = beta_step<SAT>(Pb, xw[i + 1], ls);
      bw[i] = Pb;
      if (beta_norm_at<NSB>(t0 + 1 + i, K)) {
        Pb = norm<SAT>(Pb);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < W; i++) {
    if (FULL || t0 + i < ta) {
      v2s c0, c1;
      alpha_cand<SAT>(P, xw[i], ls, c0, c1);
      const short o = llr_out<SAT>(bw[i], c0, c1);
      P             = pmax(c0, c1);
      if (alpha_norm_at<NSB>(t0 + i)) {
        P = norm<SAT>(P);
      }
      xyo[2 * (t0 + i)] = o;
    }
  }
  return P;
}

// Phase-2 beta side, full window at t0: recompute alpha[t0 .. t0+W-1] from the
// entry checkpoint, then beta backward with the LLR of every position.  Bst is
// the stored (pre-normalisation) beta of the position above the window.
template <int NSB>
__device__ __forceinline__ v2s beta_llr_window(v2s P, v2s& Bst, const uint32_t* xy, short* xyo, int t0, int K,
                                               v2s cka, const LaneSel& ls)
{
  constexpr bool SAT = Geo<NSB>::SAT;
  v2s            xw[W];
  v2s            cw0[W], cw1[W];  // alpha candidates of every position (bit 0 / bit 1)
#pragma unroll
  for (int i = 0; i < W; i++) {
    xw[i] = u2v(xy[t0 + i]);
  }
  v2s a = cka;
#pragma unroll
  for (int i = 0; i < W; i++) {
    alpha_cand<SAT>(a, xw[i], ls, cw0[i], cw1[i]);
    if (i < W - 1) {
      a = pmax(cw0[i], cw1[i]);
      if (alpha_norm_at<NSB>(t0 + i)) {
        a = norm<SAT>(a);
      }
    }
  }
#pragma unroll
  for (int i = W - 1; i >= 0; i--) {
    xyo[2 * (t0 + i)] = llr_out<SAT>(Bst, cw0[i], cw1[i]);
    P                 = beta_step<SAT>(P, xw[i], ls);
    Bst               = P;
    if (beta_norm_at<NSB>(t0 + i, K)) {
      P = norm<SAT>(P);
    }
  }
  return P;
}

// One constituent MAP decode for this quad's sub-block, split over the two waves
// of the workgroup: wave 0 runs the alpha side, wave 1 the beta side of the
// crossover schedule; they meet only through the checkpoints, one barrier per
// phase.  XY[base + k] holds the branch inputs; the output LLR overwrites XY.lo.
// Nb = length of the beta recursion (L, or K+3 for the generic decoder), La =
// alpha length (L or K), M = Mb = beta checkpoints.  Both waves reach the same
// barriers.
template <int NSB>
__device__ __forceinline__ void map_decode(const Smem& sm, int base, int wave, int lane, int j, int s, int K, int L, int Nb, int La,
                           int M, const short* xt, const short* yt)
{
  constexpr bool SAT = Geo<NSB>::SAT;
  const LaneSel  ls  = lane_sel(j);
  const uint32_t* xy = sm.xy + base;
  short*          xyo = reinterpret_cast<short*>(sm.xy + base);
  uint32_t*       ck  = sm.ck;
  const int       Mb  = M;
  const int       Ma  = (La + W - 1) / W;
  const int       h   = max(1, min((Nb + W) / (2 * W), La / W));

  if (wave == 0) {
    // ---------------- alpha side ----------------
    v2s P = init_known(j);
    if constexpr (NSB > 1) {
      // training over the last 40 steps of the own sub-block (win.h:747-756)
      P = v2s{NEGINF, NEGINF};
#pragma unroll
      for (int k = 0; k < OVERLAP; k++) {
        v2s c0, c1;
        alpha_cand<SAT>(P, u2v(xy[L - OVERLAP + k]), ls, c0, c1);
        P = pmax(c0, c1);
        if (alpha_norm_at<NSB>(k)) {
          P = norm<SAT>(P);
        }
      }
      const v2s prv = u2v((uint32_t)__shfl_up((int)v2u(P), 4, 64));  // move_left
      P             = (s == 0) ? init_known(j) : prv;
    }
    for (int ma = 0; ma < h; ma++) {  // phase 1: windows [0, h), entry checkpoints in slots 0..h-1
      P = alpha_fw_window<NSB>(P, xy, ma * W, ma, ck, lane, ls);
    }
    __syncthreads();
    for (int ma = h; ma < Ma; ma++) {  // phase 2: windows [h, Ma) with beta recompute + LLR
      const int t0  = ma * W;
      const v2s ckb = u2v(ck[ma * 64 + lane]);
      if (t0 + W <= La) {
        P = alpha_window<NSB, true>(P, xy, xyo, t0, t0 + W, t0 + W, Nb, K, ckb, ls);
      } else {
        P = alpha_window<NSB, false>(P, xy, xyo, t0, min(t0 + W, Nb), La, Nb, K, ckb, ls);
      }
    }
  } else {
    // ---------------- beta side ----------------
    v2s P = init_known(j);
    if constexpr (NSB > 1) {
      // training over the first 40 steps of the own sub-block (win.h:622-630)
      P = v2s{NEGINF, NEGINF};
#pragma unroll
      for (int k = OVERLAP - 1; k >= 0; k--) {
        P = beta_step<SAT>(P, u2v(xy[k]), ls);
        if (beta_norm_at<NSB>(k, K)) {
          P = norm<SAT>(P);
        }
      }
      const v2s nxt = u2v((uint32_t)__shfl_down((int)v2u(P), 4, 64));  // move_right
      P             = (s == NSB - 1) ? trellis_pair(xt, yt, j) : nxt;   // last sub-block: tail trellis
    }
    ck[(Mb - 1) * 64 + lane] = v2u(P);  // ckB[Mb] = beta[Nb]
    v2s Bst                  = P;
    int mb                   = Mb - 1;
    if (Nb - mb * W < W) {  // partial top window
      P = beta_window<NSB, false>(P, xy, mb * W, Nb, mb, mb > h, K, ck, lane, ls, Bst);
      mb--;
    }
    for (; mb >= h; mb--) {  // phase 1: windows [h, Mb), checkpoints in slots h..Mb-1
      P = beta_window<NSB, true>(P, xy, mb * W, mb * W + W, mb, mb > h, K, ck, lane, ls, Bst);
    }
    __syncthreads();
    for (mb = h - 1; mb >= 0; mb--) {  // phase 2: windows [0, h) with alpha recompute + LLR
      const v2s cka = u2v(ck[mb * 64 + lane]);
      P             = beta_llr_window<NSB>(P, Bst, xy, xyo, mb * W, K, cka, ls);
    }
  }
}

__device__ __forceinline__ uint32_t pack2(short lo, short hi)
{
  return (uint32_t)(uint16_t)lo | ((uint32_t)(uint16_t)hi << 16);
}

template <int NSB, bool ES>
__device__ __forceinline__ void tdec_body(const TdecArgs& a, int bid)
{
  using Gm                = Geo<NSB>;
  constexpr bool SAT      = Gm::SAT;
  constexpr int  G        = Gm::G;        // lanes per code block in one wave
  constexpr int  G2       = 2 * G;        // threads per code block in the workgroup
  constexpr int  LOG_NSB  = NSB == 16 ? 4 : (NSB == 8 ? 3 : 0);
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];

  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int cw   = lane / G;                 // CB within the workgroup
  const int g    = lane % G;                 // lane within the CB's quad group
  const int t2   = wave * G + g;             // thread within the CB (both waves)
  const int s    = g >> 2;                   // sub-block
  const int j    = g & 3;                    // state-pair index
  const int K    = a.K;
  const int L    = a.L;
  const int Ls   = a.Ls;
  const int XYW  = a.xyw;
  const int M    = a.M;
  const int cb   = bid * Gm::CPW + cw;  // launch index
  const int cbl  = cb < (int)a.ncb ? cb : (int)a.ncb - 1;
  const bool live = cb < (int)a.ncb && (!ES || a.cbs[cbl].slot != TDEC_PAD_SLOT);
  // DL-SCH mode: blocks whose CRC already passed are not decoded; padding blocks
  // (past ncb, or TDEC_PAD_SLOT entries) never hold back the workgroup's early exit.  The block descriptor a.cbs[cbl] is
  // re-read where needed instead of being kept live across the decode loop.
  bool done = ES && (!live || *a.cbs[cbl].skip);

  Smem sm;
  sm.xy  = smem;
  sm.aux = reinterpret_cast<short*>(smem + Gm::CPW * XYW);
  sm.ck  = smem + Gm::CPW * XYW + (Gm::CPW * XYW + 1) / 2;
  uint32_t* red  = sm.ck + M * 64;  // [CPW][2] CRC partials per wave
  uint32_t* xyc  = sm.xy + cw * XYW;
  short*    xylo = reinterpret_cast<short*>(xyc);
  short*    auxc = sm.aux + cw * XYW;

  // Hard decision byte b (bits 8b..8b+7, MSB first) of the latest decoder output:
  // ext1 after DEC1 (natural slots), app1 = ext2 de-interleaved after DEC2.
  auto decide_byte = [&](int b, bool after_dec1) -> uint32_t {
    uint32_t byte = 0;
#pragma unroll
    for (int t = 0; t < 8; t++) {
      const int n = 8 * b + t;
      int       sl;
      if constexpr (NSB > 1) {
        const int sb_ = (int)__umulhi((uint32_t)n, a.magicL);  // n / L
        sl            = sb_ * Ls + (n - sb_ * L);
      } else {
        sl = n;
      }
      const short v = after_dec1 ? xylo[2 * sl] : xylo[2 * a.trev_nat[n]];
      byte |= (uint32_t)(v > 0) << (7 - t);
    }
    return byte;
  };

  const short* in = ES ? a.cbs[cbl].in : a.in + (size_t)cbl * a.in_stride;
  const bool   sb = a.layout_sb;
  // Positions are visited in "q order": the rm_turbo sub-block order for window
  // decoders (q = k*NSB + s, coalesced in the SB input), natural order otherwise.
  auto qslot = [&](int q) -> int { return NSB > 1 ? (q & (NSB - 1)) * Ls + (q >> LOG_NSB) : q; };
  const short* tail = sb ? in + 3 * (K + 32) : in + 3 * K;
  short st[3], p0t[3], x2t[3], p1t[3];
#pragma unroll
  for (int t = 0; t < 3; t++) {
    st[t]  = tail[2 * t];
    p0t[t] = tail[2 * t + 1];
    x2t[t] = tail[6 + 2 * t];
    p1t[t] = tail[6 + 2 * t + 1];
  }
  // Visit order of the prepare phase: rm_turbo SB order (q) for window decoders
  // on SB input, natural order otherwise.  The QPP tables come in both orders.
  const bool      vsb = NSB > 1 && sb;
  const uint16_t* tfq = vsb ? a.tfwd : a.tfwd_nat;  // slot of pi(n(p))
  const uint16_t* trq = vsb ? a.trev : a.trev_nat;  // slot of pi^-1(n(p))
  const int       nch = K / 4;
  auto pslot = [&](int p) -> int {  // LDS slot of visit position p
    if constexpr (NSB > 1) {
      if (vsb) {
        return qslot(p);
      }
      const int sbn = (int)__umulhi((uint32_t)p, a.magicL);  // p / L
      return sbn * Ls + (p - sbn * L);
    } else {
      return p;
    }
  };
  // Visit this thread's positions in chunks of 4 (visit order), BATCH chunks at a
  // time with all global loads of a batch issued before use:
  // fn(p, sys, par0, par1, table) -- only the streams the half-iteration needs
  // are loaded (dec1: sys+par0 [+ pi^-1 table], dec2: par1 + pi table).
  auto for_chunks = [&](int hh, auto&& fn) {
    constexpr int BATCH = NSB == 8 ? 2 : 4;
    const bool    d1    = (hh & 1) == 0;
    const bool    need_t = hh > 0;
    const uint16_t* tab  = d1 ? trq : tfq;
    for (int c0 = t2; c0 < nch; c0 += BATCH * G2) {
      uint2 w0[BATCH], w1[BATCH], w2[BATCH], tv[BATCH];
#pragma unroll
      for (int i = 0; i < BATCH; i++) {
        const int c = c0 + i * G2;
        if (c < nch) {
          if (vsb) {
            const short* b = in + 4 * c;
            if (d1) {
              w0[i] = *reinterpret_cast<const uint2*>(b);
              w1[i] = *reinterpret_cast<const uint2*>(b + (K + 32));
            } else {
              w2[i] = *reinterpret_cast<const uint2*>(b + 2 * (K + 32));
            }
          } else {
            const uint2* b = reinterpret_cast<const uint2*>(in + 12 * c);
            w0[i]          = b[0];
            w1[i]          = b[1];
            w2[i]          = b[2];
          }
          if (need_t) {
            tv[i] = *reinterpret_cast<const uint2*>(tab + 4 * c);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < BATCH; i++) {
        const int c = c0 + i * G2;
        if (c < nch) {
#pragma unroll
          for (int v = 0; v < 4; v++) {
            short x0, x1, x2;
            if (vsb) {
              const uint32_t d0 = v < 2 ? w0[i].x : w0[i].y;
              const uint32_t d1w = v < 2 ? w1[i].x : w1[i].y;
              const uint32_t d2 = v < 2 ? w2[i].x : w2[i].y;
              x0 = (short)((v & 1) ? (d0 >> 16) : (d0 & 0xffff));
              x1 = (short)((v & 1) ? (d1w >> 16) : (d1w & 0xffff));
              x2 = (short)((v & 1) ? (d2 >> 16) : (d2 & 0xffff));
            } else {  // natural: 12 interleaved values S,P0,P1 x 4
              const uint32_t e[6] = {w0[i].x, w0[i].y, w1[i].x, w1[i].y, w2[i].x, w2[i].y};
              auto el = [&](int k) -> short { return (short)((k & 1) ? (e[k >> 1] >> 16) : (e[k >> 1] & 0xffff)); };
              x0 = el(3 * v);
              x1 = el(3 * v + 1);
              x2 = el(3 * v + 2);
            }
            int t = 0;
            if (need_t) {
              const uint32_t d = v < 2 ? tv[i].x : tv[i].y;
              t                = (int)((v & 1) ? (d >> 16) : (d & 0xffff));
            }
            fn(4 * c + v, x0, x1, x2, t);
          }
        }
      }
    }
  };

  // restore state from a previous launch (srsran_tdec_iteration path)
  if (a.n_start > 0) {
    const short* se = a.state + (size_t)cbl * 2 * XYW;
    for (int i = t2; i < XYW; i += G2) {
      xylo[2 * i] = se[i];
      auxc[i]     = se[XYW + i];
    }
    __syncthreads();
  }

  const int base = cw * XYW + (NSB > 1 ? s * Ls : 0);
  const int Nb   = NSB > 1 ? L : K + 3;
  const int La   = NSB > 1 ? L : K;

  if constexpr (ES) {
    if (live && done && t2 == 0) {  // skipped block (sch.c:392, 476-480)
      const uint32_t slot = a.cbs[cbl].slot;
      a.noi_out[slot]     = 0;
      a.crc_ok[slot]      = 1;
    }
  }
  const int h_end = (ES && __syncthreads_or(!done) == 0) ? a.n_start : a.n_end;
  for (int h = a.n_start; h < h_end; h++) {
    // -------- prepare branch inputs (turbodecoder_iter.h:104-128) --------
    // Each thread owns chunks of 4 consecutive positions in visit order (SB order
    // for window decoders on SB input, natural order otherwise); all its global
    // loads are issued before any of them is consumed.
    if ((h & 1) == 0) {
      if (h == 0) {
        for_chunks(h, [&](int p, short sx, short p0, short, int) { xyc[pslot(p)] = pack2(sx, p0); });
      } else {
        // app1 = ext2 de-interleaved: gather into the dead XY.hi half of the own slot
        for_chunks(h, [&](int p, short, short, short, int t) { xylo[2 * pslot(p) + 1] = xylo[2 * t]; });
        __syncthreads();
        for_chunks(h, [&](int p, short sx, short p0, short, int) {
          const int   sl = pslot(p);
          const short a1 = (short)(xylo[2 * sl + 1] - auxc[sl]);  // app1 -= ext1 (vec_sub, wraps)
          auxc[sl]       = a1;
          const short x  = SAT ? __builtin_elementwise_add_sat(sx, a1) : (short)(sx + a1);
          xyc[sl]        = pack2(x, p0);
        });
      }
      if constexpr (NSB == 1) {
        if (t2 < 3) {
          xyc[K + t2] = pack2(st[t2], p0t[t2]);
        }
      }
    } else {
      for (int p = t2; p < K; p += G2) {  // ext1 -= app1 (h > 1), keep it in AUX
        const int   sl = pslot(p);
        const short e  = xylo[2 * sl];
        auxc[sl]       = h > 1 ? (short)(e - auxc[sl]) : e;
      }
      __syncthreads();
      // app2 = ext1 interleaved
      for_chunks(h, [&](int p, short, short, short p1, int t) { xyc[pslot(p)] = pack2(auxc[t], p1); });
      if constexpr (NSB == 1) {
        if (t2 < 3) {
          xyc[K + t2] = pack2(x2t[t2], p1t[t2]);
        }
      }
    }
    __syncthreads();

    // -------- constituent MAP decode (wave 0: alpha side, wave 1: beta side) --------
    const bool dec1 = (h & 1) == 0;
    map_decode<NSB>(sm, base, wave, lane, j, s, K, L, Nb, La, M, dec1 ? st : x2t, dec1 ? p0t : p1t);
    __syncthreads();

    // -------- DL-SCH early stop: CRC of the hard decision (sch.c:426-456) --------
    if constexpr (ES) {
      if (h + 1 >= a.min_iters) {
        // this thread's contiguous chunk of decision bytes, CRC'd from zero, then
        // shifted to its place by x^(8*bytes_after) mod P and XOR-combined
        const int nbytes = K / 8;
        const int bpt    = (nbytes + G2 - 1) / G2;
        const int b0     = t2 * bpt;
        const bool     crc_a = a.cbs[cbl].crc_a;
        const uint32_t poly = crc_a ? LTE_CRC24A : LTE_CRC24B;
        uint32_t       crc  = 0;
        const int      b1   = min(b0 + bpt, nbytes);
#pragma unroll 1
        for (int b = b0; b < b1; b++) {
          crc = crc24_byte(crc, decide_byte(b, dec1), poly);
        }
        uint32_t part = b0 < nbytes ? clmul_mod24(crc, (crc_a ? a.xpow_a : a.xpow_b)[nbytes - b1], poly) : 0;
#pragma unroll
        for (int off = 1; off < G; off <<= 1) {
          part ^= (uint32_t)__shfl_xor((int)part, off, 64);
        }
        if (g == 0) {
          red[cw * 2 + wave] = part;
        }
        __syncthreads();
        const bool ok = (red[cw * 2] ^ red[cw * 2 + 1]) == 0;
        if (ok && !done && live) {
          const uint32_t slot = a.cbs[cbl].slot;
          uint8_t*       out  = a.out + (size_t)slot * a.out_stride;
#pragma unroll 1
          for (int b = b0; b < b1; b++) {
            out[b] = (uint8_t)decide_byte(b, dec1);
          }
          if (t2 == 0) {
            a.noi_out[slot] = (uint8_t)(h + 1);
            a.crc_ok[slot]  = 1;
          }
        }
        done = done || ok;
      }
      if (__syncthreads_or(!done) == 0) {
        break;  // every code block of this workgroup has passed its CRC
      }
    }
  }

  // -------- hard decision (turbodecoder.c:370-378), natural bit order --------
  const bool last_dec1 = ((a.n_end - 1) & 1) == 0;
  if (live && !done) {
    const int cbm = ES ? (int)a.cbs[cbl].slot : cbl;  // output / state slot
    uint8_t*  out = a.out + (size_t)cbm * (ES ? a.out_stride : K / 8);
    for (int b = t2; b < K / 8; b += G2) {
      out[b] = (uint8_t)decide_byte(b, last_dec1);
    }
    if (ES && t2 == 0) {
      a.noi_out[cbm] = (uint8_t)a.n_end;
      a.crc_ok[cbm]  = 0;
    }
    if (a.state) {
      short* se = a.state + (size_t)cbm * 2 * XYW;
      for (int i = t2; i < XYW; i += G2) {
        se[i]       = xylo[2 * i];
        se[XYW + i] = auxc[i];
      }
    }
  }
}

template <int NSB, bool ES>
__global__ __launch_bounds__(128, 2) void tdec_kernel(TdecArgs a)
{
  tdec_body<NSB, ES>(a, blockIdx.x);
}

// Several code-block sizes of one decoder class in one launch: workgroup b belongs to the group
// g with first[g] <= b < first[g + 1] (descriptors in device memory, read with scalar loads).
template <int NSB>
__global__ __launch_bounds__(128, 2) void tdec_multi_kernel(const TdecArgs* __restrict__ groups,
                                                            const uint32_t* __restrict__ first, int ngroups)
{
  const uint32_t b  = blockIdx.x;
  int            lo = 0, hi = ngroups - 1;  // last g with first[g] <= b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (first[mid] <= b) {
      lo = mid;
    } else {
      hi = mid - 1;
    }
  }
  const TdecArgs a = groups[lo];
  tdec_body<NSB, false>(a, (int)(b - first[lo]));
}

hipError_t tdec_multi_launch(int nsb, const TdecArgs* d_groups, const uint32_t* d_first, int ngroups,
                             uint32_t nblocks, size_t lds, hipStream_t stream)
{
  StageScope timing_scope(ST_TDEC, stream);
  if (ngroups == 0 || nblocks == 0) {
    return hipSuccess;
  }
  tdec_set_last_kernel(nsb == 16 ? "tdec_multi_kernel<16>" : nsb == 8 ? "tdec_multi_kernel<8>" : "tdec_multi_kernel<1>");
  switch (nsb) {
    case 16:
      hipLaunchKernelGGL(tdec_multi_kernel<16>, dim3(nblocks), dim3(128), lds, stream, d_groups, d_first, ngroups);
      break;
    case 8:
      hipLaunchKernelGGL(tdec_multi_kernel<8>, dim3(nblocks), dim3(128), lds, stream, d_groups, d_first, ngroups);
      break;
    case 1:
      hipLaunchKernelGGL(tdec_multi_kernel<1>, dim3(nblocks), dim3(128), lds, stream, d_groups, d_first, ngroups);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

int tdec_cpw(int nsb) { return 64 / (4 * nsb); }

template <int NSB>
static hipError_t launch(const TdecArgs& a, hipStream_t stream)
{
  StageScope timing_scope(ST_TDEC, stream);
  const int    cpw  = Geo<NSB>::CPW;
  const int    grid = (a.ncb + cpw - 1) / cpw;
  const size_t lds  = tdec_lds_bytes(NSB, a.xyw, a.M);
  tdec_set_last_kernel(NSB == 16 ? "tdec_kernel<16>" : NSB == 8 ? "tdec_kernel<8>" : "tdec_kernel<1>");
  if (a.cbs) {
    hipLaunchKernelGGL((tdec_kernel<NSB, true>), dim3(grid), dim3(128), lds, stream, a);
  } else {
    hipLaunchKernelGGL((tdec_kernel<NSB, false>), dim3(grid), dim3(128), lds, stream, a);
  }
  return hipGetLastError();
}

hipError_t tdec_launch(int nsb, const TdecArgs& a, hipStream_t stream)
{
  if (a.ncb == 0) {
    return hipSuccess;
  }
  if (tdec16_eligible(nsb, a)) {
    return tdec16_choice(a.ncb) == 2 ? (a.K <= tdecs_w8_max_k() ? tdecs16w8::launch(a, stream) : tdecs16::launch(a, stream))
                                     : tdec16_launch(a, stream);
  }
  if (tdec8s_eligible(nsb, a)) {
    return a.K <= tdecs_w8_max_k() ? tdecs8w8::launch(a, stream) : tdecs8::launch(a, stream);
  }
  if (tdec1s_eligible(nsb, a)) {
    return tdecs1::launch(a, stream);
  }
  switch (nsb) {
    case 16:
      return launch<16>(a, stream);
    case 8:
      return launch<8>(a, stream);
    case 1:
      return launch<1>(a, stream);
    default:
      return hipErrorInvalidValue;
  }
}

size_t tdec_lds_bytes(int nsb, int xyw, int M)
{
  const int cpw = 64 / (4 * nsb);
  return (size_t)cpw * xyw * 4 + (((size_t)cpw * xyw + 1) / 2) * 4 + (size_t)M * 64 * 4 + (size_t)cpw * 2 * 4;
}

static thread_local const char* t_last_kernel = "";
const char* tdec_last_kernel() { return t_last_kernel; }
void        tdec_set_last_kernel(const char* name) { t_last_kernel = name; }

uint32_t tdec_pair_cbs(const TdecCb* src, uint32_t n, size_t dst_group_start, void* dst_vec)
{
  std::vector<TdecCb>& dst = *static_cast<std::vector<TdecCb>*>(dst_vec);
  uint32_t             pads = 0;
  uintptr_t            lo = 0, hi = 0;  // address range of the open group
  for (uint32_t i = 0; i < n; i++) {
    const uintptr_t p   = (uintptr_t)src[i].in;
    size_t          pos = (dst.size() - dst_group_start) % TDEC_GROUP;
    if (pos != 0 && (std::max(hi, p) - std::min(lo, p)) >= TDEC_PAIR_SPAN) {
      // too far from the group's blocks: pad the group out (the pads repeat its last block, so they
      // stay inside its range) and start a new one
      TdecCb pad = dst.back();
      pad.slot   = TDEC_PAD_SLOT;
      for (; pos < TDEC_GROUP; pos++) {
        dst.push_back(pad);
        pads++;
      }
      pos = 0;
    }
    if (pos == 0) {
      lo = hi = p;
    }
    lo = std::min(lo, p);
    hi = std::max(hi, p);
    dst.push_back(src[i]);
  }
  return pads;
}

void crc24_xpow_table(uint32_t poly, uint32_t* out, int nm)
{
  uint32_t v = 1;  // x^0
  for (int m = 0; m < nm; m++) {
    out[m] = v;
    for (int k = 0; k < 8; k++) {  // v *= x (mod P)
      v = (v & 0x800000u) ? ((v << 1) ^ poly) : (v << 1);
      v &= 0xFFFFFFu;
    }
  }
}

}  // namespace srsran_amd
