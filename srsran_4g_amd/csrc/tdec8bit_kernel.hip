// srsran_4g_amd/csrc/tdec8bit_kernel.hip -- the 8-bit LLR turbo decoder (srsran_tdec_run_all_8bit):
// srsRAN_4G's SSE 8-bit window decoder (16 sub-blocks, 800 < K <= 2048) and AVX2 8-bit window decoder
// (32 sub-blocks, K > 2048), turbodecoder_win.h with WINIMP_IS_SSE8 / WINIMP_IS_AVX8 (lines 154-300,
// 480-832) driven by turbodecoder_iter.h:72-144 (LLR_IS_8BIT) and turbodecoder.c:455-483.  Smaller K
// take the 16-bit decoders on the widened input, as the reference does (srsran_tdec_gpu_run_batch_8bit in tdec_api.cpp).
//
// The arithmetic of those decoders, restated:
//   * metrics are int8 with saturating add / sub (_mm_adds_epi8), -INF = 0 (INF 0): unknown states
//     start at 0, and the first sub-block's alpha start state is all zeros too;
//   * normalisation every step but k = 0 by the maximum over the 8 states (normalize_max);
//   * the tail trellis (beta_trellis) saturates upwards only ((int16)x + y > 127 ? 127 : (int8));
//   * the LLR m1 - m0 (saturating) is halved by an arithmetic shift (divide_output 1).
//
// Mapping: TWO LANES PER SUB-BLOCK, one in each of the workgroup's two waves (alpha / beta, meeting in the middle
// of the sub-block: map_pass), the 8 states in 8 registers (int8 values held in int32).  A workgroup is two waves
// over 64 / NSB code blocks.  The block's input streams, a-priori and
// extrinsic arrays live in LDS (6 x (K + 4) bytes; ext2 overwrites app2 in place); the metrics a MAP pass hands from
// one wave to the other go to a global scratch ([block][position][lane] x 8 bytes, one 8-byte store a lane a
// position, coalesced over the block's lanes): the betas of the upper half, the alphas of the lower half.  All half-iterations run in one launch.
// This is the off-by-default path of srsUE (srsue/src/main.cc:404-406); it is written for parity, not
// tuned like the 16-bit decoders.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc24_dev.h"
#include "sch_kernel.h"
#include "tdec8bit_kernel.h"
#include "tdec_kernel.h"

namespace srsran_amd {
namespace {

constexpr int OVL = 40;  // win_overlap_len (turbodecoder_win.h:182, 291)

__device__ __forceinline__ int sat8(int v) { return v > 127 ? 127 : (v < -128 ? -128 : v); }
__device__ __forceinline__ int sadd(int a, int b) { return sat8(a + b); }
__device__ __forceinline__ int ssub(int a, int b) { return sat8(a - b); }
// beta_trellis's sadd (turbodecoder_win.h:470-478 with use_saturated_add): upper clamp, int8 wrap below
__device__ __forceinline__ int tadd(int a, int b)
{
  const int z = a + b;
  return z > 127 ? 127 : (int)(int8_t)z;
}

// ---- the same arithmetic on packed int16 pairs (v_pk_*): the 8 states as (s0, s1) (s2, s3) (s4, s5) (s6, s7), int8
// values in int16 lanes.  The sum of two int8 values never leaves int16, so an int8 saturating add is a packed add
// and a clamp to [-128, 127]; and since the clamp is monotonic, max(sat(u), sat(v)) = sat(max(u, v)): a trellis
// step clamps once per state, after its max. ----
typedef short v2s __attribute__((ext_vector_type(2)));
struct S8 {
  v2s a, b, c, d;  // (s0, s1), (s2, s3), (s4, s5), (s6, s7)
};
__device__ __forceinline__ v2s pmax(v2s u, v2s v) { return __builtin_elementwise_max(u, v); }
__device__ __forceinline__ v2s psat(v2s u)
{
  return __builtin_elementwise_min(__builtin_elementwise_max(u, (v2s){-128, -128}), (v2s){127, 127});
}
__device__ __forceinline__ v2s plo(v2s u) { return __builtin_shufflevector(u, u, 0, 0); }
__device__ __forceinline__ v2s phi(v2s u) { return __builtin_shufflevector(u, u, 1, 1); }
__device__ __forceinline__ v2s pv(int u, int v) { return (v2s){(short)u, (short)v}; }

// beta_step (win.h:641-664) on packed states
__device__ __forceinline__ void p_beta_step(S8& o, int x, int y)
{
  const int xy = sadd(x, y);
  const v2s n01 = psat(pmax(plo(o.c) + pv(xy, 0), plo(o.a) + pv(0, xy)));
  const v2s n23 = psat(pmax(phi(o.c) + pv(y, x), phi(o.a) + pv(x, y)));
  const v2s n45 = psat(pmax(plo(o.d) + pv(x, y), plo(o.b) + pv(y, x)));
  const v2s n67 = psat(pmax(phi(o.d) + pv(0, xy), phi(o.b) + pv(xy, 0)));
  o                = S8{n01, n23, n45, n67};
}

// alpha_cand (win.h:767-785) on packed states: mb / nw in state order, each saturated (the LLR adds to them again)
__device__ __forceinline__ void p_alpha_cand(const S8& o, int x, int y, S8& mb, S8& nw)
{
  const int xy = sadd(x, y);
  const v2s p1 = __builtin_shufflevector(o.a, o.b, 0, 3);  // (s0, s3)
  const v2s p2 = __builtin_shufflevector(o.c, o.d, 0, 3);  // (s4, s7)
  const v2s p3 = __builtin_shufflevector(o.a, o.b, 1, 2);  // (s1, s2)
  const v2s p4 = __builtin_shufflevector(o.c, o.d, 1, 2);  // (s5, s6)
  mb = S8{psat(p1 + pv(0, y)), psat(p2 + pv(y, 0)), psat(p3 + pv(0, y)), psat(p4 + pv(y, 0))};
  nw = S8{psat(p3 + pv(xy, x)), psat(p4 + pv(x, xy)), psat(p1 + pv(xy, x)), psat(p2 + pv(x, xy))};
}
__device__ __forceinline__ S8 p_max(const S8& u, const S8& v)
{
  return S8{pmax(u.a, v.a), pmax(u.b, v.b), pmax(u.c, v.c), pmax(u.d, v.d)};
}

// normalize (normalize_max, period 1): o - max, which is <= 0, clamped below
__device__ __forceinline__ void p_normalize(int k, S8& o)
{
  if (k != 0) {
    const v2s m2 = pmax(pmax(o.a, o.b), pmax(o.c, o.d));
    const v2s m  = plo(pmax(m2, __builtin_shufflevector(m2, m2, 1, 0)));
    const v2s lo = (v2s){-128, -128};
    o            = S8{pmax(o.a - m, lo), pmax(o.b - m, lo), pmax(o.c - m, lo), pmax(o.d - m, lo)};
  }
}

// the LLR of a position (win.h:795-813): max over states of sadd(beta, mb) and of sadd(beta, nw), their saturating
// difference halved
__device__ __forceinline__ int8_t p_llr(const S8& b, const S8& mb, const S8& nw)
{
  const v2s s0 = pmax(pmax(b.a + mb.a, b.b + mb.b), pmax(b.c + mb.c, b.d + mb.d));
  const v2s s1 = pmax(pmax(b.a + nw.a, b.b + nw.b), pmax(b.c + nw.c, b.d + nw.d));
  const int m0 = sat8(max((int)s0.x, (int)s0.y)), m1 = sat8(max((int)s1.x, (int)s1.y));
  return (int8_t)(ssub(m1, m0) >> 1);
}

__device__ __forceinline__ uint2 p_pack(const S8& o)
{
  const uint32_t a = __builtin_bit_cast(uint32_t, o.a), b = __builtin_bit_cast(uint32_t, o.b);
  const uint32_t c = __builtin_bit_cast(uint32_t, o.c), d = __builtin_bit_cast(uint32_t, o.d);
  // the low byte of every int16 lane: bytes 0, 2 of a and b, then of c and d
  return make_uint2(__builtin_amdgcn_perm(b, a, 0x06040200u), __builtin_amdgcn_perm(d, c, 0x06040200u));
}
__device__ __forceinline__ S8 p_unpack(uint2 r)
{
  // byte i to the high byte of an int16 lane, then an arithmetic shift right by 8 sign-extends it
  const v2s a = __builtin_bit_cast(v2s, __builtin_amdgcn_perm(0u, r.x, 0x010c000cu)) >> (v2s){8, 8};
  const v2s b = __builtin_bit_cast(v2s, __builtin_amdgcn_perm(0u, r.x, 0x030c020cu)) >> (v2s){8, 8};
  const v2s c = __builtin_bit_cast(v2s, __builtin_amdgcn_perm(0u, r.y, 0x010c000cu)) >> (v2s){8, 8};
  const v2s d = __builtin_bit_cast(v2s, __builtin_amdgcn_perm(0u, r.y, 0x030c020cu)) >> (v2s){8, 8};
  return S8{a, b, c, d};
}
__device__ __forceinline__ S8 p_zero() { return S8{(v2s){0, 0}, (v2s){0, 0}, (v2s){0, 0}, (v2s){0, 0}}; }
__device__ __forceinline__ S8 p_shfl_down(const S8& o, int w)
{
  auto sh = [&](v2s v) {
    return __builtin_bit_cast(v2s, __shfl_down((int)__builtin_bit_cast(uint32_t, v), 1, w));
  };
  return S8{sh(o.a), sh(o.b), sh(o.c), sh(o.d)};
}
__device__ __forceinline__ S8 p_shfl_up(const S8& o, int w)
{
  auto sh = [&](v2s v) { return __builtin_bit_cast(v2s, __shfl_up((int)__builtin_bit_cast(uint32_t, v), 1, w)); };
  return S8{sh(o.a), sh(o.b), sh(o.c), sh(o.d)};
}

// One MAP pass of sub-block d (turbodecoder_win.h:551-832) by TWO lanes, one in each wave of the workgroup (side 0:
// alpha, side 1: beta), meeting in the middle h = Ls / 2.  X systematic (or the de-interleaved extrinsic of DEC 1),
// A optional a-priori, P parity, all SB-ordered in LDS with the tail at [K, K + 3); OUT the extrinsic LLRs.
//   phase 1: side 1 trains beta (first OVL positions, shifted down a lane; the last sub-block from the tail trellis)
//            and runs it over positions Ls-1 .. h, storing every beta before its normalisation (win.h:666-678) at
//            [k + 1]; side 0 trains alpha (last OVL positions, shifted up a lane) and runs it over 0 .. h-1, storing
//            the alpha that enters position k at [k] -- the two index ranges of `sc` do not overlap;
//   phase 2 (after a workgroup barrier): side 0 carries alpha over h .. Ls-1 with the stored betas, side 1 carries
//            beta over h-1 .. 0 with the stored alphas; each emits the LLRs of its positions.
// Every value is the one the reference's single lane computes (alpha through all positions, beta through all
// positions, the LLR from alpha_k and beta_{k+1} before normalisation), so the output is the same; the chain of
// dependent steps a lane walks is halved.  sc: this block's scratch, [Ls + 1][NSB] x 8 bytes.
template <int NSB>
__device__ __forceinline__ void map_pass(const int8_t* X, const int8_t* A, const int8_t* P, int8_t* OUT, int d, int Ls, int K,
                         uint2* sc, int side, bool live)
{
  const int h = Ls / 2;
  S8        o  = p_zero();
  S8        bk = p_zero();  // side 1: the beta of position k + 1 before its normalisation (the LLR of position k reads it)
  if (side == 1) {
    if (live) {
      // ---- beta training over the first OVL positions of this sub-block, from unknown (0) states ----
      for (int k = OVL - 1; k >= 0; k--) {
        const int q = k * NSB + d;
        int       x = X[q];
        if (A) {
          x = sadd(A[q], x);
        }
        p_beta_step(o, x, P[q]);
        p_normalize(k, o);
      }
    }
    // the end state of sub-block d is the training result of sub-block d + 1 (move_right, the whole wave takes part
    // in the shuffle); the last sub-block's comes from the tail (beta_trellis, win.h:500-548)
    o = p_shfl_down(o, NSB);
    if (live && d == NSB - 1) {
      int t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int k = K + 2; k >= K; k--) {
        const int x = X[k], y = P[k], xy = tadd(x, y);
        int       mb[8], nw[8];
        mb[0] = tadd(t[4], xy);
        mb[1] = t[4];
        mb[2] = tadd(t[5], y);
        mb[3] = tadd(t[5], x);
        mb[4] = tadd(t[6], x);
        mb[5] = tadd(t[6], y);
        mb[6] = t[7];
        mb[7] = tadd(t[7], xy);
        nw[0] = t[0];
        nw[1] = tadd(t[0], xy);
        nw[2] = tadd(t[1], x);
        nw[3] = tadd(t[1], y);
        nw[4] = tadd(t[2], y);
        nw[5] = tadd(t[2], x);
        nw[6] = tadd(t[3], xy);
        nw[7] = t[3];
#pragma unroll
        for (int i = 0; i < 8; i++) {
          t[i] = mb[i] > nw[i] ? mb[i] : nw[i];
        }
      }
      o = S8{pv(t[0], t[1]), pv(t[2], t[3]), pv(t[4], t[5]), pv(t[6], t[7])};
    }
    if (live) {
      bk                       = o;  // beta_Ls: the end state, read by the LLR of position Ls - 1
      sc[(size_t)Ls * NSB + d] = p_pack(o);
      for (int k = Ls - 1; k >= h; k--) {
        const int q = k * NSB + d;
        int       x = X[q];
        if (A) {
          x = sadd(A[q], x);
        }
        p_beta_step(o, x, P[q]);
        sc[(size_t)k * NSB + d] = p_pack(o);  // stored before normalisation (win.h:666-678)
        bk                      = o;
        p_normalize(k, o);
      }
    }
  } else {
    if (live) {
      // ---- alpha training over the last OVL positions of this sub-block ----
      for (int k = 0; k < OVL; k++) {
        const int q = (Ls - OVL + k) * NSB + d;
        int       x = X[q];
        if (A) {
          x = sadd(A[q], x);
        }
        S8 mb, nw;
        p_alpha_cand(o, x, P[q], mb, nw);
        o = p_max(mb, nw);
        p_normalize(k, o);
      }
    }
    // the start state of sub-block d is the training result of sub-block d - 1 (move_left); sub-block 0
    // starts known: state 0 at 0, the others at -INF = 0
    o = p_shfl_up(o, NSB);
    if (d == 0) {
      o = p_zero();
    }
    if (live) {
      for (int k = 0; k < h; k++) {
        const int q = k * NSB + d;
        sc[(size_t)k * NSB + d] = p_pack(o);  // the alpha entering position k
        int x = X[q];
        if (A) {
          x = sadd(A[q], x);
        }
        S8 mb, nw;
        p_alpha_cand(o, x, P[q], mb, nw);
        o = p_max(mb, nw);
        p_normalize(k, o);
      }
    }
  }
  __syncthreads();
  if (!live) {
    return;
  }
  // the stored metrics are loaded two positions ahead (s0 / s1): the load latency hides behind two steps
  if (side == 0) {
    // ---- alpha over h .. Ls-1 with the stored betas (win.h:684-832) ----
    uint2 s0 = sc[(size_t)(h + 1) * NSB + d], s1 = sc[(size_t)min(h + 2, Ls) * NSB + d];
    for (int k = h; k < Ls; k++) {
      const int   q  = k * NSB + d;
      const uint2 bv = s0;
      s0             = s1;
      s1             = sc[(size_t)min(k + 3, Ls) * NSB + d];
      int x          = X[q];
      if (A) {
        x = sadd(A[q], x);
      }
      S8 mb, nw;
      p_alpha_cand(o, x, P[q], mb, nw);
      OUT[q] = p_llr(p_unpack(bv), mb, nw);  // simd_rb_shift by divide_output (win.h:810-813)
      o      = p_max(mb, nw);
      p_normalize(k, o);
    }
  } else {
    // ---- beta over h-1 .. 0 with the stored alphas ----
    uint2 s0 = sc[(size_t)(h - 1) * NSB + d], s1 = sc[(size_t)max(h - 2, 0) * NSB + d];
    for (int k = h - 1; k >= 0; k--) {
      const int   q  = k * NSB + d;
      const uint2 av = s0;
      s0             = s1;
      s1             = sc[(size_t)max(k - 2, 0) * NSB + d];
      int x          = X[q];
      if (A) {
        x = sadd(A[q], x);
      }
      const int y = P[q];
      S8        mb, nw;
      p_alpha_cand(p_unpack(av), x, y, mb, nw);
      const int8_t l = p_llr(bk, mb, nw);
      p_beta_step(o, x, y);  // beta_k from the normalised beta_{k+1}
      bk = o;
      p_normalize(k, o);
      OUT[q] = l;
    }
  }
}

// ES: the DL-SCH form -- per-block descriptors, skipped blocks, CRC early stop (decode_tb_cb, sch.c:420-456)
template <int NSB, bool ES>
__global__ __launch_bounds__(128) void tdec8bit_kernel(Tdec8Args a)
{
  constexpr int CPW = 64 / NSB;
  extern __shared__ __align__(16) int8_t lds[];
  __shared__ uint32_t passed[CPW];  // ES: the block's CRC passed at this half-iteration (side 0 -> side 1)
  const int      side = threadIdx.x >> 6;  // 0: the alpha wave, 1: the beta wave (map_pass)
  const int      lane = threadIdx.x & 63;
  const int      cb_l = lane / NSB;
  const int      d    = lane % NSB;
  const int      t2   = side * NSB + d;  // this thread's index among the block's 2 NSB (element-wise loops)
  const int      K    = (int)a.K;
  const int      Ls   = K / NSB;
  const int      AL   = (K + 4 + 15) & ~15;
  const uint32_t cb   = blockIdx.x * CPW + cb_l;
  uint32_t       slot = cb;
  bool           live = cb < a.ncb;
  bool           done = false;  // ES: the block's CRC passed (or it was skipped): no more work
  if constexpr (ES) {
    if (live) {
      slot = a.cbs[cb].slot;
      live = slot != TDEC_PAD_SLOT;
    }
    if (live && *a.cbs[cb].skip) {  // CRC already OK in the soft buffer (sch.c:392)
      done = true;
      if (t2 == 0) {
        a.noi_out[slot] = 0;
        a.crc_ok[slot]  = 1;
      }
    }
  }
  live = live && !done;

  int8_t* base = lds + (size_t)cb_l * 6 * AL;
  int8_t* SY   = base;           // systematic
  int8_t* P0   = base + AL;      // parity 0
  int8_t* P1   = base + 2 * AL;  // parity 1
  int8_t* A1   = base + 3 * AL;  // app1
  int8_t* A2   = base + 4 * AL;  // app2
  int8_t* E1   = base + 5 * AL;  // ext1
  // ext2 overwrites app2 in place: DEC 2 reads app2 at a position before it writes ext2 there, each lane
  // only its own sub-block's positions, and app2's tail (read by the tail trellis) is never written
  int8_t* E2   = A2;

  // ---- input streams (turbodecoder_iter.h:61-96 / win.h:880-923) ----
  if (live) {
    const int8_t* in = ES ? reinterpret_cast<const int8_t*>(a.cbs[cb].in) : a.in + (size_t)cb * a.in_stride;
    if (a.layout_sb) {
      for (int q = t2; q < K; q += 2 * NSB) {
        SY[q] = in[q];
        P0[q] = in[K + 32 + q];
        P1[q] = in[2 * (K + 32) + q];
      }
      if (t2 < 3) {
        const int t = 3 * (K + 32) + 2 * d;
        SY[K + d] = in[t];
        P0[K + d] = in[t + 1];
        A2[K + d] = in[t + 6];
        P1[K + d] = in[t + 7];
      }
    } else {
      for (int i = side; i < Ls; i += 2) {
        const int q = i * NSB + d, n = i + d * Ls;
        SY[q] = in[3 * n];
        P0[q] = in[3 * n + 1];
        P1[q] = in[3 * n + 2];
      }
      if (t2 < 3) {
        const int t = 3 * K + 2 * t2;
        SY[K + d] = in[t];
        P0[K + d] = in[t + 1];
        A2[K + d] = in[t + 6];
        P1[K + d] = in[t + 7];
      }
    }
  }
  __syncthreads();

  uint2* beta = a.beta + (size_t)cb * (Ls + 1) * NSB;
  const int nbytes = K / 8;
  for (int n = 0; n < a.n_end; n++) {
    if ((n & 1) == 0) {
      if (n && live) {
        for (int q = t2; q < K; q += 2 * NSB) {
          A1[q] = (int8_t)ssub(A1[q], E1[q]);  // srsran_vec_sub_bbb (saturating for K % 16 == 0)
        }
      }
      __syncthreads();
      map_pass<NSB>(SY, n ? A1 : nullptr, P0, E1, d, Ls, K, beta, side, live);
      __syncthreads();
    } else {
      if (n > 1 && live) {
        for (int q = t2; q < K; q += 2 * NSB) {
          E1[q] = (int8_t)ssub(E1[q], A1[q]);
        }
      }
      __syncthreads();
      if (live) {
        // app2[deinter[i]] = ext1[i]  <=>  app2[j] = ext1[forward[j]]  (srsran_vec_lut_bbb)
        for (int j = t2; j < K; j += 2 * NSB) {
          A2[j] = E1[a.qpp[j]];
        }
      }
      __syncthreads();
      map_pass<NSB>(A2, nullptr, P1, E2, d, Ls, K, beta, side, live);
      __syncthreads();
      if (live) {
        // app1[inter[i]] = ext2[i]
        for (int i = t2; i < K; i += 2 * NSB) {
          A1[a.qpp[i]] = E2[i];
        }
      }
      __syncthreads();
    }
    if constexpr (ES) {
      // decision of this half-iteration (tdec_decision_byte after srsran_tdec_iteration_8bit) and the block's CRC
      // (sch.c:433-456): lane d decides a contiguous byte range, CRCs it from zero, and the ranges combine by
      // x^(8 * bytes after) (crc24_dev.h); the first CRC pass at >= min_iters half-iterations stops the block
      const bool last = n + 1 == a.n_end;
      const bool chk  = n + 1 >= a.min_iters;
      if (live && (chk || last) && side == 0) {  // the alpha wave decides, CRCs and reports; the beta wave follows
        const int8_t*  src = ((n + 1) & 1) ? E1 : A1;
        uint8_t*       out = a.out + (size_t)slot * a.out_stride;
        const int      bpl = (nbytes + NSB - 1) / NSB;
        const int      b0 = min(d * bpl, nbytes), b1 = min(b0 + bpl, nbytes);
        const bool     crc_a = a.cbs[cb].crc_a != 0;
        const uint32_t poly  = crc_a ? LTE_CRC24A : LTE_CRC24B;
        uint32_t       crc   = 0;
        for (int byte = b0; byte < b1; byte++) {
          uint32_t v = 0;
#pragma unroll
          for (int b = 0; b < 8; b++) {
            const int m = byte * 8 + b;
            v |= (src[(m % Ls) * NSB + m / Ls] > 0 ? 1u : 0u) << (7 - b);
          }
          out[byte] = (uint8_t)v;
          crc       = crc24_byte(crc, v, poly);
        }
        uint32_t part = b0 < b1 ? clmul_mod24(crc, (crc_a ? a.xpow_a : a.xpow_b)[nbytes - b1], poly) : 0u;
#pragma unroll
        for (int off = 1; off < NSB; off <<= 1) {
          part ^= (uint32_t)__shfl_xor((int)part, off, 64);
        }
        if (d == 0) {
          passed[cb_l] = chk && part == 0;
          if (chk && part == 0) {
            a.noi_out[slot] = (uint8_t)(n + 1);
            a.crc_ok[slot]  = 1;
          } else if (last) {
            a.noi_out[slot] = (uint8_t)a.n_end;
            a.crc_ok[slot]  = 0;
          }
        }
      }
      __syncthreads();
      if (live && (chk || last) && passed[cb_l]) {
        done = true;
        live = false;
      }
      if (__syncthreads_or(live ? 1 : 0) == 0) {
        break;  // every block of the workgroup is done
      }
    }
  }
  if constexpr (ES) {
    return;  // the decisions were written above
  }

  // ---- decision (turbodecoder.c:370-378, win.h:973-993): bit n = latest(SB slot of n) > 0 ----
  if (live) {
    const int8_t* src = (a.n_end & 1) ? E1 : A1;
    uint8_t*      out = a.out + (size_t)cb * (K / 8);
    for (int byte = t2; byte < K / 8; byte += 2 * NSB) {
      uint32_t v = 0;
#pragma unroll
      for (int b = 0; b < 8; b++) {
        const int n = byte * 8 + b;
        v |= (src[(n % Ls) * NSB + n / Ls] > 0 ? 1u : 0u) << (7 - b);
      }
      out[byte] = (uint8_t)v;
    }
  }
}

// convert_8_to_16 (turbodecoder.c:438-444) over ncb blocks: int8 rows of in_stride bytes -> int16 rows of len
__global__ void tdec8bit_widen_kernel(const int8_t* in, uint32_t in_stride, short* out, uint32_t len, uint32_t ncb)
{
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < (size_t)len * ncb) {
    const size_t b = i / len, j = i % len;
    out[i]         = in[b * in_stride + j];
  }
}

__global__ void rm8_rx_kernel(const int8_t* e, int8_t* sb, const uint16_t* inv, uint32_t E, uint32_t len, uint32_t N)
{
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < len && inv[p] != 0xFFFFu) {
    int acc = sb[p];
    for (uint32_t k = inv[p]; k < E; k += N) {
      acc += e[k];
    }
    sb[p] = (int8_t)acc;  // output[l] += x on int8 (rm_turbo.c:576-579)
  }
}

// the batch form: grid (positions / 256, slot)
__global__ void rm8_rx_slots_kernel(const RmSlot* __restrict__ slots)
{
  const RmSlot&  r = slots[blockIdx.y];
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= r.len || (!r.overwrite && *r.skip)) {
    return;
  }
  const uint32_t start = r.inv[p];
  if (start == 0xFFFFu) {
    return;
  }
  const int8_t* e   = reinterpret_cast<const int8_t*>(r.e);
  int8_t*       sb  = reinterpret_cast<int8_t*>(r.sb);
  int           acc = r.overwrite ? 0 : sb[p];  // a new transmission starts from the reset (zero) buffer
  for (uint32_t k = start; k < r.E; k += r.N) {
    acc += e[k];
  }
  sb[p] = (int8_t)acc;
}

__global__ void widen8_kernel(const Widen8* __restrict__ items)
{
  const Widen8&  w = items[blockIdx.y];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < w.len) {
    w.dst[i] = w.src[i];
  }
}

}  // namespace

hipError_t rm8_rx_slots_launch(const RmSlot* d_slots, uint32_t nslots, uint32_t max_len, hipStream_t stream)
{
  if (nslots == 0 || max_len == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(rm8_rx_slots_kernel, dim3((max_len + 255) / 256, nslots), dim3(256), 0, stream, d_slots);
  return hipGetLastError();
}

hipError_t widen8_launch(const Widen8* d_items, uint32_t n, uint32_t max_len, hipStream_t stream)
{
  if (n == 0 || max_len == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(widen8_kernel, dim3((max_len + 255) / 256, n), dim3(256), 0, stream, d_items);
  return hipGetLastError();
}

hipError_t rm8_rx_launch(const int8_t* e, int8_t* sb, const uint16_t* inv, uint32_t E, uint32_t len, uint32_t N,
                         hipStream_t stream)
{
  hipLaunchKernelGGL(rm8_rx_kernel, dim3((len + 255) / 256), dim3(256), 0, stream, e, sb, inv, E, len, N);
  return hipGetLastError();
}

hipError_t tdec8bit_widen(const int8_t* in, uint32_t in_stride, short* out, uint32_t len, uint32_t ncb,
                          hipStream_t stream)
{
  const size_t n = (size_t)len * ncb;
  hipLaunchKernelGGL(tdec8bit_widen_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, in, in_stride, out,
                     len, ncb);
  return hipGetLastError();
}

size_t tdec8bit_lds_bytes(int nsb, uint32_t K) { return (size_t)(64 / nsb) * 6 * ((K + 4 + 15) & ~15u); }
size_t tdec8bit_beta_bytes(int nsb, uint32_t K, uint32_t ncb) { return (size_t)ncb * (K / nsb + 1) * nsb * 8; }

hipError_t tdec8bit_launch(int nsb, const Tdec8Args& a, hipStream_t stream)
{
  if ((nsb != 16 && nsb != 32) || a.K % nsb || a.K / nsb < (uint32_t)OVL || a.ncb == 0) {
    return hipErrorInvalidValue;
  }
  const uint32_t cpw  = 64 / nsb;
  const dim3     grid((a.ncb + cpw - 1) / cpw);
  const size_t   lds  = tdec8bit_lds_bytes(nsb, a.K);
  if (a.cbs) {
    if (nsb == 16) {
      hipLaunchKernelGGL((tdec8bit_kernel<16, true>), grid, dim3(128), lds, stream, a);
    } else {
      hipLaunchKernelGGL((tdec8bit_kernel<32, true>), grid, dim3(128), lds, stream, a);
    }
  } else if (nsb == 16) {
    hipLaunchKernelGGL((tdec8bit_kernel<16, false>), grid, dim3(128), lds, stream, a);
  } else {
    hipLaunchKernelGGL((tdec8bit_kernel<32, false>), grid, dim3(128), lds, stream, a);
  }
  return hipGetLastError();
}

}  // namespace srsran_amd
