// srsran_4g_amd/csrc/tdec1s_kernel.hip -- LTE turbo decoder for K <= 400 (the generic decoder), ONE LANE
// PER CODE BLOCK AND DIRECTION.
//
// Bit-exact with srsRAN_4G's generic decoder (turbodecoder_gen.c:58-236: no sub-blocks, int16
// wrap-around arithmetic, normalisation every 4 positions, the tail steps inside the backward pass)
// driven by the half-iteration loop of turbodecoder_iter.h:72-144 on the natural input layout
// (3K + 12 values: (systematic, parity0, parity1) per position, then the tails; rm_turbo.c:403-425
// keeps K <= 400 natural).
//
// Mapping: the 8 states of a code block's forward (alpha) recursion in one lane of wave 0, those of its
// backward (beta) recursion in one lane of wave 1, four packed int16 registers each, with the trellis
// step of tdecs_kernel.hip (the same 10 v_pk_add / v_pk_max + 4 v_perm for both directions), here with
// wrapping adds.  A workgroup is 64 code blocks of one K; every lane of a wave works on the same
// position of its own block, so the QPP slots of the second constituent decoder are wave-uniform
// (scalar loads) and the a-priori array S of each block (LDS) is read and written at one offset
// by all lanes (no bank conflicts from the interleaver).
//
// Schedule per half-iteration (the crossover of tdec16_kernel.hip over the whole block instead of a
// sub-block): phase 1: alpha over windows [0, h) storing window-entry checkpoints || beta from the
// end of the tail down to window h storing window-top checkpoints; phase 2: alpha over [h, Ma) with
// beta recomputed per window from its checkpoint, LLRs || beta over [0, h) with alpha recomputed per
// window, LLRs.  W = 16 positions a window.
//
// LDS of a workgroup, every array interleaved over its 64 code blocks ([position][block]) so that the
// lanes of a wave, all at one position, touch consecutive words: S [K][64] int16 | CK [M][64] 16 B
// (alpha window-entry checkpoints for windows < h, beta window-top checkpoints from h) |
// BITS [K/32][64] dwords | RED [2][64].
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc24_dev.h"
#include "stage_timing.h"
#include "tdec_kernel.h"

namespace srsran_amd {
namespace tdecs1 {
namespace {

typedef short v2s __attribute__((ext_vector_type(2)));

constexpr int   W    = 16;      // window
constexpr short NEG  = -10000;  // -INF (turbodecoder_gen.c)
constexpr int   CPWG = 64;      // code blocks per workgroup (one lane each per wave)

__device__ __forceinline__ v2s u2v(uint32_t u) { return __builtin_bit_cast(v2s, u); }
__device__ __forceinline__ uint32_t v2u(v2s v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ v2s lo2(v2s a) { return __builtin_shufflevector(a, a, 0, 0); }
__device__ __forceinline__ v2s hi2(v2s a) { return __builtin_shufflevector(a, a, 1, 1); }
__device__ __forceinline__ v2s swp(v2s a) { return __builtin_shufflevector(a, a, 1, 0); }
__device__ __forceinline__ v2s pmax(v2s a, v2s b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ v2s perm(v2s hi_src, v2s lo_src, uint32_t sel)
{
  return u2v(__builtin_amdgcn_perm(v2u(hi_src), v2u(lo_src), sel));
}

// state layouts as tdecs_kernel.hip: alpha (a0,a1)(a7,a6)(a3,a2)(a4,a5), beta (b0,b4)(b7,b3)(b2,b6)(b5,b1)
struct St {
  v2s a, b, c, d;
};
template <bool BETA>
struct Sel {
  static constexpr uint32_t c = BETA ? 0x01000504u : 0x05040100u;
  static constexpr uint32_t d = BETA ? 0x03020706u : 0x07060302u;
};
struct Bm {
  v2s s, x, y;
};
// wrap-around arithmetic (turbodecoder_gen.c): x + y and every candidate in int16 two's complement
__device__ __forceinline__ Bm bm(uint32_t xyw)
{
  const v2s xy = u2v(xyw);
  return Bm{xy + swp(xy), lo2(xy), hi2(xy)};
}
struct Cand {
  v2s c01, c11, c02, c12, c03, c13, c04, c14;
};
__device__ __forceinline__ Cand cand(const St& p, const Bm& m)
{
  Cand c;
  c.c01 = p.a;
  c.c11 = swp(p.a) + m.s;
  c.c02 = p.b;
  c.c12 = swp(p.b) + m.s;
  c.c03 = p.c + m.y;
  c.c13 = swp(p.c) + m.x;
  c.c04 = p.d + m.y;
  c.c14 = swp(p.d) + m.x;
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
template <bool BETA>
__device__ __forceinline__ St step(const St& p, uint32_t xyw)
{
  return next<BETA>(cand(p, bm(xyw)));
}
// LLR = max_s(beta + c1) - max_s(beta + c0), all wrapping (turbodecoder_gen.c:196-214)
__device__ __forceinline__ short llr(const Cand& c, const St& B)
{
  const v2s b1 = B.a, b2 = swp(B.b), b3 = swp(B.d), b4 = B.c;
  const v2s m0 = pmax(pmax(b1 + c.c01, b2 + c.c02), pmax(b3 + c.c03, b4 + c.c04));
  const v2s m1 = pmax(pmax(b1 + c.c11, b2 + c.c12), pmax(b3 + c.c13, b4 + c.c14));
  return (pmax(m1, swp(m1)) - pmax(m0, swp(m0))).x;
}
// normalisation (turbodecoder_gen.c:120-127, 220-227): subtract state 0, wrapping
__device__ __forceinline__ St norm(const St& p)
{
  const v2s z = lo2(p.a);
  return St{p.a - z, p.b - z, p.c - z, p.d - z};
}
__device__ __forceinline__ St known_state() { return St{v2s{0, NEG}, v2s{NEG, NEG}, v2s{NEG, NEG}, v2s{NEG, NEG}}; }

// workgroup LDS layout (dword offsets)
struct Geo {
  int ck_dw, bits_dw, red_dw, total_dw;
};
__host__ __device__ __forceinline__ Geo geo(int K)
{
  Geo       g;
  const int M = (K + 3 + W - 1) / W;
  g.ck_dw     = ((K + 1) / 2) * CPWG;              // S: K int16 x 64 blocks
  g.bits_dw   = g.ck_dw + M * 4 * CPWG;           // CK: M x 16 B x 64
  g.red_dw    = g.bits_dw + ((K + 31) / 32) * CPWG;
  g.total_dw  = g.red_dw + 2 * CPWG;
  return g;
}

typedef short __attribute__((address_space(3)))* lshort;

struct Ctx {
  int             K, N, Ma, M, h;
  const short*    in;    // this block's input (natural layout), global
  const uint16_t* tfwd;  // slot of pi(n), K entries (wave-uniform reads)
  lshort          S;     // this block's column of the a-priori / extrinsic array: S[k * CPWG]
  uint4*          CK;    // this block's column of the checkpoints: CK[m * CPWG]
  uint32_t*       BITS;  // this block's column of the decision bitmap: BITS[w * CPWG]
  short           xt[3], yt[3];  // this half-iteration's tail inputs

  __device__ __forceinline__ short sget(int k) const { return S[k * CPWG]; }
  __device__ __forceinline__ void  sset(int k, short v) const { S[k * CPWG] = v; }
};

__device__ __forceinline__ void ck_put(const Ctx& c, int m, const St& p)
{
  c.CK[m * CPWG] = make_uint4(v2u(p.a), v2u(p.b), v2u(p.c), v2u(p.d));
}
__device__ __forceinline__ St ck_get(const Ctx& c, int m)
{
  const uint4 v = c.CK[m * CPWG];
  return St{u2v(v.x), u2v(v.y), u2v(v.z), u2v(v.w)};
}

// Branch inputs of the window at t0 (positions t0 .. t0 + W - 1, those past the tail unused):
//   DEC1: x = syst + S[k] (wrapping), y = parity0; aux = S[k]       (tail: systematic / parity0 tails)
//   DEC2: x = S[pi(k)], y = parity1; aux = pi(k)                      (tail: app2 / parity1 tails)
template <bool D2>
__device__ __forceinline__ void window_in(const Ctx& c, int t0, uint32_t* xw, uint32_t* aux)
{
  short ya[W], xa[W];
#pragma unroll
  for (int i = 0; i < W; i++) {
    const int k = t0 + i;
    if (k < c.K) {
      ya[i] = c.in[3 * k + (D2 ? 2 : 1)];
      xa[i] = D2 ? (short)0 : c.in[3 * k];
    }
  }
#pragma unroll
  for (int i = 0; i < W; i++) {
    const int k = t0 + i;
    if (k < c.K) {
      if (D2) {
        const uint32_t b = __builtin_amdgcn_readfirstlane((uint32_t)c.tfwd[k]);
        aux[i]           = b;
        xw[i]            = ((uint32_t)(uint16_t)ya[i] << 16) | (uint16_t)c.sget((int)b);
      } else {
        const short s = c.sget(k);
        aux[i]        = (uint16_t)s;
        xw[i]         = ((uint32_t)(uint16_t)ya[i] << 16) | (uint16_t)(short)(xa[i] + s);
      }
    } else if (k < c.N) {
      xw[i] = ((uint32_t)(uint16_t)c.yt[k - c.K] << 16) | (uint16_t)c.xt[k - c.K];
    }
  }
}

// LLR o of position k: S update (vec_sub, wraps) and, when needed, the decision bit (turbodecoder.c:370-378)
template <bool D2, bool BITS>
__device__ __forceinline__ void emit(const Ctx& c, int k, short o, uint32_t aux)
{
  const int   slot = D2 ? (int)aux : k;
  const short old  = D2 ? c.sget(slot) : (short)aux;  // DEC1: S[k] as read for the branch input
  c.sset(slot, (short)(o - old));
  if (BITS) {
    const int n = slot;
    atomicOr(&c.BITS[(n >> 5) * CPWG], (uint32_t)(o > 0) << (((n >> 3) & 3) * 8 + 7 - (n & 7)));
  }
}

// beta positions normalise at k % 4 == 0 && k < K; alpha after position j when (j + 1) % 4 == 0
__device__ __forceinline__ bool bnorm(int k, int K) { return (k & 3) == 0 && k < K; }

template <bool D2, bool BITS>
__device__ __forceinline__ void map1s(const Ctx& c, int wave)
{
  uint32_t xw[W], aux[W];
  const int K = c.K, N = c.N, h = c.h;
  if (wave == 0) {
    // ================= alpha side =================
    St P = known_state();
    // phase 1: windows [0, h), entry checkpoints
#pragma unroll 1
    for (int m = 0; m < h; m++) {
      const int t0 = m * W;
      window_in<D2>(c, t0, xw, aux);
      ck_put(c, m, P);
#pragma unroll
      for (int i = 0; i < W; i++) {
        if (t0 + i < K) {
          P = step<false>(P, xw[i]);
          if (((t0 + i + 1) & 3) == 0) P = norm(P);
        }
      }
    }
    __syncthreads();
    // phase 2: windows [h, Ma): beta of the window recomputed from its top checkpoint, then alpha + LLR
#pragma unroll 1
    for (int m = h; m < c.Ma; m++) {
      const int t0  = m * W;
      const int top = min(t0 + W, N);
      window_in<D2>(c, t0, xw, aux);
      St Pb = ck_get(c, m);
      St bw[W];  // bw[i] = stored beta at t0 + i + 1
#pragma unroll
      for (int i = W - 1; i >= 0; i--) {
        const int k = t0 + i + 1;  // position whose stored beta bw[i] is
        if (k == top) {
          bw[i] = Pb;
          if (bnorm(k, K)) Pb = norm(Pb);
        } else if (k < top) {
          Pb    = step<true>(Pb, xw[i + 1]);
          bw[i] = Pb;
          if (bnorm(k, K)) Pb = norm(Pb);
        }
      }
#pragma unroll
      for (int i = 0; i < W; i++) {
        const int j = t0 + i;
        if (j < K) {
          const Cand  cd = cand(P, bm(xw[i]));
          const short o  = llr(cd, bw[i]);
          P              = next<false>(cd);
          if (((j + 1) & 3) == 0) P = norm(P);
          emit<D2, BITS>(c, j, o, aux[i]);
        }
      }
    }
  } else {
    // ================= beta side =================
    St P = known_state();  // beta at N = K + 3: state 0 (turbodecoder_gen.c:102-107)
    St Bst = P;            // stored beta of the position above the current window
    // phase 1: windows [M - 1 .. h] from the end of the tail; the stored beta at each window's bottom
    // is the top checkpoint of the window below
    ck_put(c, c.M - 1, P);
#pragma unroll 1
    for (int m = c.M - 1; m >= h; m--) {
      const int t0 = m * W;
      window_in<D2>(c, t0, xw, aux);
#pragma unroll
      for (int i = W - 1; i >= 0; i--) {
        const int k = t0 + i;
        if (k < N) {
          P = step<true>(P, xw[i]);
          if (i == 0) {
            Bst = P;
            if (m - 1 >= h) {
              ck_put(c, m - 1, P);  // below h the slots hold the alpha checkpoints
            }
          }
          if (bnorm(k, K)) P = norm(P);
        }
      }
    }
    __syncthreads();
    // phase 2: windows [h - 1 .. 0]: alpha recomputed from the entry checkpoint, beta + LLR backwards
#pragma unroll 1
    for (int m = h - 1; m >= 0; m--) {
      const int t0 = m * W;
      window_in<D2>(c, t0, xw, aux);
      St Pa = ck_get(c, m);
      St aw[W];
#pragma unroll
      for (int i = 0; i < W; i++) {
        aw[i] = Pa;
        if (i < W - 1) {
          Pa = step<false>(Pa, xw[i]);
          if (((t0 + i + 1) & 3) == 0) Pa = norm(Pa);
        }
      }
#pragma unroll
      for (int i = W - 1; i >= 0; i--) {
        const int   k = t0 + i;
        const short o = llr(cand(aw[i], bm(xw[i])), Bst);
        P             = step<true>(P, xw[i]);
        Bst           = P;
        if (bnorm(k, K)) P = norm(P);
        emit<D2, BITS>(c, k, o, aux[i]);
      }
    }
  }
}

// decision byte b of this lane's block (MSB first, as the bitmap stores it)
__device__ __forceinline__ uint32_t dbyte(const Ctx& c, int b) { return (c.BITS[(b >> 2) * CPWG] >> (8 * (b & 3))) & 0xffu; }

}  // namespace

template <bool ES>
__device__ __forceinline__ void body(const TdecArgs& a, int bid)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int  lane = threadIdx.x & 63;
  const int  wave = threadIdx.x >> 6;
  const int  K    = (int)a.K;
  const Geo  g    = geo(K);
  const int  cb   = bid * CPWG + lane;
  const int  cbl  = cb < (int)a.ncb ? cb : (int)a.ncb - 1;
  const bool live = cb < (int)a.ncb && (!ES || a.cbs[cbl].slot != TDEC_PAD_SLOT);
  bool       done = ES && (!live || *a.cbs[cbl].skip);

  Ctx       c;
  c.K    = K;
  c.N    = K + 3;
  c.Ma   = (K + W - 1) / W;
  c.M    = (K + 3 + W - 1) / W;
  c.h    = max(1, min(c.Ma - 1, (c.M + 1) / 2));
  c.in   = ES ? a.cbs[cbl].in : a.in + (size_t)cbl * a.in_stride;
  c.tfwd = a.tfwd_nat;
  c.S    = (lshort)(short*)smem + lane;
  c.CK   = reinterpret_cast<uint4*>(smem + g.ck_dw) + lane;
  c.BITS = smem + g.bits_dw + lane;
  uint32_t* RED = smem + g.red_dw + lane;  // RED[wave * CPWG]

  if constexpr (ES) {
    if (live && done && wave == 0) {  // skipped block (sch.c:392, 476-480)
      const uint32_t slot = a.cbs[cbl].slot;
      a.noi_out[slot]     = 0;
      a.crc_ok[slot]      = 1;
    }
  }
  for (int i = threadIdx.x; i < g.ck_dw; i += 128) {  // S = 0
    smem[i] = 0u;
  }
  const int h_end = (ES && __syncthreads_or(!done) == 0) ? 0 : a.n_end;
  // tails of the natural layout: systematic / parity0 (DEC1), app2 / parity1 (DEC2) (turbodecoder.c)
  const short* tail = c.in + 3 * K;

#pragma unroll 1
  for (int hi = 0; hi < h_end; hi++) {
    const bool crc_now = ES && hi + 1 >= a.min_iters;
    for (int i = g.bits_dw + threadIdx.x; i < g.red_dw; i += 128) {
      smem[i] = 0u;
    }
    const bool d2 = hi & 1;
#pragma unroll
    for (int t = 0; t < 3; t++) {
      c.xt[t] = tail[(d2 ? 6 : 0) + 2 * t];
      c.yt[t] = tail[(d2 ? 6 : 0) + 2 * t + 1];
    }
    __syncthreads();
    const bool bits = ES ? crc_now : hi + 1 == h_end;
    if (d2) {
      if (bits) {
        map1s<true, true>(c, wave);
      } else {
        map1s<true, false>(c, wave);
      }
    } else {
      if (bits) {
        map1s<false, true>(c, wave);
      } else {
        map1s<false, false>(c, wave);
      }
    }
    __syncthreads();

    if constexpr (ES) {
      if (crc_now) {
        // the block's decision bytes, half a side: CRC of each half from zero, the first moved by
        // x^(8 * bytes after it), XOR (crc24_dev.h)
        const int      nbytes = K / 8;
        const int      b0     = wave ? nbytes / 2 : 0;
        const int      b1     = wave ? nbytes : nbytes / 2;
        const bool     crc_a  = a.cbs[cbl].crc_a;
        const uint32_t poly   = crc_a ? LTE_CRC24A : LTE_CRC24B;
        uint32_t       crc    = 0;
#pragma unroll 1
        for (int b = b0; b < b1; b++) {
          crc = crc24_byte(crc, dbyte(c, b), poly);
        }
        RED[wave * CPWG] = b0 < b1 ? clmul_mod24(crc, (crc_a ? a.xpow_a : a.xpow_b)[nbytes - b1], poly) : 0u;
        __syncthreads();
        const bool ok = (RED[0] ^ RED[CPWG]) == 0;
        if (ok && !done && live) {
          const uint32_t slot = a.cbs[cbl].slot;
          uint8_t*       out  = a.out + (size_t)slot * a.out_stride;
          for (int b = b0; b < b1; b++) {
            out[b] = dbyte(c, b);
          }
          if (wave == 0) {
            a.noi_out[slot] = (uint8_t)(hi + 1);
            a.crc_ok[slot]  = 1;
          }
        }
        done = done || ok;
      }
      if (__syncthreads_or(!done) == 0) {
        break;
      }
    }
  }

  if (live && !done && h_end > 0) {
    const int      cbm    = ES ? (int)a.cbs[cbl].slot : cbl;
    uint8_t*       out    = a.out + (size_t)cbm * (ES ? a.out_stride : K / 8);
    const int      nbytes = K / 8;
    for (int b = wave ? nbytes / 2 : 0; b < (wave ? nbytes : nbytes / 2); b++) {
      out[b] = dbyte(c, b);
    }
    if (ES && wave == 0) {
      a.noi_out[cbm] = (uint8_t)a.n_end;
      a.crc_ok[cbm]  = 0;
    }
  }
}

template <bool ES>
__global__ __launch_bounds__(128, 1) void tdec1s_kernel(TdecArgs a)
{
  body<ES>(a, blockIdx.x);
}

__global__ __launch_bounds__(128, 1) void tdec1s_multi_kernel(const TdecArgs* __restrict__ groups,
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
  body<false>(a, (int)(b - first[lo]));
}

size_t lds_bytes(const TdecArgs& a) { return (size_t)geo((int)a.K).total_dw * 4; }

int cpw() { return CPWG; }

hipError_t launch(const TdecArgs& a, hipStream_t stream)
{
  StageScope timing_scope(ST_TDEC, stream);
  const int    grid = (a.ncb + CPWG - 1) / CPWG;
  const size_t lds  = lds_bytes(a);
  tdec_set_last_kernel(a.cbs ? "tdec1s_kernel<true>" : "tdec1s_kernel<false>");
  if (a.cbs) {
    hipLaunchKernelGGL((tdec1s_kernel<true>), dim3(grid), dim3(128), lds, stream, a);
  } else {
    hipLaunchKernelGGL((tdec1s_kernel<false>), dim3(grid), dim3(128), lds, stream, a);
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
  tdec_set_last_kernel("tdec1s_multi_kernel");
  hipLaunchKernelGGL(tdec1s_multi_kernel, dim3(nblocks), dim3(128), lds, stream, d_groups, d_first, ngroups);
  return hipGetLastError();
}

}  // namespace tdecs1
}  // namespace srsran_amd
