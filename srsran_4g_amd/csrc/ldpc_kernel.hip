// srsran_4g_amd/csrc/ldpc_kernel.hip -- NR LDPC decoder (layered normalised min-sum, 8-bit
// messages) for CDNA4 (gfx950).
//
// Bit-exact with srsRAN's 8-bit decoders: ldpc_decoder.c:44-95 (driver, CRC early stop),
// ldpc_dec_c.c:171-319 (SRSRAN_LDPC_DECODER_C: scaling m*s100/100) and
// ldpc_dec_c_avx2.c / _avx2long.c / _avx512*.c (SRSRAN_LDPC_DECODER_C_AVX2 / _AVX512: scaling
// (m * (uint16)((s + 2^-16) * 65535)) >> 16, _mm256_scalei_epi8).
//
// Mapping: one thread per lifted check node z of the current layer, ls threads per codeword,
// several codewords per workgroup for small lifting sizes.
//   * soft bits (a-posteriori LLRs) of the codeword live in LDS as int8, column c at c*CS
//     (CS = compile-time column stride >= ls, so every column offset folds into the LDS
//     instruction's immediate).  Check z of a layer reads / writes position (z + shift) mod ls
//     of every connected column: within a layer every soft bit belongs to exactly one thread,
//     so a layer needs no synchronisation, only a barrier between layers.
//   * check-to-variable messages are never stored per edge: a thread keeps, for each layer,
//     its check node's compressed min-sum state in VGPRs -- scaled min1 / min2 (7 bits each),
//     the index of the min1 edge (5 bits) and one sign bit per edge -- one dword per layer
//     (two for the four degree-19 rows of BG1).  c2v of edge k = +-(k == idx ? min2 : min1),
//     exactly the values the reference stores in check_to_var.
//   * the base graph topology (columns, degrees) is compile time: every layer is unrolled, so
//     the state array is statically indexed and stays in registers; the lifting size's shifts
//     are copied to LDS once and read as broadcasts with immediate offsets.
// Built twice (Makefile): -DLDPC_BG_ONLY=0 (BG1 kernels + the host launch helpers) and =1 (BG2),
// so the twelve instantiations compile in parallel.
//   * CRC early stop (decode_crc_c): after every iteration each thread CRCs its K contiguous
//     hard bits from zero, moves the CRC to its place with x^(bits after) mod P and the parts
//     XOR together in LDS; zero <=> srsran_crc_match over liftK bits.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "ldpc_kernel.h"
#include "stage_timing.h"

#ifndef LDPC_BG_ONLY
#error "build with -DLDPC_BG_ONLY=0 (BG1) or 1 (BG2)"
#endif
#define LDPC_TBL static constexpr
#include "ldpc_bg_tables.inc"

namespace srsran_amd {

template <int BG>
struct Topo;
template <>
struct Topo<0> {
  static constexpr int                   M = 46, N = 68, K = 22;
  static constexpr const unsigned short* rs  = LDPC_BG1_ROW_START;
  static constexpr const unsigned char*  col = LDPC_BG1_COL;
};
template <>
struct Topo<1> {
  static constexpr int                   M = 42, N = 52, K = 10;
  static constexpr const unsigned short* rs  = LDPC_BG2_ROW_START;
  static constexpr const unsigned char*  col = LDPC_BG2_COL;
};

template <int BG>
constexpr int deg_of(int l)
{
  return Topo<BG>::rs[l + 1] - Topo<BG>::rs[l];
}

static constexpr int PK_ONE_WORD_MAX_DEG = 11;  // signs of both checks + 5-bit indices in one dword

template <int BG>
constexpr int words_before_pk(int L)
{
  int w = 0;
  for (int l = 0; l < L; ++l) {
    w += deg_of<BG>(l) > PK_ONE_WORD_MAX_DEG ? 3 : 2;
  }
  return w;
}

// Arithmetic of the one-check-per-thread path: 8-bit (ldpc_dec_c.c / _avx2*.c) or 16-bit
// (ldpc_dec_s.c: 15-bit messages, soft-bit infinity INT16_MAX) messages and their VGPR state.
template <typename E>
struct Ar;
template <>
struct Ar<int8_t> {
  static constexpr int INF_MSG = 63, INF_SOFT = 127;  // infinity7, INT8_MAX (ldpc_dec_c.c:52, 292)
  // state: s1 | s2 << 7 | idx << 14 | signs << 19 (one dword up to degree 13, else signs apart)
  static constexpr int words(int deg) { return deg > 13 ? 2 : 1; }
};
template <>
struct Ar<int16_t> {
  static constexpr int INF_MSG = 16383, INF_SOFT = 32767;  // infinity15, INT16_MAX (ldpc_dec_s.c:52, 318)
  // state: s1 | s2 << 16, idx | signs << 5
  static constexpr int words(int) { return 2; }
};

template <int BG, typename E>
constexpr int words_before_e(int L)
{
  int w = 0;
  for (int l = 0; l < L; ++l) {
    w += Ar<E>::words(deg_of<BG>(l));
  }
  return w;
}

template <typename E>
struct Lane {
  E*              soft;  // this codeword's soft bits (LDS), column stride CS
  const uint32_t* sh;    // shift of every edge for this lifting size (LDS copy)
  int             z;     // lifted check index
  int             ls;
  bool            busy;  // decodes this layer (live codeword, CRC not yet matched)
  int             n_layers;     // this codeword's layers
  int             n_layers_wg;  // the workgroup's largest (barrier count)
  int             scale_mode;
  int             sf;
};

template <typename E>
__device__ __forceinline__ int scale_mag(const Lane<E>& ln, int m)
{
  // _mm256_scalei_epi8: mulhi_epu16 of the (non-negative) byte by sf; ldpc_dec_c.c: m*sf/100
  return ln.scale_mode == LDPC_SCALE_SIMD ? (int)(((uint32_t)m * (uint32_t)ln.sf) >> 16) : m * ln.sf / 100;
}

// One layer (row L of the base graph) for this thread's check node.
template <int BG, int CS, typename E, int L, int NW>
__device__ __forceinline__ void run_layer(const Lane<E>& ln, uint32_t (&st)[NW])
{
  using T               = Topo<BG>;
  using A               = Ar<E>;
  constexpr int  e0     = T::rs[L];
  constexpr int  deg    = deg_of<BG>(L);
  constexpr int  w0     = words_before_e<BG, E>(L);
  constexpr bool is8    = sizeof(E) == 1;
  constexpr bool two    = A::words(deg) == 2;
  if (L >= ln.n_layers_wg) {
    return;
  }
  __syncthreads();  // soft bits written by the previous layer
  if (!ln.busy || L >= ln.n_layers) {
    return;
  }
  // Opaque per-layer copy: without it LICM hoists every edge's address (316 VGPRs) out of the
  // iteration loop and the kernel spills.
  int zz = ln.z;
  asm volatile("" : "+v"(zz));
  const uint32_t* shp = ln.sh + e0;  // LDS: broadcast reads with immediate offsets
  const int       ls  = ln.ls;

  int      o1, o2, oix;
  uint32_t sg;
  if constexpr (is8) {
    const uint32_t s0 = st[w0];
    sg                = two ? st[w0 + 1] : (s0 >> 19);
    o1                = (int)(s0 & 127u);
    o2                = (int)((s0 >> 7) & 127u);
    oix               = (int)((s0 >> 14) & 31u);
  } else {
    o1  = (int)(st[w0] & 0xFFFFu);
    o2  = (int)(st[w0] >> 16);
    oix = (int)(st[w0 + 1] & 31u);
    sg  = st[w0 + 1] >> 5;
  }

  int      v2c[deg];
  uint32_t pos[deg];
  int      m1 = A::INF_SOFT, m2 = A::INF_SOFT, mi = 0;  // INT8_MAX / INT16_MAX start (ldpc_dec_c.c:223-228)
  int      px = 0;                                      // XOR of all v2c: its sign = product of signs
#pragma unroll
  for (int k = 0; k < deg; ++k) {
    const int      col = T::col[e0 + k];
    const uint32_t p   = (uint32_t)zz + shp[k];
    pos[k]             = min(p, p - (uint32_t)ls);  // (z + shift) mod ls
    __builtin_assume(pos[k] < (uint32_t)CS);
    const int x        = ln.soft[col * CS + pos[k]];
    // previous c2v of this edge: +-(k == idx ? min2 : min1)
    const int mag = k == oix ? o2 : o1;
    const int sgn = -(int)((sg >> k) & 1u);
    const int c   = (mag ^ sgn) - sgn;
    // inner_var_to_check: |x| >= INF_SOFT propagates as +-INF_SOFT, else clip(x - c) to +-INF_MSG
    const int vn = min(max(x - c, -A::INF_MSG), A::INF_MSG);
    int       v;
    if constexpr (is8) {
      v = (uint32_t)(x + 126) > 252u ? (x | 1) : vn;
    } else {
      v = (x >= A::INF_SOFT || x <= -A::INF_SOFT) ? min(max(x, -A::INF_SOFT), A::INF_SOFT) : vn;
    }
    v2c[k]         = v;
    const int  av  = max(v, -v);
    const bool lt  = av < m1;                // strict: the first minimum keeps the index
    m2             = min(max(m1, av), m2);   // = med3(m1, m2, av) for m1 <= m2
    mi             = lt ? k : mi;
    m1             = min(m1, av);
    px ^= v;
  }
  const int s1   = scale_mag(ln, m1);
  const int s2   = scale_mag(ln, m2);
  const int prod = px >> 31;  // -1 if the product of the signs is negative
  uint32_t  csg  = 0;
#pragma unroll
  for (int k = 0; k < deg; ++k) {
    const int col = T::col[e0 + k];
    const int mag = k == mi ? s2 : s1;
    const int sgn = (prod ^ v2c[k]) >> 31;  // sign of c2v_k = prod ^ sign(v2c_k)
    const int c   = (mag ^ sgn) - sgn;
    csg |= (uint32_t)(sgn & 1) << k;
    const int t = c + v2c[k];  // update_ldpc_soft_bits: beyond +-INF_MSG -> +-INF_SOFT
    const int r = (uint32_t)(t + A::INF_MSG) > (uint32_t)(2 * A::INF_MSG) ? A::INF_SOFT * ((t >> 31) | 1) : t;
    ln.soft[col * CS + pos[k]] = (E)r;
  }
  if constexpr (is8) {
    const uint32_t w = (uint32_t)s1 | ((uint32_t)s2 << 7) | ((uint32_t)mi << 14);
    if constexpr (two) {
      st[w0]     = w;
      st[w0 + 1] = csg;
    } else {
      st[w0] = w | (csg << 19);
    }
  } else {
    st[w0]     = (uint32_t)s1 | ((uint32_t)s2 << 16);
    st[w0 + 1] = (uint32_t)mi | (csg << 5);
  }
}

template <int BG, int CS, typename E, int NW, int... Ls>
__device__ __forceinline__ void run_iteration(const Lane<E>& ln, uint32_t (&st)[NW], std::integer_sequence<int, Ls...>)
{
  (run_layer<BG, CS, E, Ls, NW>(ln, st), ...);
}

// ---------------------------------------------------------------------------------------
// Packed path (even ls >= 18): one thread serves the two check nodes z and z + ls/2 of a layer
// with packed 16-bit arithmetic (v_pk_*_i16), so each VALU instruction advances two checks.
// Soft bits stay int8 in LDS; the pair is gathered with ds_read_i8 / ds_read_i8_d16_hi and
// scattered with ds_write_b8 / ds_write_b8_d16_hi.  Per layer and thread the state is
//   M  = bytes (s1a, s2a, s1b, s2b): scaled min1 / min2 of checks a (lo half) and b (hi half)
//   S0 = c2v sign bits of a (bits 0..) | idx_a << 11 | signs of b << 16 | idx_b << 27
//        (degree <= 11; degree 19 rows keep edges 16.. and the indices in a third word S1).
// Input LLRs of -128 load as -127: the reference maps both to -127 in every use (v2c infinity,
// sign of the message), so the two are indistinguishable.
typedef short          v2s __attribute__((ext_vector_type(2)));
typedef unsigned short v2u __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v2s as_s(uint32_t u) { return __builtin_bit_cast(v2s, u); }
__device__ __forceinline__ v2u as_u(uint32_t u) { return __builtin_bit_cast(v2u, u); }
__device__ __forceinline__ uint32_t bits(v2s v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ uint32_t bits(v2u v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ v2s pmin(v2s a, v2s b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ v2s pmax(v2s a, v2s b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ v2s pclamp(v2s a, short lo, short hi) { return pmin(pmax(a, v2s{lo, lo}), v2s{hi, hi}); }
// The 0/1 flags and the multiply-add selects below are written as VOP3P instructions: in plain
// C the compiler turns them into per-half compares + v_cndmask + v_perm (three times the work).
__device__ __forceinline__ uint32_t pk_min1(uint32_t a)  // min(a, 1) per unsigned half
{
  uint32_t r;
  asm("v_pk_min_u16 %0, %1, 1 op_sel_hi:[1,0]" : "=v"(r) : "v"(a));
  return r;
}
__device__ __forceinline__ uint32_t pk_subsat(uint32_t a, uint32_t b)  // max(a - b, 0) per unsigned half
{
  uint32_t r;
  asm("v_pk_sub_u16 %0, %1, %2 clamp" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ v2s pk_mad(v2s a, v2s b, v2s c)  // a * b + c per half (low 16 bits)
{
  uint32_t r;
  asm("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(r) : "v"(bits(a)), "v"(bits(b)), "v"(bits(c)));
  return as_s(r);
}
// 1 where a > b (unsigned halves), else 0
__device__ __forceinline__ v2s pgt01(uint32_t a, uint32_t b) { return as_s(pk_min1(pk_subsat(a, b))); }
// 1 where a != b, else 0
__device__ __forceinline__ v2s pne01(uint32_t a, uint32_t b) { return as_s(pk_min1(a ^ b)); }

// LDS pointers built from integer offsets: the dynamic LDS block starts at address 0 (the kernel
// has no static LDS), and addressing it this way lets every column offset fold into the
// instruction (a generic `smem` symbol would cost an extra v_add per address).
typedef __attribute__((address_space(3))) int8_t lds_i8;

struct LanePk {
  lds_i8*         soft;   // this codeword's soft bits (LDS), column stride CS
  const uint32_t* sh;     // shifts (LDS)
  const uint8_t*  scale;  // scale(m) for m = 0..127 (LDS)
  int             z;      // first check of the pair
  int             ls, h;
  bool            busy;
  int             n_layers;     // this codeword's layers
  int             n_layers_wg;  // the workgroup's largest (barrier count)
};

template <int BG, int CS, int L, int NW>
__device__ __forceinline__ void run_layer_pk(const LanePk& ln, uint32_t (&st)[NW])
{
  using T               = Topo<BG>;
  constexpr int  e0     = T::rs[L];
  constexpr int  deg    = deg_of<BG>(L);
  constexpr int  w0     = words_before_pk<BG>(L);
  constexpr bool two    = deg > PK_ONE_WORD_MAX_DEG;
  if (L >= ln.n_layers_wg) {
    return;
  }
  __syncthreads();  // soft bits written by the previous layer
  if (!ln.busy || L >= ln.n_layers) {
    return;
  }
  int zz = ln.z;
  asm volatile("" : "+v"(zz));
  const uint32_t* shp = ln.sh + e0;
  const uint32_t  ls  = (uint32_t)ln.ls;
  const uint32_t  h   = (uint32_t)ln.h;

  const uint32_t M   = st[w0];
  const uint32_t S0  = st[w0 + 1];
  const uint32_t SI  = two ? st[w0 + 2] : S0;  // word holding the indices
  const v2s      P1  = as_s(M & 0x00FF00FFu);
  const v2s      P2  = as_s((M >> 8) & 0x00FF00FFu);
  const v2s      D1  = P1 - P2;
  const v2u      IDX = as_u(SI) >> (unsigned short)11;
  const uint32_t c126 = 0x007E007Eu;

  v2s      v2c[deg];  // first the gathered soft bits, then the v2c messages
  uint32_t pos[deg];
  v2s      m1 = {127, 127}, m2 = {127, 127}, mi = {0, 0};
  v2s      px = {0, 0};
  // gather every edge's pair first: all LDS reads of the layer in flight together
#pragma unroll
  for (int k = 0; k < deg; ++k) {
    const int      col = T::col[e0 + k];
    const uint32_t p   = (uint32_t)zz + shp[k];
    const uint32_t p1  = min(p, p - ls);         // (z + shift) mod ls
    const uint32_t q   = p1 + h;
    const uint32_t p2  = min(q, q - ls);         // (z + ls/2 + shift) mod ls
    __builtin_assume(p1 < (uint32_t)CS);
    __builtin_assume(p2 < (uint32_t)CS);
    pos[k]             = p1 | (p2 << 16);
    const lds_i8* sc   = ln.soft + col * CS;
    v2c[k]             = v2s{(short)sc[p1], (short)sc[p2]};
  }
#pragma unroll
  for (int k = 0; k < deg; ++k) {
    const v2s x = v2c[k];
    // previous c2v: +-(k == idx ? min2 : min1)
    const uint32_t Sw   = (k < 16) ? S0 : SI;
    const int      kk   = k & 15;
    const v2s      smk  = as_s(bits(as_u(Sw) << (unsigned short)(15 - kk))) >> (short)15;
    const v2s      mag  = pk_mad(pne01(bits(IDX), (uint32_t)k * 0x10001u), D1, P2);
    const v2s      xmc  = (x + smk) - (mag ^ smk);  // x - c
    const v2s      vn   = pclamp(xmc, -63, 63);
    const v2s      ax   = pmax(x, -x);
    const v2s      big  = pgt01(bits(ax), c126);  // |x| == 127
    const v2s      v    = pk_mad(big, x - vn, vn);
    v2c[k]              = v;
    const v2s av        = pmax(v, -v);
    const v2s lt        = pgt01(bits(m1), bits(av));  // av < m1
    mi                  = pk_mad(lt, v2s{(short)k, (short)k} - mi, mi);
    m2                  = pmin(pmax(m1, av), m2);
    m1                  = pmin(m1, av);
    px                  = px ^ v;
  }
  // scaled magnitudes through the LDS table (both scaling arithmetics)
  const v2s  S1   = {(short)ln.scale[bits(m1) & 0xFFFFu], (short)ln.scale[bits(m1) >> 16]};
  const v2s  S2   = {(short)ln.scale[bits(m2) & 0xFFFFu], (short)ln.scale[bits(m2) >> 16]};
  const v2s  D2   = S1 - S2;
  const v2s  prod = px >> (short)15;
  uint32_t   acc0 = 0, acc1 = 0;
#pragma unroll
  for (int k = 0; k < deg; ++k) {
    const int      col = T::col[e0 + k];
    const v2s      mag = pk_mad(pne01(bits(mi), (uint32_t)k * 0x10001u), D2, S2);
    const v2s      sgn = (prod ^ v2c[k]) >> (short)15;
    const v2s      c   = (mag ^ sgn) - sgn;
    const uint32_t bk  = (1u << (k & 15)) | (1u << (16 + (k & 15)));
    if (k < 16) {
      acc0 |= bits(sgn) & bk;
    } else {
      acc1 |= bits(sgn) & bk;
    }
    const v2s t  = c + v2c[k];
    const v2s b  = pclamp(t, -63, 63);
    const v2s a2 = pclamp(t, -64, 64);
    const v2s r  = pk_mad(a2 - b, v2s{64, 64}, b);  // beyond +-63 -> +-127
    lds_i8*   sc = ln.soft + col * CS;
    const uint32_t pp = pos[k];
    sc[pp & 0xFFFFu]  = (int8_t)r.x;
    sc[pp >> 16]      = (int8_t)r.y;
  }
  st[w0] = bits(S1) | (bits(S2) << 8);
  const uint32_t iw = bits(__builtin_bit_cast(v2u, mi) << (unsigned short)11);
  if constexpr (two) {
    st[w0 + 1] = acc0;
    st[w0 + 2] = acc1 | iw;
  } else {
    st[w0 + 1] = acc0 | iw;
  }
}

template <int BG, int CS, int NW, int... Ls>
__device__ __forceinline__ void run_iteration_pk(const LanePk& ln, uint32_t (&st)[NW], std::integer_sequence<int, Ls...>)
{
  (run_layer_pk<BG, CS, Ls, NW>(ln, st), ...);
}

// Per-thread view of its codeword: plain batch (one configuration for all) or CB mode (LdpcCw).
struct CwCtx {
  const void*     in;        // this codeword's LLRs
  bool            live;      // decodes (exists, not already decoded)
  int             n_layers;  // this codeword's layers
  const uint32_t* xpow;      // CRC early stop (nullptr: none)
  uint32_t        poly;
  int             order;
};

__device__ __forceinline__ CwCtx cw_ctx(const LdpcArgs& a, uint32_t cw, bool act, int elem_bytes)
{
  CwCtx c;
  const bool exists = act && cw < a.ncw;
  if (a.cws) {
    const LdpcCw& d = a.cws[exists ? cw : 0];
    c.in            = d.in;
    c.live          = exists && *d.flag == 0;
    c.n_layers      = d.n_layers;
    c.xpow          = a.xpow3[d.crc];
    c.poly          = d.crc == 0 ? 0x1800063u : (d.crc == 1 ? 0x1864CFBu : 0x11021u);  // phy_common.h:72-74
    c.order         = d.crc == 2 ? 16 : 24;
  } else {
    c.in       = reinterpret_cast<const char*>(a.in) + (size_t)cw * a.in_stride;
    c.live     = exists;
    c.n_layers = a.n_layers;
    c.xpow     = a.xpow;
    c.poly     = a.crc_poly;
    c.order    = a.crc_order;
  }
  (void)elem_bytes;
  return c;
}

// Largest layer count of the workgroup's codewords (CB mode): every thread reaches every barrier
// of the layers up to it.  `slot` is a dword of dynamic LDS.
__device__ __forceinline__ int wg_layers(const LdpcArgs& a, const CwCtx& c, uint32_t* slot)
{
  if (!a.cws) {
    return a.n_layers;
  }
  if (threadIdx.x == 0) {
    *slot = 0u;
  }
  __syncthreads();
  if (c.live) {
    atomicMax(slot, (uint32_t)c.n_layers);
  }
  __syncthreads();
  return (int)*slot;
}

// CB-mode outputs of one codeword (sch_nr.c:664-690): packed message on CRC success, cb_crc flag,
// iterations; `bit(i)` = hard decision of message bit i.
template <typename F>
__device__ __forceinline__ void cb_finish(const LdpcArgs& a, uint32_t cw, bool exists, const CwCtx& c, int ret,
                                          int t0, int nthreads, F&& bit)
{
  const LdpcCw& d = a.cws[cw];
  if (!exists) {
    return;
  }
  if (!c.live) {  // already decoded in an earlier transmission: untouched, no iterations
    if (t0 == 0) {
      *d.iters = 0;
    }
    return;
  }
  if (ret > 0) {  // srsran_bit_pack_vector(temp_cb, data[r], cb_len): whole bytes, then MSB-aligned rest
    const int nb = (d.cb_len + 7) / 8;
    for (int b = t0; b < nb; b += nthreads) {
      uint32_t byte = 0;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int i = 8 * b + t;
        byte |= (uint32_t)(i < (int)d.cb_len ? bit(i) : 0) << (7 - t);
      }
      d.data[b] = (uint8_t)byte;
    }
  }
  if (t0 == 0) {
    *d.iters = (uint8_t)(ret == 0 ? a.max_iter : ret);
    if (ret > 0) {
      *d.flag = 1;
    }
  }
}

// a * b mod P (P of degree `order`, given with its x^order bit), Horner over b's bits
// (b < 2^order <= 2^24: Horner over b's 24 low bits, leading zero bits leave r = 0; unrolled, so
// the per-iteration CRC check is a straight dependency chain without loop overhead)
__device__ __forceinline__ uint32_t mulmod(uint32_t a, uint32_t b, uint32_t poly, int order)
{
  uint32_t r = 0;
#pragma unroll
  for (int i = 23; i >= 0; i--) {
    r = (r << 1) ^ (((b >> i) & 1u) ? a : 0u);
    r ^= ((r >> order) & 1u) ? poly : 0u;
  }
  return r;
}

template <int BG, int CS, typename E>
__global__ __launch_bounds__(LDPC_WG) void ldpc_kernel(LdpcArgs a)
{
  using T          = Topo<BG>;
  constexpr int NW = words_before_e<BG, E>(T::M);
  constexpr int CW = T::N * CS * (int)sizeof(E);  // LDS bytes per codeword
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  const int      ls    = a.ls;
  const int      liftK = T::K * ls;
  const int      cwl   = CS >= 384 ? 0 : (int)threadIdx.x / ls;
  const int      z     = (int)threadIdx.x - cwl * ls;
  const bool     act   = cwl < a.cw_per_wg && z < ls;
  const uint32_t cw    = blockIdx.x * (uint32_t)a.cw_per_wg + (uint32_t)cwl;
  const bool     exists = act && cw < a.ncw;
  const CwCtx    cc    = cw_ctx(a, cw, act, (int)sizeof(E));
  const bool     live  = cc.live;
  uint32_t*      shl   = reinterpret_cast<uint32_t*>(smem);  // LDPC_MAX_EDGES shifts
  E*             soft  = reinterpret_cast<E*>(smem + LDPC_LDS_HDR + (act ? cwl : 0) * CW);
  uint32_t*      red   = reinterpret_cast<uint32_t*>(smem + LDPC_LDS_HDR + a.cw_per_wg * CW);  // CRC parts
  uint32_t*      anyb  = red + a.cw_per_wg;  // "some codeword still decoding" flag
  for (int e = (int)threadIdx.x; e < Topo<BG>::rs[T::M]; e += (int)blockDim.x) {
    shl[e] = a.sh[e];
  }

  // ---- load: columns 0, 1 = 0 (punctured), column c >= 2 from llr[(c-2) ls] (init_ldpc_dec_c) ----
  if (live) {
    const E* in  = reinterpret_cast<const E*>(cc.in) + z;
    soft[z]      = 0;
    soft[CS + z] = 0;
    const int ncols = min(T::N, T::K + max(cc.n_layers, 4));  // columns the codeword's layers touch
#pragma unroll 4
    for (int c = 2; c < ncols; ++c) {
      soft[c * CS + z] = in[(c - 2) * ls];
    }
  }

  Lane<E> ln;
  ln.soft        = soft;
  ln.sh          = shl;
  ln.z           = z;
  ln.ls          = ls;
  ln.busy        = live;
  ln.n_layers    = cc.n_layers;
  ln.n_layers_wg = wg_layers(a, cc, anyb + 1);
  ln.scale_mode  = a.scale_mode;
  ln.sf          = a.sf;

  uint32_t st[NW];
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    st[i] = 0u;
  }
  const bool use_crc = a.xpow || a.cws;
  int        ret     = use_crc ? 0 : a.max_iter;
  for (int it = 0; it < a.max_iter; ++it) {
    run_iteration<BG, CS, E, NW>(ln, st, std::make_integer_sequence<int, T::M>{});
    if (use_crc) {
      if (z == 0 && act) {
        red[cwl] = 0u;
      }
      if (threadIdx.x == 0) {
        *anyb = 0u;
      }
      __syncthreads();  // last layer's soft bits; red / anyb cleared
      if (ln.busy) {
        // bits [z K, z K + K) of the message, natural order i = c ls + p
        const int order = cc.order;
        const int b0    = z * T::K;
        int       c     = (int)__umulhi((uint32_t)b0, a.magic_ls);  // b0 / ls
        int       p     = b0 - c * ls;
        uint32_t  crc   = 0;
#pragma unroll
        for (int b = 0; b < T::K; ++b) {
          const uint32_t bit = soft[c * CS + p] < 0 ? 1u : 0u;
          const uint32_t fb  = ((crc >> (order - 1)) & 1u) ^ bit;
          crc                = ((crc << 1) ^ (fb ? cc.poly : 0u)) & ((1u << order) - 1u);
          ++p;
          if (p == ls) {
            p = 0;
            ++c;
          }
        }
        const uint32_t part = mulmod(crc, cc.xpow[liftK - b0 - T::K], cc.poly, order) & ((1u << order) - 1u);
        if (part) {
          atomicXor(&red[cwl], part);
        }
      }
      __syncthreads();
      if (ln.busy && red[cwl] == 0u) {  // srsran_crc_match: stop with this iteration's message
        ln.busy = false;
        ret     = it + 1;
      }
      if (ln.busy) {
        *anyb = 1u;  // (no __syncthreads_or: its LDS scratch would shift every soft-bit address)
      }
      __syncthreads();
      if (*anyb == 0u) {
        break;
      }
    }
  }
  __syncthreads();

  // ---- message: bit i = soft[i] < 0 for i < liftK (extract_ldpc_message_c) ----
  auto bit = [&](int i) -> uint32_t {
    const int c = (int)__umulhi((uint32_t)i, a.magic_ls);
    return soft[c * CS + (i - c * ls)] < 0 ? 1u : 0u;
  };
  if (a.cws) {
    cb_finish(a, cw, exists, cc, ret, z, ls, bit);
  } else if (live) {
    uint8_t* out = a.out + (size_t)cw * a.out_stride;
    if (a.out_packed) {
      for (int b = z; b < liftK / 8; b += ls) {
        uint32_t byte = 0;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          byte |= bit(8 * b + t) << (7 - t);
        }
        out[b] = (uint8_t)byte;
      }
    } else {
      for (int c = 0; c < T::K; ++c) {
        out[c * ls + z] = soft[c * CS + z] < 0 ? 1 : 0;
      }
    }
    if (a.ret && z == 0) {
      a.ret[cw] = (uint8_t)ret;
    }
  }
}

// ML: layers the instantiation can process (the compressed check state is sized for them); the
// ML = 8 instantiations serve high-rate codewords (rv 0 at code rates above ~0.6 for BG1) with a
// fraction of the VGPRs, hence more resident workgroups
template <int BG, int CS, int ML>
__global__ __launch_bounds__(LDPC_WG) void ldpc_kernel_pk(LdpcArgs a)
{
  using T          = Topo<BG>;
  static_assert(ML <= T::M, "layers");
  constexpr int NW = words_before_pk<BG>(ML);
  constexpr int CW = T::N * CS;  // LDS bytes per codeword
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  const int      ls     = a.ls;
  const int      h      = ls >> 1;
  const int      liftK  = T::K * ls;
  const int      cwl    = CS >= 384 ? 0 : (int)threadIdx.x / h;
  const int      z      = (int)threadIdx.x - cwl * h;
  const bool     act    = cwl < a.cw_per_wg && z < h;
  const uint32_t cw     = blockIdx.x * (uint32_t)a.cw_per_wg + (uint32_t)cwl;
  const bool     exists = act && cw < a.ncw;
  const CwCtx    cc     = cw_ctx(a, cw, act, 1);
  const bool     live   = cc.live;
  uint32_t*      shl    = reinterpret_cast<uint32_t*>(smem);                      // LDPC_MAX_EDGES shifts
  uint8_t*       lut    = reinterpret_cast<uint8_t*>(smem + LDPC_MAX_EDGES * 4);  // 128-entry scaling table
  int8_t*        soft   = smem + LDPC_LDS_HDR + (act ? cwl : 0) * CW;
  uint32_t*      red    = reinterpret_cast<uint32_t*>(smem + LDPC_LDS_HDR + a.cw_per_wg * CW);  // CRC parts
  uint32_t*      anyb   = red + a.cw_per_wg;  // "some codeword still decoding" flag
  for (int e = (int)threadIdx.x; e < Topo<BG>::rs[T::M]; e += (int)blockDim.x) {
    shl[e] = a.sh[e];
  }
  for (int m = (int)threadIdx.x; m < 128; m += (int)blockDim.x) {
    lut[m] = a.scale_lut[m];
  }

  // ---- load (init_ldpc_dec_c), -128 -> -127 (see above) ----
  if (live) {
    const int8_t* in = reinterpret_cast<const int8_t*>(cc.in) + z;
    soft[z]          = 0;
    soft[z + h]      = 0;
    soft[CS + z]     = 0;
    soft[CS + z + h] = 0;
    // extension column K + 4 + j belongs to layer 4 + j only: columns past the codeword's last layer
    // are never read (for rv 0 transmissions most of the circular buffer)
    const int ncols = min(T::N, T::K + max(cc.n_layers, 4));
    if ((ls & 3) == 0 && (reinterpret_cast<uintptr_t>(cc.in) & 3) == 0) {
      // dwords, 8 in flight a thread: the load is latency-bound (one round trip instead of ncols)
      const int       q   = ls >> 2;  // dwords per column
      const int       tot = (ncols - 2) * q;
      const uint32_t* in4 = reinterpret_cast<const uint32_t*>(cc.in);
      for (int f0 = z; f0 < tot; f0 += 8 * h) {
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int f = f0 + k * h;
          v[k]        = f < tot ? in4[f] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int f = f0 + k * h;
          if (f < tot) {
            const int      c  = (int)__umulhi((uint32_t)(4 * f), a.magic_ls);  // 4 f / ls
            const uint32_t t  = v[k] ^ 0x80808080u;                              // bytes that were -128 -> 0
            const uint32_t nz = (((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
            *reinterpret_cast<uint32_t*>(soft + (c + 2) * CS + (4 * f - c * ls)) = v[k] + ((~nz & 0x80808080u) >> 7);
          }
        }
      }
    } else {
#pragma unroll 4
      for (int c = 2; c < ncols; ++c) {
        soft[c * CS + z]     = (int8_t)max((int)in[(c - 2) * ls], -127);
        soft[c * CS + z + h] = (int8_t)max((int)in[(c - 2) * ls + h], -127);
      }
    }
  }

  LanePk ln;
  ln.soft        = (lds_i8*)(uintptr_t)(uint32_t)(LDPC_LDS_HDR + (act ? cwl : 0) * CW);
  ln.sh          = shl;
  ln.scale       = lut;
  ln.z           = z;
  ln.ls          = ls;
  ln.h           = h;
  ln.busy        = live;
  ln.n_layers    = cc.n_layers;
  ln.n_layers_wg = wg_layers(a, cc, anyb + 1);

  uint32_t st[NW];
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    st[i] = 0u;
  }
  const bool use_crc = a.xpow || a.cws;
  int        ret     = use_crc ? 0 : a.max_iter;
  for (int it = 0; it < a.max_iter; ++it) {
    run_iteration_pk<BG, CS, NW>(ln, st, std::make_integer_sequence<int, ML>{});
    if (use_crc) {
      if (z == 0 && act) {
        red[cwl] = 0u;
      }
      if (threadIdx.x == 0) {
        *anyb = 0u;
      }
      __syncthreads();  // last layer's soft bits; red / anyb cleared
      if (ln.busy) {
        // bits [2 z K, 2 z K + 2 K) of the message, natural order i = c ls + p
        const int order = cc.order;
        const int b0    = 2 * z * T::K;
        int       c     = (int)__umulhi((uint32_t)b0, a.magic_ls);  // b0 / ls
        int       p     = b0 - c * ls;
        uint32_t  crc   = 0;
#pragma unroll
        for (int b = 0; b < 2 * T::K; ++b) {
          const uint32_t bit = soft[c * CS + p] < 0 ? 1u : 0u;
          const uint32_t fb  = ((crc >> (order - 1)) & 1u) ^ bit;
          crc                = ((crc << 1) ^ (fb ? cc.poly : 0u)) & ((1u << order) - 1u);
          ++p;
          if (p == ls) {
            p = 0;
            ++c;
          }
        }
        const uint32_t part = mulmod(crc, cc.xpow[liftK - b0 - 2 * T::K], cc.poly, order) & ((1u << order) - 1u);
        if (part) {
          atomicXor(&red[cwl], part);
        }
      }
      __syncthreads();
      if (ln.busy && red[cwl] == 0u) {  // srsran_crc_match: stop with this iteration's message
        ln.busy = false;
        ret     = it + 1;
      }
      if (ln.busy) {
        *anyb = 1u;  // (no __syncthreads_or: its LDS scratch would shift every soft-bit address)
      }
      __syncthreads();
      if (*anyb == 0u) {
        break;
      }
    }
  }
  __syncthreads();

  // ---- message: bit i = soft[i] < 0 for i < liftK (extract_ldpc_message_c) ----
  auto bit = [&](int i) -> uint32_t {
    const int c = (int)__umulhi((uint32_t)i, a.magic_ls);
    return soft[c * CS + (i - c * ls)] < 0 ? 1u : 0u;
  };
  if (a.cws) {
    cb_finish(a, cw, exists, cc, ret, z, h, bit);
  } else if (live) {
    uint8_t* out = a.out + (size_t)cw * a.out_stride;
    if (a.out_packed) {
      for (int b = z; b < liftK / 8; b += h) {
        uint32_t byte = 0;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          byte |= bit(8 * b + t) << (7 - t);
        }
        out[b] = (uint8_t)byte;
      }
    } else {
      for (int c = 0; c < T::K; ++c) {
        out[c * ls + z]     = soft[c * CS + z] < 0 ? 1 : 0;
        out[c * ls + z + h] = soft[c * CS + z + h] < 0 ? 1 : 0;
      }
    }
    if (a.ret && z == 0) {
      a.ret[cw] = (uint8_t)ret;
    }
  }
}

static int col_stride(int ls, int bits)
{
  if (bits == 16) {
    return ls > 128 ? 384 : (ls > 32 ? 128 : 32);
  }
  return ls > 256 ? 384 : (ls > 128 ? 256 : (ls > 64 ? 128 : (ls > 32 ? 64 : (ls > 16 ? 32 : 16))));
}

#if LDPC_BG_ONLY == 0
// the 8-bit packed path serves two check nodes a thread (even ls > 16)
int ldpc_threads_per_cw(int ls, int bits) { return (bits == 8 && ls > 16) ? ls / 2 : ls; }

int ldpc_cw_per_wg(int ls, int bits)
{
  const int cs = col_stride(ls, bits);
  if (cs >= 384) {
    return 1;
  }
  // up to 256 threads, and at most 64 KiB of LDS (BG1 geometry bounds both base graphs)
  return max(1, min(256 / ldpc_threads_per_cw(ls, bits), 65536 / (68 * cs * (bits / 8))));
}

size_t ldpc_lds_bytes(int bg, int ls, int bits)
{
  const int n = (bg == 0 ? 68 : 52) * col_stride(ls, bits) * (bits / 8);
  return LDPC_LDS_HDR + (size_t)ldpc_cw_per_wg(ls, bits) * (n + 4) + 16;  // + CRC parts, flag, layer max
}
#endif

template <int BG>
hipError_t ldpc_launch_bg(const LdpcArgs& a, dim3 grid, dim3 block, size_t lds, hipStream_t s);

#if LDPC_BG_ONLY == 1
template <>
hipError_t ldpc_launch_bg<1>(const LdpcArgs& a, dim3 grid, dim3 block, size_t lds, hipStream_t s)
#else
template <>
hipError_t ldpc_launch_bg<0>(const LdpcArgs& a, dim3 grid, dim3 block, size_t lds, hipStream_t s)
#endif
{
  constexpr int BG = LDPC_BG_ONLY;
  if (a.llr_bits == 16) {
    switch (col_stride(a.ls, 16)) {
      case 384:
        hipLaunchKernelGGL((ldpc_kernel<BG, 384, int16_t>), grid, block, lds, s, a);
        break;
      case 128:
        hipLaunchKernelGGL((ldpc_kernel<BG, 128, int16_t>), grid, block, lds, s, a);
        break;
      default:
        hipLaunchKernelGGL((ldpc_kernel<BG, 32, int16_t>), grid, block, lds, s, a);
        break;
    }
    return hipGetLastError();
  }
  const bool few = a.n_layers <= LDPC_FEW_LAYERS;  // every codeword of the launch within 8 layers
#define LDPC_PK(CSV)                                                                                                   \
  case CSV:                                                                                                            \
    if (few) {                                                                                                         \
      hipLaunchKernelGGL((ldpc_kernel_pk<BG, CSV, LDPC_FEW_LAYERS>), grid, block, lds, s, a);                          \
    } else {                                                                                                           \
      hipLaunchKernelGGL((ldpc_kernel_pk<BG, CSV, Topo<BG>::M>), grid, block, lds, s, a);                              \
    }                                                                                                                  \
    break;
  switch (col_stride(a.ls, 8)) {
    LDPC_PK(384)
    LDPC_PK(256)
    LDPC_PK(128)
    LDPC_PK(64)
    LDPC_PK(32)
#undef LDPC_PK
    default:
      hipLaunchKernelGGL((ldpc_kernel<BG, 16, int8_t>), grid, block, lds, s, a);
      break;
  }
  return hipGetLastError();
}

#if LDPC_BG_ONLY == 0
hipError_t ldpc_launch(int bg, const LdpcArgs& a, hipStream_t stream)
{
  if (a.ncw == 0) {
    return hipSuccess;
  }
  const int    bits    = a.llr_bits == 16 ? 16 : 8;
  const int    cpw     = a.cw_per_wg;
  const int    threads = ((cpw * ldpc_threads_per_cw(a.ls, bits) + 63) / 64) * 64;
  const int    grid    = (int)((a.ncw + cpw - 1) / cpw);
  const size_t lds     = ldpc_lds_bytes(bg, a.ls, bits);
  if (threads > LDPC_WG || cpw != ldpc_cw_per_wg(a.ls, bits) || a.ls < 2 || a.ls > 384 ||
      (bits == 16 && a.scale_mode != LDPC_SCALE_C)) {
    return hipErrorInvalidValue;
  }
  StageScope timing_scope(ST_LDPC, stream);
  return bg == 0 ? ldpc_launch_bg<0>(a, dim3(grid), dim3(threads), lds, stream)
                 : ldpc_launch_bg<1>(a, dim3(grid), dim3(threads), lds, stream);
}
#endif

}  // namespace srsran_amd
