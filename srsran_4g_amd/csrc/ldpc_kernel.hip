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
//   * soft bits (a-posteriori LLRs) of the codeword live in LDS as int8, natural order
//     (column c, position p at c*ls + p).  Check z of a layer reads / writes position
//     (z + shift) mod ls of every connected column: within a layer every soft bit belongs to
//     exactly one thread, so a layer needs no synchronisation, only a barrier between layers.
//   * check-to-variable messages are never stored per edge: a thread keeps, for each layer,
//     its check node's compressed min-sum state in VGPRs -- scaled min1 / min2 (7 bits each),
//     the index of the min1 edge (5 bits) and one sign bit per edge -- one dword per layer
//     (two for the four degree-19 rows of BG1).  c2v of edge k = +-(k == idx ? min2 : min1),
//     exactly the values the reference stores in check_to_var.
//   * the base graph topology (columns, degrees) is compile time: every layer is unrolled, so
//     the state array is statically indexed and stays in registers; the lifting size's shifts
//     are kernel arguments (scalar loads).
//   * CRC early stop (decode_crc_c): after every iteration each thread CRCs its K contiguous
//     hard bits from zero, moves the CRC to its place with x^(bits after) mod P and the parts
//     XOR together in LDS; zero <=> srsran_crc_match over liftK bits.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "ldpc_kernel.h"

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

static constexpr int ONE_WORD_MAX_DEG = 13;  // 7 + 7 + 5 + 13 sign bits

template <int BG>
constexpr int deg_of(int l)
{
  return Topo<BG>::rs[l + 1] - Topo<BG>::rs[l];
}
template <int BG>
constexpr int words_before(int L)
{
  int w = 0;
  for (int l = 0; l < L; ++l) {
    w += deg_of<BG>(l) > ONE_WORD_MAX_DEG ? 2 : 1;
  }
  return w;
}

struct Lane {
  int8_t*         soft;  // this codeword's soft bits (LDS)
  const uint16_t* sh;    // shift of every edge for this lifting size (device)
  int     z;         // lifted check index
  int     ls;
  bool    busy;      // decodes this layer (live codeword, CRC not yet matched)
  int     n_layers;
  int     scale_mode;
  int     sf;
};

__device__ __forceinline__ int scale_mag(const Lane& ln, int m)
{
  // _mm256_scalei_epi8: mulhi_epu16 of the (non-negative) byte by sf; ldpc_dec_c.c: m*sf/100
  return ln.scale_mode == LDPC_SCALE_SIMD ? (int)(((uint32_t)m * (uint32_t)ln.sf) >> 16) : m * ln.sf / 100;
}

// One layer (row L of the base graph) for this thread's check node.
template <int BG, int L, int NW>
__device__ __forceinline__ void run_layer(const Lane& ln, const LdpcArgs& a, uint32_t (&st)[NW])
{
  using T                  = Topo<BG>;
  constexpr int  e0        = T::rs[L];
  constexpr int  deg       = deg_of<BG>(L);
  constexpr int  w0        = words_before<BG>(L);
  constexpr bool two       = deg > ONE_WORD_MAX_DEG;
  constexpr uint32_t degmask = (deg >= 32) ? 0xFFFFFFFFu : ((1u << deg) - 1u);
  if (L >= ln.n_layers) {
    return;
  }
  __syncthreads();  // soft bits written by the previous layer
  if (!ln.busy) {
    return;
  }
  // Opaque per-layer copies: without them LICM hoists every edge's address (316 VGPRs) and
  // every col*ls (SGPRs) out of the iteration loop and the kernel spills.
  int             zz  = ln.z;
  int             lsz = ln.ls;
  const uint16_t* shp = ln.sh;
  asm volatile("" : "+v"(zz), "+s"(lsz), "+s"(shp));
  const uint32_t s0  = st[w0];
  const uint32_t sg  = two ? st[w0 + 1] : (s0 >> 19);
  const int      o1  = (int)(s0 & 127u);
  const int      o2  = (int)((s0 >> 7) & 127u);
  const int      oix = (int)((s0 >> 14) & 31u);

  int      v2c[deg];
  uint32_t adr[deg];
  int      m1 = 127, m2 = 127, mi = 0;  // INT8_MAX start (ldpc_dec_c.c:223-228)
  uint32_t negs = 0;
#pragma unroll
  for (int k = 0; k < deg; ++k) {
    const int      col = T::col[e0 + k];
    const uint32_t p   = (uint32_t)zz + shp[e0 + k];
    const uint32_t q   = p - (uint32_t)lsz;
    adr[k]             = (uint32_t)(col * lsz) + min(p, q);  // (z + shift) mod ls
    const int x        = ln.soft[adr[k]];
    // previous c2v of this edge
    const int mag = k == oix ? o2 : o1;
    const int sgn = -(int)((sg >> k) & 1u);
    const int c   = (mag ^ sgn) - sgn;
    // inner_var_to_check: infinity (|x| >= 127) propagates, else clip(x - c) to +-63
    const int v   = (x >= 127 || x <= -127) ? min(max(x, -127), 127) : min(max(x - c, -63), 63);
    v2c[k]        = v;
    const int av  = v < 0 ? -v : v;
    const bool lt = av < m1;  // strict: the first minimum keeps the index
    m2            = lt ? m1 : min(m2, av);
    mi            = lt ? k : mi;
    m1            = min(m1, av);
    negs |= (uint32_t)(v < 0) << k;
  }
  const int      s1  = scale_mag(ln, m1);
  const int      s2  = scale_mag(ln, m2);
  const uint32_t csg = (__builtin_popcount(negs) & 1) ? (negs ^ degmask) : negs;  // sign of c2v_k = prod ^ neg_k
#pragma unroll
  for (int k = 0; k < deg; ++k) {
    const int mag = k == mi ? s2 : s1;
    const int sgn = -(int)((csg >> k) & 1u);
    const int c   = (mag ^ sgn) - sgn;
    int       t   = c + v2c[k];  // update_ldpc_soft_bits: beyond +-63 -> +-127
    t             = t > 63 ? 127 : (t < -63 ? -127 : t);
    ln.soft[adr[k]] = (int8_t)t;
  }
  const uint32_t w = (uint32_t)s1 | ((uint32_t)s2 << 7) | ((uint32_t)mi << 14);
  if constexpr (two) {
    st[w0]     = w;
    st[w0 + 1] = csg;
  } else {
    st[w0] = w | (csg << 19);
  }
}

template <int BG, int NW, int... Ls>
__device__ __forceinline__ void run_iteration(const Lane& ln, const LdpcArgs& a, uint32_t (&st)[NW],
                                              std::integer_sequence<int, Ls...>)
{
  (run_layer<BG, Ls, NW>(ln, a, st), ...);
}

// a * b mod P (P of degree `order`, given with its x^order bit), Horner over b's bits
__device__ __forceinline__ uint32_t mulmod(uint32_t a, uint32_t b, uint32_t poly, int order)
{
  uint32_t r = 0;
#pragma unroll 1
  for (int i = order - 1; i >= 0; i--) {
    r = (r << 1) ^ (((b >> i) & 1u) ? a : 0u);
    r ^= ((r >> order) & 1u) ? poly : 0u;
  }
  return r;
}

template <int BG>
__global__ __launch_bounds__(LDPC_WG) void ldpc_kernel(LdpcArgs a)
{
  using T             = Topo<BG>;
  constexpr int NW    = words_before<BG>(T::M);
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  const int ls        = a.ls;
  const int liftN     = T::N * ls;
  const int liftK     = T::K * ls;
  const int cwl       = (int)threadIdx.x / ls;
  const int z         = (int)threadIdx.x - cwl * ls;
  const bool act      = cwl < a.cw_per_wg;
  const uint32_t cw   = blockIdx.x * (uint32_t)a.cw_per_wg + (uint32_t)cwl;
  const bool live     = act && cw < a.ncw;
  const int  stride   = (liftN + 15) & ~15;
  int8_t*    soft     = smem + (act ? cwl : 0) * stride;
  uint32_t*  red      = reinterpret_cast<uint32_t*>(smem + a.cw_per_wg * stride);  // CRC parts per codeword

  // ---- load: soft[0 .. 2ls) = 0 (punctured), soft[2ls + i] = llr[i] (init_ldpc_dec_c) ----
  if (live) {
    const int8_t* in = a.in + (size_t)cw * a.in_stride;
    for (int i = z; i < liftN; i += ls) {
      soft[i] = i < 2 * ls ? (int8_t)0 : in[i - 2 * ls];
    }
  }

  Lane ln;
  ln.soft       = soft;
  ln.sh         = a.sh;
  ln.z          = z;
  ln.ls         = ls;
  ln.busy       = live;
  ln.n_layers   = a.n_layers;
  ln.scale_mode = a.scale_mode;
  ln.sf         = a.sf;

  uint32_t st[NW];
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    st[i] = 0u;
  }
  int ret = a.xpow ? 0 : a.max_iter;
  for (int it = 0; it < a.max_iter; ++it) {
    run_iteration<BG, NW>(ln, a, st, std::make_integer_sequence<int, T::M>{});
    if (a.xpow) {
      if (z == 0 && act) {
        red[cwl] = 0u;
      }
      __syncthreads();  // last layer's soft bits; red cleared
      if (ln.busy) {
        const int order = a.crc_order;
        uint32_t  crc   = 0;
        const int b0    = z * T::K;
#pragma unroll
        for (int b = 0; b < T::K; ++b) {
          const uint32_t bit = soft[b0 + b] < 0 ? 1u : 0u;
          const uint32_t fb  = ((crc >> (order - 1)) & 1u) ^ bit;
          crc                = (crc << 1) ^ (fb ? a.crc_poly : 0u);
          crc &= (1u << order) - 1u;
        }
        const uint32_t part = mulmod(crc, a.xpow[liftK - b0 - T::K], a.crc_poly, order) & ((1u << order) - 1u);
        if (part) {
          atomicXor(&red[cwl], part);
        }
      }
      __syncthreads();
      if (ln.busy && red[cwl] == 0u) {  // srsran_crc_match: stop with this iteration's message
        ln.busy = false;
        ret     = it + 1;
      }
      if (__syncthreads_or(ln.busy) == 0) {
        break;
      }
    }
  }
  __syncthreads();

  // ---- message: bit i = soft[i] < 0 for i < liftK (extract_ldpc_message_c) ----
  if (live) {
    uint8_t* out = a.out + (size_t)cw * a.out_stride;
    if (a.out_packed) {
      for (int b = z; b < liftK / 8; b += ls) {
        uint32_t byte = 0;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          byte |= (uint32_t)(soft[8 * b + t] < 0) << (7 - t);
        }
        out[b] = (uint8_t)byte;
      }
    } else {
      for (int i = z; i < liftK; i += ls) {
        out[i] = soft[i] < 0 ? 1 : 0;
      }
    }
    if (a.ret && z == 0) {
      a.ret[cw] = (uint8_t)ret;
    }
  }
}

int ldpc_cw_per_wg(int ls) { return ls >= 192 ? 1 : max(1, 256 / ls); }

size_t ldpc_lds_bytes(int bg, int ls)
{
  const int n = (bg == 0 ? 68 : 52) * ls;
  return (size_t)ldpc_cw_per_wg(ls) * ((n + 15) & ~15) + (size_t)ldpc_cw_per_wg(ls) * 4 + 16;
}

hipError_t ldpc_launch(int bg, const LdpcArgs& a, hipStream_t stream)
{
  if (a.ncw == 0) {
    return hipSuccess;
  }
  const int    cpw     = a.cw_per_wg;
  const int    threads = ((cpw * a.ls + 63) / 64) * 64;
  const int    grid    = (int)((a.ncw + cpw - 1) / cpw);
  const size_t lds     = ldpc_lds_bytes(bg, a.ls);
  if (threads > LDPC_WG || cpw != ldpc_cw_per_wg(a.ls)) {
    return hipErrorInvalidValue;
  }
  if (bg == 0) {
    hipLaunchKernelGGL(ldpc_kernel<0>, dim3(grid), dim3(threads), lds, stream, a);
  } else {
    hipLaunchKernelGGL(ldpc_kernel<1>, dim3(grid), dim3(threads), lds, stream, a);
  }
  return hipGetLastError();
}

}  // namespace srsran_amd
