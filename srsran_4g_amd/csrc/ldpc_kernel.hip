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
  int8_t*         soft;  // this codeword's soft bits (LDS), column stride CS
  const uint32_t* sh;    // shift of every edge for this lifting size (LDS copy)
  int             z;     // lifted check index
  int             ls;
  bool            busy;  // decodes this layer (live codeword, CRC not yet matched)
  int             n_layers;
  int             scale_mode;
  int             sf;
};

__device__ __forceinline__ int scale_mag(const Lane& ln, int m)
{
  // _mm256_scalei_epi8: mulhi_epu16 of the (non-negative) byte by sf; ldpc_dec_c.c: m*sf/100
  return ln.scale_mode == LDPC_SCALE_SIMD ? (int)(((uint32_t)m * (uint32_t)ln.sf) >> 16) : m * ln.sf / 100;
}

// One layer (row L of the base graph) for this thread's check node.
template <int BG, int CS, int L, int NW>
__device__ __forceinline__ void run_layer(const Lane& ln, uint32_t (&st)[NW])
{
  using T                = Topo<BG>;
  constexpr int  e0      = T::rs[L];
  constexpr int  deg     = deg_of<BG>(L);
  constexpr int  w0      = words_before<BG>(L);
  constexpr bool two     = deg > ONE_WORD_MAX_DEG;
  if (L >= ln.n_layers) {
    return;
  }
  __syncthreads();  // soft bits written by the previous layer
  if (!ln.busy) {
    return;
  }
  // Opaque per-layer copy: without it LICM hoists every edge's address (316 VGPRs) out of the
  // iteration loop and the kernel spills.
  int zz = ln.z;
  asm volatile("" : "+v"(zz));
  const uint32_t* shp = ln.sh + e0;  // LDS: broadcast reads with immediate offsets
  const int       ls  = ln.ls;

  const uint32_t s0  = st[w0];
  const uint32_t sg  = two ? st[w0 + 1] : (s0 >> 19);
  const int      o1  = (int)(s0 & 127u);
  const int      o2  = (int)((s0 >> 7) & 127u);
  const int      oix = (int)((s0 >> 14) & 31u);

  int      v2c[deg];
  uint32_t pos[deg];
  int      m1 = 127, m2 = 127, mi = 0;  // INT8_MAX start (ldpc_dec_c.c:223-228)
  int      px = 0;                      // XOR of all v2c: its sign = product of signs
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
    // inner_var_to_check: |x| >= 127 (infinity) propagates as +-127, else clip(x - c) to +-63
    const int  vn  = min(max(x - c, -63), 63);
    const bool big = (uint32_t)(x + 126) > 252u;
    const int  v   = big ? (x | 1) : vn;
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
    const int t = c + v2c[k];  // update_ldpc_soft_bits: beyond +-63 -> +-127
    const int r = (uint32_t)(t + 63) > 126u ? 127 * ((t >> 31) | 1) : t;
    ln.soft[col * CS + pos[k]] = (int8_t)r;
  }
  const uint32_t w = (uint32_t)s1 | ((uint32_t)s2 << 7) | ((uint32_t)mi << 14);
  if constexpr (two) {
    st[w0]     = w;
    st[w0 + 1] = csg;
  } else {
    st[w0] = w | (csg << 19);
  }
}

template <int BG, int CS, int NW, int... Ls>
__device__ __forceinline__ void run_iteration(const Lane& ln, uint32_t (&st)[NW], std::integer_sequence<int, Ls...>)
{
  (run_layer<BG, CS, Ls, NW>(ln, st), ...);
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

template <int BG, int CS>
__global__ __launch_bounds__(LDPC_WG) void ldpc_kernel(LdpcArgs a)
{
  using T          = Topo<BG>;
  constexpr int NW = words_before<BG>(T::M);
  constexpr int CW = T::N * CS;  // LDS bytes per codeword
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  const int      ls    = a.ls;
  const int      liftK = T::K * ls;
  const int      cwl   = CS >= 256 ? 0 : (int)threadIdx.x / ls;
  const int      z     = (int)threadIdx.x - cwl * ls;
  const bool     act   = cwl < a.cw_per_wg && z < ls;
  const uint32_t cw    = blockIdx.x * (uint32_t)a.cw_per_wg + (uint32_t)cwl;
  const bool     live  = act && cw < a.ncw;
  uint32_t*      shl   = reinterpret_cast<uint32_t*>(smem);  // LDPC_MAX_EDGES shifts
  int8_t*        soft  = smem + LDPC_MAX_EDGES * 4 + (act ? cwl : 0) * CW;
  uint32_t*      red   = reinterpret_cast<uint32_t*>(smem + LDPC_MAX_EDGES * 4 + a.cw_per_wg * CW);  // CRC parts
  for (int e = (int)threadIdx.x; e < Topo<BG>::rs[T::M]; e += (int)blockDim.x) {
    shl[e] = a.sh[e];
  }

  // ---- load: columns 0, 1 = 0 (punctured), column c >= 2 from llr[(c-2) ls] (init_ldpc_dec_c) ----
  if (live) {
    const int8_t* in = a.in + (size_t)cw * a.in_stride + z;
    soft[z]          = 0;
    soft[CS + z]     = 0;
#pragma unroll 4
    for (int c = 2; c < T::N; ++c) {
      soft[c * CS + z] = in[(c - 2) * ls];
    }
  }

  Lane ln;
  ln.soft       = soft;
  ln.sh         = shl;
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
    run_iteration<BG, CS, NW>(ln, st, std::make_integer_sequence<int, T::M>{});
    if (a.xpow) {
      if (z == 0 && act) {
        red[cwl] = 0u;
      }
      __syncthreads();  // last layer's soft bits; red cleared
      if (ln.busy) {
        // bits [z K, z K + K) of the message, natural order i = c ls + p
        const int order = a.crc_order;
        const int b0    = z * T::K;
        int       c     = (int)__umulhi((uint32_t)b0, a.magic_ls);  // b0 / ls
        int       p     = b0 - c * ls;
        uint32_t  crc   = 0;
#pragma unroll
        for (int b = 0; b < T::K; ++b) {
          const uint32_t bit = soft[c * CS + p] < 0 ? 1u : 0u;
          const uint32_t fb  = ((crc >> (order - 1)) & 1u) ^ bit;
          crc                = ((crc << 1) ^ (fb ? a.crc_poly : 0u)) & ((1u << order) - 1u);
          ++p;
          if (p == ls) {
            p = 0;
            ++c;
          }
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
        const int i0   = 8 * b;
        int       c    = (int)__umulhi((uint32_t)i0, a.magic_ls);
        int       p    = i0 - c * ls;
        uint32_t  byte = 0;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          byte |= (uint32_t)(soft[c * CS + p] < 0) << (7 - t);
          ++p;
          if (p == ls) {
            p = 0;
            ++c;
          }
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

static int col_stride(int ls)
{
  return ls > 256 ? 384 : (ls > 128 ? 256 : (ls > 64 ? 128 : (ls > 32 ? 64 : (ls > 16 ? 32 : 16))));
}

#if LDPC_BG_ONLY == 0
int ldpc_cw_per_wg(int ls)
{
  const int cs = col_stride(ls);
  if (cs >= 256) {
    return 1;
  }
  // up to 256 threads, and at most 64 KiB of LDS (BG1 geometry bounds both base graphs)
  return max(1, min(256 / ls, 65536 / (68 * cs)));
}

size_t ldpc_lds_bytes(int bg, int ls)
{
  const int n = (bg == 0 ? 68 : 52) * col_stride(ls);
  return LDPC_MAX_EDGES * 4 + (size_t)ldpc_cw_per_wg(ls) * (n + 4) + 16;
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
  switch (col_stride(a.ls)) {
    case 384:
      hipLaunchKernelGGL((ldpc_kernel<BG, 384>), grid, block, lds, s, a);
      break;
    case 256:
      hipLaunchKernelGGL((ldpc_kernel<BG, 256>), grid, block, lds, s, a);
      break;
    case 128:
      hipLaunchKernelGGL((ldpc_kernel<BG, 128>), grid, block, lds, s, a);
      break;
    case 64:
      hipLaunchKernelGGL((ldpc_kernel<BG, 64>), grid, block, lds, s, a);
      break;
    case 32:
      hipLaunchKernelGGL((ldpc_kernel<BG, 32>), grid, block, lds, s, a);
      break;
    default:
      hipLaunchKernelGGL((ldpc_kernel<BG, 16>), grid, block, lds, s, a);
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
  const int    cpw     = a.cw_per_wg;
  const int    threads = ((cpw * a.ls + 63) / 64) * 64;
  const int    grid    = (int)((a.ncw + cpw - 1) / cpw);
  const size_t lds     = ldpc_lds_bytes(bg, a.ls);
  if (threads > LDPC_WG || cpw != ldpc_cw_per_wg(a.ls) || a.ls < 2 || a.ls > 384) {
    return hipErrorInvalidValue;
  }
  return bg == 0 ? ldpc_launch_bg<0>(a, dim3(grid), dim3(threads), lds, stream)
                 : ldpc_launch_bg<1>(a, dim3(grid), dim3(threads), lds, stream);
}
#endif

}  // namespace srsran_amd
