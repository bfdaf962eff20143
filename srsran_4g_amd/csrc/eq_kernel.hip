// srsran_4g_amd/csrc/eq_kernel.hip -- PDSCH MIMO predecoding (MMSE with CSI) for CDNA4.
//
// Formulas of the reference's CSI predecoders (the PDSCH always passes CSI buffers,
// pdsch.c:325/871):
//   PORT0  srsran_predecoding_single_csi        precoding.c:307-355
//   CDD    srsran_predecoding_ccd_2x2_mmse_csi  precoding.c:1043-1121 (precoder alternates per RE)
//   SM     srsran_predecoding_multiplex_2x2_mmse_csi precoding.c:1437-1540 (codebooks 0..2)
//   TXD    srsran_predecoding_diversity_csi     precoding.c:671-775 (2-port SFBC pairs, 4-port SFBC + FSTD)
//   2x2    srsran_mat_2x2_mmse_csi_gen          mat.c:63-109
// computed in IEEE float with the scalar ("gen") operation order and no FMA contraction, so
// the result equals oracle/phy_oracle.c bit for bit.  (The reference's SIMD bodies use
// rcp_ps, ~1e-3 relative; see DESIGN.md.)  One thread per resource element: 2x2 CDD reads
// 48 B and writes 24 B per RE -- HBM-bound elementwise work.  The per-layer CSI maximum that
// csi_correction needs (pdsch.c:530) is reduced per wave and folded in with one atomicMax.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "eq_dev.h"
#include "eq_kernel.h"
#include "gmem.h"
#include "stage_timing.h"

#pragma clang fp contract(off)

namespace srsran_amd {

struct cpx {
  float r, i;
};
__device__ __forceinline__ cpx cadd(cpx a, cpx b) { return {a.r + b.r, a.i + b.i}; }
__device__ __forceinline__ cpx csub(cpx a, cpx b) { return {a.r - b.r, a.i - b.i}; }
__device__ __forceinline__ cpx cmul(cpx a, cpx b) { return {a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r}; }
__device__ __forceinline__ cpx cconj(cpx a) { return {a.r, -a.i}; }
__device__ __forceinline__ cpx cneg(cpx a) { return {-a.r, -a.i}; }
__device__ __forceinline__ cpx cscale(cpx a, float s) { return {a.r * s, a.i * s}; }
__device__ __forceinline__ cpx cmulj(cpx a) { return {-a.i, a.r}; }
__device__ __forceinline__ cpx ld(const float2* p, uint32_t k)
{
  const float2 v = gptr(p)[k];  // global address space (gmem.h): the pointers come from descriptors
  return {v.x, v.y};
}

__device__ __forceinline__ void mmse_csi(cpx y0, cpx y1, cpx h00, cpx h01, cpx h10, cpx h11, cpx& x0, cpx& x1,
                                         float& csi0, float& csi1, float noise, float norm)
{
  const cpx c00 = cconj(h00), c01 = cconj(h01), c10 = cconj(h10), c11 = cconj(h11);
  cpx       a00 = cadd(cmul(c00, h00), cmul(c10, h10));
  a00.r += noise;
  const cpx a01 = cadd(cmul(c00, h01), cmul(c10, h11));
  const cpx a10 = cadd(cmul(c01, h00), cmul(c11, h10));
  cpx       a11 = cadd(cmul(c01, h01), cmul(c11, h11));
  a11.r += noise;
  const cpx   det = csub(cmul(a00, a11), cmul(a01, a10));
  const float den = det.r * det.r + det.i * det.i;
  const cpx   rcp = {det.r / den, -det.i / den};
  const cpx   nrm = cscale(rcp, norm);
  const cpx   b00 = cmul(a11, nrm), b01 = cmul(cneg(a01), nrm), b10 = cmul(cneg(a10), nrm), b11 = cmul(a00, nrm);
  const cpx   w00 = cadd(cmul(b00, c00), cmul(b01, c01));
  const cpx   w01 = cadd(cmul(b00, c10), cmul(b01, c11));
  const cpx   w10 = cadd(cmul(b10, c00), cmul(b11, c01));
  const cpx   w11 = cadd(cmul(b10, c10), cmul(b11, c11));
  x0              = cadd(cmul(y0, w00), cmul(y1, w01));
  x1              = cadd(cmul(y0, w10), cmul(y1, w11));
  csi0            = 1.0f / b00.r;
  csi1            = 1.0f / b11.r;
}

// block-wide max of the per-thread CSI maxima (csi >= 0: IEEE bits order like the values), then
// one atomicMax per block and layer
template <int NL>
__device__ __forceinline__ void block_max_atomic(uint32_t* dst, const uint32_t (&v)[NL], uint32_t* red)
{
  uint32_t b[NL];
#pragma unroll
  for (int l = 0; l < NL; l++) {
    b[l] = v[l];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      b[l] = max(b[l], (uint32_t)__shfl_xor((int)b[l], off, 64));
    }
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int l = 0; l < NL; l++) {
      red[w * NL + l] = b[l];
    }
  }
  __syncthreads();
  if (threadIdx.x < NL) {
    uint32_t m = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); i++) {
      m = max(m, red[i * NL + threadIdx.x]);
    }
    atomicMax(&dst[threadIdx.x], m);
  }
}

static constexpr int EQ_THREADS = 256;

// grid position, estimate position and y scale of PDSCH RE k (fused srsran_pdsch_get)
__device__ __forceinline__ void re_at(const PredArgs& a, uint32_t k, uint32_t& gy, uint32_t& gh, float& ys)
{
  gy = k, gh = k, ys = 1.0f;
  if (a.idx) {
    const uint32_t e = a.idx[k];
    gy               = e & 0x7fffffffu;
    gh               = a.ce_row ? gy % a.ce_row : gy;
    ys               = (e >> 31) ? a.rho_b_inv : 1.0f;
  }
}

// srsran_predecoding_diversity_csi, 2 ports (precoding.c:671-700): thread k decodes the SFBC pair
// (2k, 2k+1); x / hh in float then * M_SQRT2 in double, as the C expression promotes it.
__device__ __forceinline__ void diversity_pair(const PredArgs& a, uint32_t k, uint32_t (&mx)[2])
{
  const bool     valid = k < a.n / 2;
  const uint32_t kk    = valid ? k : 0;
  uint32_t       gy0, gh0, gy1, gh1;
  float          s0, s1;
  re_at(a, 2 * kk, gy0, gh0, s0);
  re_at(a, 2 * kk + 1, gy1, gh1, s1);
  float hh = 0.f;
  cpx   x0 = {0.f, 0.f}, x1 = {0.f, 0.f};
  for (int p = 0; p < a.nrx; p++) {
    const cpx h00 = ld(a.h[0][p], gh0), h01 = ld(a.h[0][p], gh1), h10 = ld(a.h[1][p], gh0), h11 = ld(a.h[1][p], gh1);
    hh += h00.r * h00.r + h00.i * h00.i + h11.r * h11.r + h11.i * h11.i;
    cpx r0 = ld(a.y[p], gy0), r1 = ld(a.y[p], gy1);
    if (s0 != 1.0f) {
      r0 = cscale(r0, s0);
    }
    if (s1 != 1.0f) {
      r1 = cscale(r1, s1);
    }
    if (hh == 0.f) {
      hh = 1e-4f;
    }
    x0 = cadd(x0, cadd(cmul(cconj(h00), r0), cmul(h11, cconj(r1))));
    x1 = cadd(x1, cadd(cmul(cneg(h10), cconj(r0)), cmul(cconj(h01), r1)));
  }
  const float csi = hh;
  hh *= a.norm;  // scaling
  const double sq2 = 1.41421356237309504880;
  const float2 o0  = make_float2((float)((double)(x0.r / hh) * sq2), (float)((double)(x0.i / hh) * sq2));
  const float2 o1  = make_float2((float)((double)(x1.r / hh) * sq2), (float)((double)(x1.i / hh) * sq2));
  if (valid) {
    if (a.interleave) {  // srsran_layerdemap_diversity fused: codeword order d[2k + l] = x_l[k]
      a.x[0][2 * k]     = o0;
      a.x[0][2 * k + 1] = o1;
    } else {
      a.x[0][k] = o0;
      a.x[1][k] = o1;
    }
    a.csi[0][2 * k]     = csi;
    a.csi[0][2 * k + 1] = csi;
    mx[0]               = max(mx[0], __float_as_uint(csi));
  }
}

// srsran_predecoding_diversity_csi, 4 ports (precoding.c:714-775): thread k decodes the SFBC + FSTD
// group (4k .. 4k+3), ports (0, 2) on the first pair and (1, 3) on the second, for k < m_ap (a
// trailing half group is not decoded by the reference; the layer-demapped codeword gets 0 there).  CSI =
// a_l * scaling / nof_rxant per RE; with a.interleave the codeword is written layer-demapped (d[4k + l] = x_l[k]).
__device__ __forceinline__ void diversity_quad(const PredArgs& a, uint32_t k, uint32_t (&mx)[2])
{
  const uint32_t m_ap  = (a.n % 4) ? (a.n >= 2 ? (a.n - 2) / 4 : 0u) : a.n / 4;  // C int division of the reference
  const bool     valid = k < m_ap;
  const uint32_t kk    = valid ? k : 0;
  uint32_t       gy[4], gh[4];
  float          s[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    re_at(a, 4 * kk + j, gy[j], gh[j], s[j]);
  }
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  cpx   x0 = {0.f, 0.f}, x1 = {0.f, 0.f}, x2 = {0.f, 0.f}, x3 = {0.f, 0.f};
  if (!a.csi[0]) {
    // no CSI (the control channels, pcfich.c:202 / pdcch.c:498): srsran_predecoding_diversity_gen_,
    // 4 ports (precoding.c:465-499) -- one channel RE per pair, one gain per pair
    for (int p = 0; p < a.nrx; p++) {
      cpx r[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        r[j] = ld(a.y[p], gy[j]);
        if (s[j] != 1.0f) {
          r[j] = cscale(r[j], s[j]);
        }
      }
      const cpx h0 = ld(a.h[0][p], gh[0]), h1 = ld(a.h[1][p], gh[2]), h2 = ld(a.h[2][p], gh[0]),
                h3 = ld(a.h[3][p], gh[2]);
      a0 += h0.r * h0.r + h0.i * h0.i + h2.r * h2.r + h2.i * h2.i;
      a2 += h1.r * h1.r + h1.i * h1.i + h3.r * h3.r + h3.i * h3.i;
      x0 = cadd(x0, cadd(cmul(cconj(h0), r[0]), cmul(h2, cconj(r[1]))));
      x1 = cadd(x1, cadd(cmul(cneg(h2), cconj(r[0])), cmul(cconj(h0), r[1])));
      x2 = cadd(x2, cadd(cmul(cconj(h1), r[2]), cmul(h3, cconj(r[3]))));
      x3 = cadd(x3, cadd(cmul(cneg(h3), cconj(r[2])), cmul(cconj(h1), r[3])));
    }
    a0 *= a.norm;
    a2 *= a.norm;
    const float  g[4]  = {a0, a0, a2, a2};
    const cpx    xv[4] = {x0, x1, x2, x3};
    const double sq2   = 1.41421356237309504880;
    if (valid) {
#pragma unroll
      for (int l = 0; l < 4; l++) {
        const float2 o = make_float2((float)((double)(xv[l].r / g[l]) * sq2), (float)((double)(xv[l].i / g[l]) * sq2));
        if (a.interleave) {
          a.x[0][4 * k + l] = o;
        } else {
          a.x[l][k] = o;
        }
      }
    }
    return;
  }
  for (int p = 0; p < a.nrx; p++) {
    cpx r[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      r[j] = ld(a.y[p], gy[j]);
      if (s[j] != 1.0f) {
        r[j] = cscale(r[j], s[j]);
      }
    }
    cpx h00 = ld(a.h[0][p], gh[0]), h01 = ld(a.h[2][p], gh[0]), h10 = ld(a.h[0][p], gh[1]), h11 = ld(a.h[2][p], gh[1]);
    a0 += h00.r * h00.r + h00.i * h00.i + h11.r * h11.r + h11.i * h11.i;
    a1 += h10.r * h10.r + h10.i * h10.i + h01.r * h01.r + h01.i * h01.i;
    x0 = cadd(x0, cadd(cmul(cconj(h00), r[0]), cmul(h11, cconj(r[1]))));
    x1 = cadd(x1, cadd(cmul(cneg(h01), cconj(r[0])), cmul(cconj(h10), r[1])));
    h00 = ld(a.h[1][p], gh[2]), h01 = ld(a.h[3][p], gh[2]), h10 = ld(a.h[1][p], gh[3]), h11 = ld(a.h[3][p], gh[3]);
    a2 += h00.r * h00.r + h00.i * h00.i + h11.r * h11.r + h11.i * h11.i;
    a3 += h10.r * h10.r + h10.i * h10.i + h01.r * h01.r + h01.i * h01.i;
    x2 = cadd(x2, cadd(cmul(cconj(h00), r[2]), cmul(h11, cconj(r[3]))));
    x3 = cadd(x3, cadd(cmul(cneg(h01), cconj(r[2])), cmul(cconj(h10), r[3])));
  }
  const float  av[4] = {a0 * a.norm, a1 * a.norm, a2 * a.norm, a3 * a.norm};  // scaling
  const cpx    xv[4] = {x0, x1, x2, x3};
  const double sq2   = 1.41421356237309504880;
  if (valid) {
#pragma unroll
    for (int l = 0; l < 4; l++) {
      const float c           = av[l] / (float)a.nrx;
      const float2 o          = make_float2((float)((double)(xv[l].r / av[l]) * sq2), (float)((double)(xv[l].i / av[l]) * sq2));
      if (a.interleave) {
        a.x[0][4 * k + l] = o;  // srsran_layerdemap_diversity fused
      } else {
        a.x[l][k] = o;
      }
      a.csi[0][4 * k + l]     = c;
      mx[0]                   = max(mx[0], __float_as_uint(c));
    }
  } else if (k == m_ap && (a.n % 4) && a.interleave) {  // the undecoded half group
    for (uint32_t j = 4 * m_ap; j < a.n; j++) {
      a.x[0][j]   = make_float2(0.f, 0.f);
      a.csi[0][j] = 0.f;
    }
  }
}

template <int SCHEME>
__device__ __forceinline__ void predecode_item(const PredArgs& a, uint32_t k, uint32_t (&mx)[2])
{
  if constexpr (SCHEME == 1) {
    diversity_pair(a, k, mx);
    return;
  }
  if constexpr (SCHEME == 4) {
    diversity_quad(a, k, mx);
    return;
  }
  const bool     valid = k < a.n;
  const uint32_t kk    = valid ? k : 0;
  // grid / estimate positions of RE kk (fused srsran_pdsch_get)
  uint32_t gy = kk, gh = kk;
  float    ys = 1.0f;
  if (a.idx) {
    const uint32_t e = a.idx[kk];
    gy               = e & 0x7fffffffu;
    gh               = a.ce_row ? gy % a.ce_row : gy;
    ys               = (e >> 31) ? a.rho_b_inv : 1.0f;
  }
  const float noise = a.noise_ptr ? *a.noise_ptr : a.noise;
  auto        Y     = [&](int r) -> cpx {
    cpx v = ld(a.y[r], gy);
    if (ys != 1.0f) {
      v = cscale(v, ys);
    }
    return v;
  };
  if constexpr (SCHEME == 0) {
    cpx   r  = {0.f, 0.f};
    float hh = 0.f;
    for (int p = 0; p < a.nrx; p++) {
      const cpx hv = ld(a.h[0][p], gh);
      r            = cadd(r, cmul(Y(p), cconj(hv)));
      hh += hv.r * hv.r + hv.i * hv.i;
    }
    const float csi = hh + noise;
    const cpx   t   = cscale(r, a.norm);
    if (valid) {
      a.csi[0][k] = csi;
      a.x[0][k]   = make_float2(t.r / csi, t.i / csi);
    }
    if (valid) {
      mx[0] = max(mx[0], __float_as_uint(csi));
    }
  } else {
    const cpx p0 = ld(a.h[0][0], gh), p1 = ld(a.h[0][1], gh), q0 = ld(a.h[1][0], gh), q1 = ld(a.h[1][1], gh);
    cpx       h00, h01, h10, h11;
    if constexpr (SCHEME == 3) {  // CDD: the large-delay precoder alternates with the RE index
      if ((kk & 1) == 0) {
        h00 = cadd(p0, q0);
        h10 = cadd(p1, q1);
        h01 = csub(p0, q0);
        h11 = csub(p1, q1);
      } else {
        h00 = csub(p0, q0);
        h10 = csub(p1, q1);
        h01 = cadd(p0, q0);
        h11 = cadd(p1, q1);
      }
    } else {
      if (a.codebook == 0) {
        h00 = p0;
        h01 = q0;
        h10 = p1;
        h11 = q1;
      } else if (a.codebook == 1) {
        h00 = cadd(p0, q0);
        h01 = csub(p0, q0);
        h10 = cadd(p1, q1);
        h11 = csub(p1, q1);
      } else {
        h00 = cadd(p0, cmulj(q0));
        h01 = csub(p0, cmulj(q0));
        h10 = cadd(p1, cmulj(q1));
        h11 = csub(p1, cmulj(q1));
      }
    }
    cpx   x0, x1;
    float c0, c1;
    mmse_csi(Y(0), Y(1), h00, h01, h10, h11, x0, x1, c0, c1, noise, a.norm);
    if (valid) {
      if (a.interleave == 2) {  // one codeword on both layers: srsran_layerdemap_multiplex -> _diversity
        if (k < a.n / 2) {      // (layermap.c:138-147) over n/2 layer symbols (pdsch.c:862-863)
          a.x[0][2 * k]     = make_float2(x0.r, x0.i);
          a.x[0][2 * k + 1] = make_float2(x1.r, x1.i);
        }
      } else {
        a.x[0][k] = make_float2(x0.r, x0.i);
        a.x[1][k] = make_float2(x1.r, x1.i);
      }
      a.csi[0][k] = c0;  // not layer-demapped: the codeword's CSI correction reads layer 0's (pdsch.c:530)
      a.csi[1][k] = c1;
    }
    if (valid) {
      mx[0] = max(mx[0], __float_as_uint(c0));
      mx[1] = max(mx[1], __float_as_uint(c1));
    }
  }
}

static constexpr int EQ_RPT = 4;  // REs per thread (strided by the block size: coalesced)

// predecode_item for the EQ_RPT REs of a thread at once (PORT0, SM, CDD): every RE-map entry first, then
// every grid / estimate load, then the arithmetic (eq_dev.h, shared with the fused predecode + LLR kernel) and the
// stores -- two HBM round trips a thread instead of two per RE.  CSI_ONLY: the CSI maxima only (no received
// samples read, nothing stored) -- the pre-pass of the fused path (pdsch_api.cpp)
template <int SCHEME, bool CSI_ONLY = false>
__device__ __forceinline__ void predecode_items(const PredArgs& a, uint32_t k0, uint32_t (&mx)[2])
{
  static_assert(SCHEME == 0 || SCHEME == 2 || SCHEME == 3, "one RE per unit");
  constexpr int U = EQ_RPT;
  uint32_t      k[U], kk[U], gy[U], gh[U];
  float         ys[U];
  bool          valid[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    k[u]     = k0 + u * EQ_THREADS + threadIdx.x;
    valid[u] = k[u] < a.n;
    kk[u]    = valid[u] ? k[u] : 0;
    gy[u]    = kk[u];
    gh[u]    = kk[u];
    ys[u]    = 1.0f;
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
      if (CSI_ONLY && a.pairs) {
        kk[u] = e[u] >> 31;  // the RE parity of the pair (CDD's precoder); ys is unused here
      }
    }
  }
  const float noise = a.noise_ptr ? *gptr(a.noise_ptr) : a.noise;
  auto        Ys    = [&](eqd::cpx v, int u) -> eqd::cpx { return ys[u] != 1.0f ? eqd::cscale(v, ys[u]) : v; };
  if constexpr (SCHEME == 0) {
    eqd::cpx yv[U][4], hv[U][4];
#pragma unroll
    for (int u = 0; u < U; u++) {
#pragma unroll
      for (int p = 0; p < 4; p++) {
        if (p < a.nrx) {
          yv[u][p] = CSI_ONLY ? eqd::cpx{0.f, 0.f} : eqd::ld(a.y[p], gy[u]);
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
      float    csi;
      eqd::port0(y, hv[u], a.nrx, noise, a.norm, x, csi);
      if (valid[u]) {
        if (!CSI_ONLY) {
          gptr(a.csi[0])[k[u]] = csi;
          gptr(a.x[0])[k[u]]   = make_float2(x.r, x.i);
        }
        mx[0] = max(mx[0], __float_as_uint(csi));
      }
    }
  } else {
    eqd::cpx y0[U], y1[U], p0[U], p1[U], q0[U], q1[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      p0[u] = eqd::ld(a.h[0][0], gh[u]);
      p1[u] = eqd::ld(a.h[0][1], gh[u]);
      q0[u] = eqd::ld(a.h[1][0], gh[u]);
      q1[u] = eqd::ld(a.h[1][1], gh[u]);
      y0[u] = CSI_ONLY ? eqd::cpx{0.f, 0.f} : eqd::ld(a.y[0], gy[u]);
      y1[u] = CSI_ONLY ? eqd::cpx{0.f, 0.f} : eqd::ld(a.y[1], gy[u]);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      eqd::cpx h00, h01, h10, h11;
      eqd::effective_h<SCHEME>(a.codebook, kk[u], p0[u], p1[u], q0[u], q1[u], h00, h01, h10, h11);
      eqd::cpx x0, x1;
      float    c0, c1;
      eqd::mmse_csi(Ys(y0[u], u), Ys(y1[u], u), h00, h01, h10, h11, x0, x1, c0, c1, noise, a.norm);
      if (valid[u]) {
        if (!CSI_ONLY) {
          if (a.interleave == 2) {    // one codeword on both layers: srsran_layerdemap_multiplex -> _diversity
            if (k[u] < a.n / 2) {     // (layermap.c:138-147) over n/2 layer symbols (pdsch.c:862-863)
              gptr(a.x[0])[2 * k[u]]     = make_float2(x0.r, x0.i);
              gptr(a.x[0])[2 * k[u] + 1] = make_float2(x1.r, x1.i);
            }
          } else {
            gptr(a.x[0])[k[u]] = make_float2(x0.r, x0.i);
            gptr(a.x[1])[k[u]] = make_float2(x1.r, x1.i);
          }
          gptr(a.csi[0])[k[u]] = c0;  // not layer-demapped: the codeword's CSI correction reads layer 0's
          gptr(a.csi[1])[k[u]] = c1;
        }
        mx[0] = max(mx[0], __float_as_uint(c0));
        mx[1] = max(mx[1], __float_as_uint(c1));
      }
    }
  }
}

template <int SCHEME, bool CSI_ONLY = false>
__device__ __forceinline__ void predecode_block(const PredArgs& a, uint32_t k0)
{
  __shared__ uint32_t red[2 * EQ_THREADS / 64];
  uint32_t            mx[2] = {0u, 0u};
  if constexpr (SCHEME == 0 || SCHEME == 2 || SCHEME == 3) {
    predecode_items<SCHEME, CSI_ONLY>(a, k0, mx);
  } else {
#pragma unroll
    for (int r = 0; r < EQ_RPT; r++) {
      predecode_item<SCHEME>(a, k0 + r * EQ_THREADS + threadIdx.x, mx);
    }
  }
  if (a.csi_max) {
    if constexpr (SCHEME == 0 || SCHEME == 1 || SCHEME == 4) {
      const uint32_t m1[1] = {mx[0]};
      block_max_atomic<1>(a.csi_max, m1, red);
    } else {
      block_max_atomic<2>(a.csi_max, mx, red);
    }
  }
}

template <int SCHEME>
__global__ __launch_bounds__(EQ_THREADS) void predecode_kernel(PredArgs a)
{
  predecode_block<SCHEME>(a, blockIdx.x * EQ_THREADS * EQ_RPT);
}

template <int SCHEME, bool CSI_ONLY = false>
__global__ __launch_bounds__(EQ_THREADS) void predecode_batch_kernel(const PredArgs* __restrict__ items)
{
  const PredArgs& a  = items[blockIdx.y];
  const uint32_t  k0 = blockIdx.x * EQ_THREADS * EQ_RPT;
  if (k0 >= (SCHEME == 1 ? a.n / 2 : SCHEME == 4 ? a.n / 4 + 1 : a.n)) {
    return;  // whole block past this item's end (uniform: the block reduction stays intact)
  }
  predecode_block<SCHEME, CSI_ONLY>(a, k0);
}

hipError_t csi_max_batch_launch(const PredArgs* d_items, uint32_t nitems, int scheme, uint32_t max_n, hipStream_t stream)
{
  StageScope timing_scope(ST_PRED, stream);
  if (nitems == 0 || max_n == 0) {
    return hipSuccess;
  }
  const dim3 grid((max_n + EQ_THREADS * EQ_RPT - 1) / (EQ_THREADS * EQ_RPT), nitems);
  switch (scheme) {
    case 0:
      hipLaunchKernelGGL((predecode_batch_kernel<0, true>), grid, dim3(EQ_THREADS), 0, stream, d_items);
      break;
    case 2:
      hipLaunchKernelGGL((predecode_batch_kernel<2, true>), grid, dim3(EQ_THREADS), 0, stream, d_items);
      break;
    case 3:
      hipLaunchKernelGGL((predecode_batch_kernel<3, true>), grid, dim3(EQ_THREADS), 0, stream, d_items);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t predecode_batch_launch(const PredArgs* d_items, uint32_t nitems, int scheme, uint32_t max_n,
                                  hipStream_t stream)
{
  StageScope timing_scope(ST_PRED, stream);
  if (nitems == 0 || max_n == 0) {
    return hipSuccess;
  }
  // diversity: one thread per SFBC pair (2 ports) or SFBC + FSTD group (4 ports, + 1 for a half group)
  const uint32_t units = scheme == 1 ? max_n / 2 : scheme == 4 ? max_n / 4 + 1 : max_n;
  if (units == 0) {
    return hipSuccess;
  }
  const dim3 grid((units + EQ_THREADS * EQ_RPT - 1) / (EQ_THREADS * EQ_RPT), nitems);
  switch (scheme) {
    case 0:
      hipLaunchKernelGGL(predecode_batch_kernel<0>, grid, dim3(EQ_THREADS), 0, stream, d_items);
      break;
    case 1:
      hipLaunchKernelGGL(predecode_batch_kernel<1>, grid, dim3(EQ_THREADS), 0, stream, d_items);
      break;
    case 2:
      hipLaunchKernelGGL(predecode_batch_kernel<2>, grid, dim3(EQ_THREADS), 0, stream, d_items);
      break;
    case 3:
      hipLaunchKernelGGL(predecode_batch_kernel<3>, grid, dim3(EQ_THREADS), 0, stream, d_items);
      break;
    case 4:
      hipLaunchKernelGGL(predecode_batch_kernel<4>, grid, dim3(EQ_THREADS), 0, stream, d_items);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t predecode_launch(const PredArgs& a, hipStream_t stream)
{
  StageScope timing_scope(ST_PRED, stream);
  if (a.n == 0) {
    return hipSuccess;
  }
  const uint32_t units = a.scheme == 1 ? a.n / 2 : a.scheme == 4 ? a.n / 4 + 1 : a.n;
  if (units == 0) {
    return hipSuccess;
  }
  const dim3 grid((units + EQ_THREADS * EQ_RPT - 1) / (EQ_THREADS * EQ_RPT));
  switch (a.scheme) {
    case 0:
      hipLaunchKernelGGL(predecode_kernel<0>, grid, dim3(EQ_THREADS), 0, stream, a);
      break;
    case 1:
      hipLaunchKernelGGL(predecode_kernel<1>, grid, dim3(EQ_THREADS), 0, stream, a);
      break;
    case 2:
      hipLaunchKernelGGL(predecode_kernel<2>, grid, dim3(EQ_THREADS), 0, stream, a);
      break;
    case 3:
      hipLaunchKernelGGL(predecode_kernel<3>, grid, dim3(EQ_THREADS), 0, stream, a);
      break;
    case 4:
      hipLaunchKernelGGL(predecode_kernel<4>, grid, dim3(EQ_THREADS), 0, stream, a);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace srsran_amd
