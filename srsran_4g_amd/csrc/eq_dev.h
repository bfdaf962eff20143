// srsran_4g_amd/csrc/eq_dev.h -- the predecoder's per-RE arithmetic, shared by the predecoder kernels
// (eq_kernel.hip) and the fused predecode + LLR kernel (llr_kernel.hip), so both compute the same floats.
//
// Formulas of the reference's CSI predecoders (precoding.c:307-355 PORT0, 1043-1121 CDD, 1437-1540 SM;
// mat.c:63-109 srsran_mat_2x2_mmse_csi_gen) in IEEE float with the scalar ("gen") operation order and no FMA
// contraction (each function body opts out of contraction, whatever the including file does).
#ifndef SRSRAN_AMD_EQ_DEV_H
#define SRSRAN_AMD_EQ_DEV_H
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "eq_kernel.h"
#include "gmem.h"

namespace srsran_amd {
namespace eqd {

struct cpx {
  float r, i;
};
// every operation carries "no contraction" (the pragma in each body), so the including file's FP-contract mode
// cannot fuse a product of one helper into a sum of another
__device__ __forceinline__ cpx cadd(cpx a, cpx b)
{
#pragma clang fp contract(off)
  return {a.r + b.r, a.i + b.i};
}
__device__ __forceinline__ cpx csub(cpx a, cpx b)
{
#pragma clang fp contract(off)
  return {a.r - b.r, a.i - b.i};
}
__device__ __forceinline__ cpx cmul(cpx a, cpx b)
{
#pragma clang fp contract(off)
  return {a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r};
}
__device__ __forceinline__ cpx cconj(cpx a) { return {a.r, -a.i}; }
__device__ __forceinline__ cpx cneg(cpx a) { return {-a.r, -a.i}; }
__device__ __forceinline__ cpx cscale(cpx a, float s)
{
#pragma clang fp contract(off)
  return {a.r * s, a.i * s};
}
__device__ __forceinline__ cpx cmulj(cpx a) { return {-a.i, a.r}; }
__device__ __forceinline__ cpx ld(const float2* p, uint32_t k)
{
  const float2 v = gptr(p)[k];  // global address space (gmem.h): the pointers come from descriptors
  return {v.x, v.y};
}

// srsran_mat_2x2_mmse_csi_gen: x = (H^H H + noise I)^-1 H^H y * norm, csi_l = 1 / Re(B_ll)
__device__ __forceinline__ void mmse_csi(cpx y0, cpx y1, cpx h00, cpx h01, cpx h10, cpx h11, cpx& x0, cpx& x1,
                                         float& csi0, float& csi1, float noise, float norm)
{
#pragma clang fp contract(off)
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

// the 2x2 effective channel of RE kk: CDD's large-delay precoder alternates with the RE index (SCHEME 3); SM
// (SCHEME 2) applies codebook 0..2 (precoding.c:1437-1540)
template <int SCHEME>
__device__ __forceinline__ void effective_h(int codebook, uint32_t kk, cpx p0, cpx p1, cpx q0, cpx q1, cpx& h00,
                                            cpx& h01, cpx& h10, cpx& h11)
{
  if constexpr (SCHEME == 3) {
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
    if (codebook == 0) {
      h00 = p0;
      h01 = q0;
      h10 = p1;
      h11 = q1;
    } else if (codebook == 1) {
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
}

// srsran_predecoding_single_csi (precoding.c:307-355) over nrx antennas: x = norm sum(y conj h) / csi,
// csi = sum |h|^2 + noise
__device__ __forceinline__ void port0(const cpx* y, const cpx* h, int nrx, float noise, float norm, cpx& x,
                                      float& csi)
{
#pragma clang fp contract(off)
  cpx   r  = {0.f, 0.f};
  float hh = 0.f;
#pragma unroll
  for (int p = 0; p < 4; p++) {
    if (p < nrx) {
      r = cadd(r, cmul(y[p], cconj(h[p])));
      hh += h[p].r * h[p].r + h[p].i * h[p].i;
    }
  }
  csi         = hh + noise;
  const cpx t = cscale(r, norm);
  x           = {t.r / csi, t.i / csi};
}

// RE-map entry e of the fused srsran_pdsch_get: grid index, estimate index, y scale (rho_b on CRS symbols)
__device__ __forceinline__ void re_pos(const PredArgs& a, uint32_t e, uint32_t& gy, uint32_t& gh, float& ys)
{
  gy = e & 0x7fffffffu;
  gh = a.ce_row ? gy % a.ce_row : gy;
  ys = (e >> 31) ? a.rho_b_inv : 1.0f;
}

}  // namespace eqd
}  // namespace srsran_amd
#endif
