// srsran_4g_amd/csrc/pusch_kernel.hip -- PUSCH receive kernels for CDNA4.
//
//   chest_ul_kernel      srsran_chest_ul_estimate_pusch (chest_ul.c:298-433): DMRS least squares
//                        (srsran_vec_prod_conj_ccc), 3-tap smoothing with the extrapolated edges of
//                        srsran_conv_same_cf (convolution.c:182-219), copy to every symbol of the slot
//                        (interpolate_pilots without DO_LINEAR_INTERPOLATION), noise from the
//                        smoothed-vs-raw difference (estimate_noise_pilots), CFO from the slot-to-slot
//                        correlation, TA from srsran_vec_estimate_frequency, RSRP / EPRE.
//   pusch_eq_idft_kernel pusch_get + srsran_predecoding_single (precoding.c:182-305, ZF / MMSE with
//                        the chest noise) + srsran_dft_precoding (dft_precoding.c:114-126): the
//                        M-point backward DFT normalised by 1 / sqrt(M) of every data symbol.
//
// Layout: one workgroup per UE for the estimator (2M <= 2400 pilots, all reductions in one pass),
// one workgroup per (data symbol, UE) for the de-precoder.  The DFT is a mixed-radix Stockham
// autosort transform in LDS (radices 4, 2, 3, 5; M = 12 L with L = 2^a 3^b 5^c <= 100): every
// stage reads and writes LDS once, 256 threads cover the <= 600 butterflies of a stage, twiddles
// come from sincospif (no table traffic).  Both kernels are HBM-bound elementwise work (the grid
// and the estimate are read once per data RE); floating point, compared with the oracle within a
// tolerance (the reference's DFT is FFTW, absent here).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pusch_kernel.h"
#include "stage_timing.h"

namespace srsran_amd {

static constexpr int PU_THREADS = 256;

struct c2 {
  float r, i;
};
__device__ __forceinline__ c2 mk(float2 v) { return {v.x, v.y}; }
__device__ __forceinline__ c2 add(c2 a, c2 b) { return {a.r + b.r, a.i + b.i}; }
__device__ __forceinline__ c2 sub(c2 a, c2 b) { return {a.r - b.r, a.i - b.i}; }
__device__ __forceinline__ c2 mul(c2 a, c2 b) { return {a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r}; }
__device__ __forceinline__ c2 mulconj(c2 a, c2 b) { return {a.r * b.r + a.i * b.i, a.i * b.r - a.r * b.i}; }  // a conj(b)
__device__ __forceinline__ c2 scl(c2 a, float s) { return {a.r * s, a.i * s}; }
__device__ __forceinline__ c2 mulj(c2 a) { return {-a.i, a.r}; }

// sum over the block of NV floats per thread; every thread gets the totals
template <int NV>
__device__ __forceinline__ void block_sum(float (&v)[NV], float* red)
{
#pragma unroll
  for (int k = 0; k < NV; k++) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      v[k] += __shfl_xor(v[k], off, 64);
    }
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int k = 0; k < NV; k++) {
      red[w * NV + k] = v[k];
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; k++) {
    float s = 0.f;
    for (int i = 0; i < nw; i++) {
      s += red[i * NV + k];
    }
    v[k] = s;
  }
}

// ---------------------------------------------------------------- channel estimation
// 16 waves a UE: 78 UEs are 78 workgroups, so each one's 2 M pilots and 14 M estimate stores spread over more
// threads (the estimate copy to every symbol of the slot is most of the kernel's bytes)
static constexpr int CHUL_THREADS = 1024;

__global__ __launch_bounds__(CHUL_THREADS) void chest_ul_kernel(const PuschUe* __restrict__ ues)
{
  const PuschUe& u = ues[blockIdx.x];
  __shared__ float2 pe[2 * PUSCH_MAX_M];
  __shared__ float  red[(CHUL_THREADS / 64) * 11];
  const uint32_t    M = u.M;

  // LS estimates; received pilot sum and power
  float acc[11] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (uint32_t k = threadIdx.x; k < 2 * M; k += CHUL_THREADS) {
    const uint32_t s = k >= M ? 1u : 0u, j = k - s * M;
    const uint32_t L = (s + 1) * u.nsym_slot - 4;
    const c2       rx = mk(u.grid[(size_t)L * u.ncell_re + u.n_tilde[s] * 12 + j]);
    const c2       e  = mulconj(rx, mk(u.dmrs[k]));
    pe[k]             = make_float2(e.r, e.i);
    acc[0] += rx.r, acc[1] += rx.i, acc[2] += rx.r * rx.r + rx.i * rx.i;
  }
  __syncthreads();

  // smoothing, estimate grid, noise, CFO and TA correlations
  const float f0 = u.filt[0], f1 = u.filt[1], f2 = u.filt[2];
  for (uint32_t k = threadIdx.x; k < 2 * M; k += CHUL_THREADS) {
    const uint32_t s = k >= M ? 1u : 0u, j = k - s * M;
    const float2*  p = pe + s * M;
    const c2       x = mk(p[j]);
    c2             a = x;
    if (u.smooth) {
      c2 l, r;
      if (j == 0) {
        l = sub(scl(mk(p[1]), 3.0f), scl(mk(p[0]), 2.0f));
      } else {
        l = mk(p[j - 1]);
      }
      if (j == M - 1) {
        r = sub(scl(mk(p[M - 1]), 3.0f), scl(mk(p[M - 2]), 2.0f));
      } else {
        r = mk(p[j + 1]);
      }
      a = add(add(scl(l, f0), scl(x, f1)), scl(r, f2));
      const c2 d = sub(a, x);
      acc[3 + s] += d.r * d.r + d.i * d.i;
    }
    const float2 av = make_float2(a.r, a.i);
    for (uint32_t i = 0; i < u.nsym_slot; i++) {
      u.ce[(size_t)(s * u.nsym_slot + i) * u.ncell_re + u.n_prb[s] * 12 + j] = av;
    }
    if (s == 0) {
      const c2 c = mulconj(x, mk(pe[M + j]));
      acc[5] += c.r, acc[6] += c.i;
    }
    if (u.meas_ta && j > 0) {
      const c2 c = mulconj(x, mk(p[j - 1]));
      acc[7 + 2 * s] += c.r, acc[8 + 2 * s] += c.i;
    }
  }
  block_sum<11>(acc, red);
  if (threadIdx.x == 0) {
    ChestUlOut o;
    o.cfo_hz = atan2f(acc[6], acc[5]) / (2.0f * 3.14159265358979323846f * 0.0005f);
    float ta = 0.0f;
    if (u.meas_ta) {
      for (int s = 0; s < 2; s++) {
        const float f = (float)((double)-atan2f(acc[8 + 2 * s], acc[7 + 2 * s]) * 0.31830988618379067154 * 0.5);
        ta += f / 2.0f;
      }
    }
    if (isnormal(ta)) {
      ta /= 15e3f;
      ta *= 1e6f;
      ta = roundf(ta * 10.0f) / 10.0f;
    } else {
      ta = 0.0f;
    }
    o.ta_us = ta;
    if (u.smooth) {
      float power = acc[3] / (float)M;
      power += acc[4] / (float)M;
      power /= 2.0f;
      o.noise = (float)((double)power / u.noise_div);
    } else {
      o.noise = 0.0f;
    }
    const float n2   = (float)(2 * M);
    const float cr   = acc[0] / n2, ci = acc[1] / n2;
    const float epre = acc[2] / n2;
    o.rsrp           = fminf(cr * cr + ci * ci, epre);
    o.epre           = epre;
    o.data_pow       = 0.0f;
    *u.out           = o;
  }
}

hipError_t chest_ul_launch(const PuschUe* d_ues, uint32_t nue, hipStream_t stream)
{
  if (nue == 0) {
    return hipSuccess;
  }
  StageScope timing_scope(ST_CHEST_UL, stream);
  hipLaunchKernelGGL(chest_ul_kernel, dim3(nue), dim3(CHUL_THREADS), 0, stream, d_ues);
  return hipGetLastError();
}

// ---------------------------------------------------------------- equaliser + inverse DFT
// one radix-R Stockham stage (backward transform: twiddles and butterflies e^{+j...})
template <int R>
__device__ __forceinline__ void stage(const float2* __restrict__ in, float2* __restrict__ out, uint32_t N, uint32_t Ns)
{
  const uint32_t nb = N / R;
  for (uint32_t j = threadIdx.x; j < nb; j += PU_THREADS) {
    const uint32_t k = j % Ns;
    c2             v[R];
    v[0] = mk(in[j]);
#pragma unroll
    for (int r = 1; r < R; r++) {
      float sn, cs;
      sincospif(2.0f * (float)(r * k) / (float)(Ns * R), &sn, &cs);
      v[r] = mul(mk(in[j + r * nb]), c2{cs, sn});
    }
    c2 y[R];
    if (R == 2) {
      y[0] = add(v[0], v[1]);
      y[1] = sub(v[0], v[1]);
    } else if (R == 4) {
      const c2 s02 = add(v[0], v[2]), d02 = sub(v[0], v[2]);
      const c2 s13 = add(v[1], v[3]), d13 = mulj(sub(v[1], v[3]));
      y[0] = add(s02, s13);
      y[1] = add(d02, d13);
      y[2] = sub(s02, s13);
      y[3] = sub(d02, d13);
    } else if (R == 3) {
      const float h = 0.86602540378443864676f;  // sin(2 pi / 3)
      const c2    t = add(v[1], v[2]);
      const c2    m = sub(v[0], scl(t, 0.5f));
      const c2    d = mulj(scl(sub(v[1], v[2]), h));
      y[0]          = add(v[0], t);
      y[1]          = add(m, d);
      y[2]          = sub(m, d);
    } else {  // R == 5
      const float c1 = 0.30901699437494742410f, c2c = -0.80901699437494742410f;
      const float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
      const c2    t1 = add(v[1], v[4]), t2 = add(v[2], v[3]);
      const c2    d1 = sub(v[1], v[4]), d2 = sub(v[2], v[3]);
      const c2    a1 = add(v[0], add(scl(t1, c1), scl(t2, c2c)));
      const c2    a2 = add(v[0], add(scl(t1, c2c), scl(t2, c1)));
      const c2    b1 = mulj(add(scl(d1, s1), scl(d2, s2)));
      const c2    b2 = mulj(sub(scl(d1, s2), scl(d2, s1)));
      y[0]           = add(v[0], add(t1, t2));
      y[1]           = add(a1, b1);
      y[4]           = sub(a1, b1);
      y[2]           = add(a2, b2);
      y[3]           = sub(a2, b2);
    }
    const uint32_t o = (j / Ns) * Ns * R + k;
#pragma unroll
    for (int r = 0; r < R; r++) {
      out[o + r * Ns] = make_float2(y[r].r, y[r].i);
    }
  }
}

__global__ __launch_bounds__(PU_THREADS) void pusch_eq_idft_kernel(const PuschUe* __restrict__ ues)
{
  const PuschUe& u = ues[blockIdx.y];
  const uint32_t l = blockIdx.x;
  if (l >= u.nof_symb) {
    return;
  }
  __shared__ float2 buf[2][PUSCH_MAX_M];
  __shared__ float  red[PU_THREADS / 64];
  const uint32_t    M     = u.M;
  const uint32_t    g     = u.data_sym[l];
  const uint32_t    slot  = g >= u.nsym_slot ? 1u : 0u;
  const size_t      base  = (size_t)g * u.ncell_re + u.n_tilde[slot] * 12;
  const float       noise = u.noise_dev && u.out ? u.out->noise : u.noise;
  const uint32_t    nre   = M * u.nof_symb, nvec = 8 * (nre / 8);

  // srsran_predecoding_single: x = y conj(h) / (|h|^2 + n0); the 8-wide AVX body adds n0 only
  // when it is positive, the scalar tail always
  float pw[1] = {0.f};
  for (uint32_t j = threadIdx.x; j < M; j += PU_THREADS) {
    const c2 y = mk(u.grid[base + j]);
    if (u.ce) {
      const c2    h  = mk(u.ce[base + j]);
      const float hh = h.r * h.r + h.i * h.i;
      const float dn = (l * M + j < nvec) ? (noise > 0.0f ? hh + noise : hh) : hh + noise;
      const c2    z  = mulconj(y, h);
      buf[0][j]      = make_float2(z.r / dn, z.i / dn);
    } else {  // plain transform de-precoding (srsran_dft_precoding)
      buf[0][j] = make_float2(y.r, y.i);
    }
    pw[0] += y.r * y.r + y.i * y.i;
  }
  block_sum<1>(pw, red);
  if (threadIdx.x == 0 && u.out) {
    atomicAdd(&u.out->data_pow, pw[0]);
  }
  __syncthreads();

  uint32_t Ns = 1, cur = 0;
  for (uint32_t st = 0; st < u.nstages; st++) {
    const uint32_t R = u.radix[st];
    if (R == 4) {
      stage<4>(buf[cur], buf[cur ^ 1], M, Ns);
    } else if (R == 2) {
      stage<2>(buf[cur], buf[cur ^ 1], M, Ns);
    } else if (R == 3) {
      stage<3>(buf[cur], buf[cur ^ 1], M, Ns);
    } else {
      stage<5>(buf[cur], buf[cur ^ 1], M, Ns);
    }
    Ns *= R;
    cur ^= 1;
    __syncthreads();
  }
  float2* o = u.sym + (size_t)l * M;
  for (uint32_t j = threadIdx.x; j < M; j += PU_THREADS) {
    const float2 v = buf[cur][j];
    o[j]           = make_float2(v.x * u.dft_norm, v.y * u.dft_norm);
  }
}

hipError_t pusch_eq_idft_launch(const PuschUe* d_ues, uint32_t nue, hipStream_t stream)
{
  if (nue == 0) {
    return hipSuccess;
  }
  StageScope timing_scope(ST_PUSCH_EQ, stream);
  hipLaunchKernelGGL(pusch_eq_idft_kernel, dim3(14, nue), dim3(PU_THREADS), 0, stream, d_ues);
  return hipGetLastError();
}

}  // namespace srsran_amd
