// srsran_4g_amd/csrc/ofdm_kernel.hip -- OFDM receiver for CDNA4.
//
// srsran_ofdm_rx_sf (ofdm.c:551-563 -> ofdm_rx_slot 474-520) as srsran_ue_dl configures it
// (ue_dl.c:88-98: no window offset, no normalisation, DC removed): symbol i of slot s starts
// at s * slot_sz + cp0 + i * (N + cp) (the guru plan of ofdm.c:169-181), forward DFT
// (FFTW_FORWARD), then the fftshift that drops the DC bin (ofdm.c:497-498): grid[0..nre/2) =
// X[N - nre/2 ..), grid[nre/2 ..) = X[1 .. nre/2].  srsran_cfo_correct's rotation
// (cfo.c:96-107, vector_simd.c:1723-1774) can be folded into the sample load.
//
// One workgroup per OFDM symbol: the N samples are rotated on load into LDS, transformed by
// a mixed-radix (8/4/3/2) Stockham FFT in one LDS buffer (natural-order output, no bit
// reversal), and only the nre occupied subcarriers are written back.  Twiddles come from
// a per-N table computed in double precision on the host.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

#include "ofdm_kernel.h"
#include "stage_timing.h"

namespace srsran_amd {

#ifndef OFDM_THREADS_CFG
#define OFDM_THREADS_CFG 256
#endif
static constexpr int OFDM_THREADS = OFDM_THREADS_CFG;  // a workgroup per symbol

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b)
{
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }  // * (-i)
// srsran_simd_cf_prod of the AVX2 + FMA build (simd.h:898-901) and gcc's contraction of the scalar
// complex products around it: re = fma(a.re, b.re, -(a.im b.im)), im = fma(a.re, b.im, a.im b.re), the inner
// products rounded on their own
__device__ __forceinline__ float2 ref_cprod(float2 a, float2 b)
{
  return make_float2(__fmaf_rn(a.x, b.x, -__fmul_rn(a.y, b.y)), __fmaf_rn(a.x, b.y, __fmul_rn(a.y, b.x)));
}

__device__ __forceinline__ void dft2(float2* v)
{
  const float2 a = v[0];
  v[0]           = cadd(a, v[1]);
  v[1]           = csub(a, v[1]);
}
__device__ __forceinline__ void dft4(float2* v)
{
  const float2 a0 = cadd(v[0], v[2]), a1 = csub(v[0], v[2]);
  const float2 a2 = cadd(v[1], v[3]), a3 = mul_mi(csub(v[1], v[3]));
  v[0]            = cadd(a0, a2);
  v[2]            = csub(a0, a2);
  v[1]            = cadd(a1, a3);
  v[3]            = csub(a1, a3);
}
__device__ __forceinline__ void dft3(float2* v)
{
  const float  s   = 0.86602540378443864676f;  // sqrt(3)/2
  const float2 sum = cadd(v[1], v[2]);
  const float2 t1  = make_float2(v[0].x - 0.5f * sum.x, v[0].y - 0.5f * sum.y);
  const float2 d   = csub(v[1], v[2]);
  const float2 t2  = make_float2(d.y * s, -d.x * s);  // (x1 - x2) * (-i sqrt(3)/2)
  v[0]             = cadd(v[0], sum);
  v[1]             = cadd(t1, t2);
  v[2]             = csub(t1, t2);
}
__device__ __forceinline__ void dft8(float2* v)
{
  float2 e[4] = {v[0], v[2], v[4], v[6]}, o[4] = {v[1], v[3], v[5], v[7]};
  dft4(e);
  dft4(o);
  const float r = 0.70710678118654752440f;
  o[1]          = make_float2((o[1].x + o[1].y) * r, (o[1].y - o[1].x) * r);    // * e^{-i pi/4}
  o[2]          = mul_mi(o[2]);                                                  // * e^{-i pi/2}
  o[3]          = make_float2((-o[3].x + o[3].y) * r, (-o[3].y - o[3].x) * r);  // * e^{-3i pi/4}
#pragma unroll
  for (int k = 0; k < 4; k++) {
    v[k]     = cadd(e[k], o[k]);
    v[k + 4] = csub(e[k], o[k]);
  }
}

// j / Ns for j < 2^16 and Ns <= 2^12 with m = ceil(2^32 / Ns) (exact in that range)
__device__ __forceinline__ uint32_t divm(uint32_t j, uint32_t m) { return __umulhi(j, m); }

// One Stockham stage of radix R (natural-order output), in place in one LDS buffer: every thread holds its butterflies' inputs in registers
// across a barrier (at most N / OFDM_THREADS values), so a symbol needs 16 KB of LDS
// instead of the 32 KB of a ping-pong pair -- 8 workgroups a CU instead of 5 (the launch is ~2200 symbols)
template <int R>
__device__ __forceinline__ void stage_ip(float2* buf, const float2* __restrict__ tw, uint32_t N, uint32_t Ns,
                                         uint32_t mNs)
{
  // butterflies per thread: N / R <= J * OFDM_THREADS (radix 3 only divides N = 3 * 2^k <= 1536)
  constexpr int  J  = ((R == 3 ? 1536 : OFDM_MAX_N) / R + OFDM_THREADS - 1) / OFDM_THREADS;
  const uint32_t nb = N / R, tstep = N / (Ns * R);
  float2 v[J][R], w[J][R];  // w: twiddles, loaded first (independent of the data) so their latency overlaps
#pragma unroll
  for (int jj = 0; jj < J; jj++) {
    const uint32_t j = threadIdx.x + jj * OFDM_THREADS;
    if (j < nb && Ns > 1) {
      const uint32_t k = j - divm(j, mNs) * Ns;
#pragma unroll
      for (int r = 1; r < R; r++) {
        w[jj][r] = tw[r * k * tstep];
      }
    }
  }
#pragma unroll
  for (int jj = 0; jj < J; jj++) {
    const uint32_t j = threadIdx.x + jj * OFDM_THREADS;
    if (j < nb) {
#pragma unroll
      for (int r = 0; r < R; r++) {
        v[jj][r] = buf[j + r * nb];
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int jj = 0; jj < J; jj++) {
    const uint32_t j = threadIdx.x + jj * OFDM_THREADS;
    if (j < nb) {
      const uint32_t q = Ns > 1 ? divm(j, mNs) : j;
      const uint32_t k = j - q * Ns;
      if (Ns > 1) {
#pragma unroll
        for (int r = 1; r < R; r++) {
          v[jj][r] = cmul(v[jj][r], w[jj][r]);
        }
      }
      if constexpr (R == 8) {
        dft8(v[jj]);
      } else if constexpr (R == 4) {
        dft4(v[jj]);
      } else if constexpr (R == 3) {
        dft3(v[jj]);
      } else {
        dft2(v[jj]);
      }
      const uint32_t base = q * Ns * R + k;
#pragma unroll
      for (int r = 0; r < R; r++) {
        buf[base + r * Ns] = v[jj][r];
      }
    }
  }
  __syncthreads();
}

// the plan's stages in place on buf (barriers included)
__device__ __forceinline__ void fft_ip(float2* buf, const OfdmArgs& a)
{
  uint32_t Ns = 1;
  for (int st = 0; st < a.nstages; st++) {
    const int      R   = a.radix[st];
    const uint32_t mNs = a.ns_magic[st];
    if (R == 8) {
      stage_ip<8>(buf, a.tw, a.N, Ns, mNs);
    } else if (R == 4) {
      stage_ip<4>(buf, a.tw, a.N, Ns, mNs);
    } else if (R == 3) {
      stage_ip<3>(buf, a.tw, a.N, Ns, mNs);
    } else {
      stage_ip<2>(buf, a.tw, a.N, Ns, mNs);
    }
    Ns *= (uint32_t)R;
  }
}

// One Stockham stage with N and Ns known at compile time: the butterflies, twiddles and LDS traffic of stage_ip,
// its index arithmetic folded (j / Ns a shift, the twiddle stride a constant)
template <int R, uint32_t N, uint32_t NS>
__device__ __forceinline__ void stage_ct(float2* buf, const float2* __restrict__ tw)
{
  constexpr int      J  = (N / R + OFDM_THREADS - 1) / OFDM_THREADS;
  constexpr uint32_t nb = N / R, tstep = N / (NS * R);
  float2             v[J][R], w[J][R];
#pragma unroll
  for (int jj = 0; jj < J; jj++) {
    const uint32_t j = threadIdx.x + jj * OFDM_THREADS;
    if (NS > 1 && j < nb) {
      const uint32_t k = j % NS;
#pragma unroll
      for (int r = 1; r < R; r++) {
        w[jj][r] = tw[r * k * tstep];
      }
    }
  }
#pragma unroll
  for (int jj = 0; jj < J; jj++) {
    const uint32_t j = threadIdx.x + jj * OFDM_THREADS;
    if (j < nb) {
#pragma unroll
      for (int r = 0; r < R; r++) {
        v[jj][r] = buf[j + r * nb];
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int jj = 0; jj < J; jj++) {
    const uint32_t j = threadIdx.x + jj * OFDM_THREADS;
    if (j < nb) {
      const uint32_t q = j / NS, k = j % NS;
      if constexpr (NS > 1) {
#pragma unroll
        for (int r = 1; r < R; r++) {
          v[jj][r] = cmul(v[jj][r], w[jj][r]);
        }
      }
      if constexpr (R == 8) {
        dft8(v[jj]);
      } else if constexpr (R == 4) {
        dft4(v[jj]);
      } else if constexpr (R == 3) {
        dft3(v[jj]);
      } else {
        dft2(v[jj]);
      }
      const uint32_t base = q * NS * R + k;
#pragma unroll
      for (int r = 0; r < R; r++) {
        buf[base + r * NS] = v[jj][r];
      }
    }
  }
  __syncthreads();
}

// NC = 2048 / 1536 (C3's standard and reference-default rates): ofdm_plan's stages 8, 8, 8, 4 / 8, 8, 8, 3 unrolled
// at compile time; NC = 0: the runtime plan
template <uint32_t NC>
__device__ __forceinline__ void fft_n(float2* buf, const OfdmArgs& a)
{
  if constexpr (NC == 2048) {
    stage_ct<8, 2048, 1>(buf, a.tw);
    stage_ct<8, 2048, 8>(buf, a.tw);
    stage_ct<8, 2048, 64>(buf, a.tw);
    stage_ct<4, 2048, 512>(buf, a.tw);
  } else if constexpr (NC == 1536) {
    stage_ct<8, 1536, 1>(buf, a.tw);
    stage_ct<8, 1536, 8>(buf, a.tw);
    stage_ct<8, 1536, 64>(buf, a.tw);
    stage_ct<3, 1536, 512>(buf, a.tw);
  } else {
    fft_ip(buf, a);
  }
}
// the launch's choice of fft_n: the compile-time plan where ofdm_plan gives exactly it
static uint32_t fixed_plan(const OfdmArgs& a)
{
  static const int k2048[4] = {8, 8, 8, 4}, k1536[4] = {8, 8, 8, 3};
  if (a.nstages != 4 || (a.N != 2048 && a.N != 1536)) {
    return 0;
  }
  const int* want = a.N == 2048 ? k2048 : k1536;
  for (int st = 0; st < 4; st++) {
    if (a.radix[st] != want[st]) {
      return 0;
    }
  }
  return a.N;
}

template <uint32_t NC>
__global__ __launch_bounds__(OFDM_THREADS) void ofdm_rx_kernel(OfdmArgs a)
{
  __shared__ float2 buf[OFDM_MAX_N];
  const uint32_t    sym = blockIdx.x, rx = blockIdx.y, sf = blockIdx.z;
  const uint32_t    N = NC ? NC : a.N, ns = a.nsymb, slot = sym / ns, i = sym % ns;
  const uint32_t    slot_sz = ns * N + a.cp0 + (ns - 1) * a.cp;
  const uint32_t    off = a.mbsfn && slot == 0 ? a.mbsfn_off[i] : slot * slot_sz + a.cp0 + i * (N + a.cp) - a.win;
  const size_t      s0      = ((size_t)sf * a.nrx + rx) * a.sf_len + off;
  const float2*     src     = a.in + s0;
  {  // all of a thread's sample loads (and CFO factors) issued before the first use: one HBM round trip
    constexpr int U = OFDM_MAX_N / OFDM_THREADS;
    float2        x[U], c[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t n = threadIdx.x + u * OFDM_THREADS;
      if (n < N) {
        if (a.in16) {
          const short2 q = a.in16[s0 + n];
          x[u]           = make_float2((float)q.x * a.in_scale, (float)q.y * a.in_scale);
        } else {
          x[u] = src[n];
        }
        if (a.cfo_tab) {
          c[u] = a.cfo_tab[off + n];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t n = threadIdx.x + u * OFDM_THREADS;
      if (n < N) {
        buf[n] = a.cfo_tab ? ref_cprod(x[u], c[u]) : x[u];  // srsran_cfo_correct on the subframe buffer
      }
    }
  }
  __syncthreads();
  fft_n<NC>(buf, a);
  float2*        dst  = a.out + (((size_t)sf * a.nrx + rx) * 2 * ns + sym) * a.nre;
  const uint32_t half = a.nre / 2;
  for (uint32_t k = threadIdx.x; k < a.nre; k += OFDM_THREADS) {
    const uint32_t bin = k < half ? N - half + k : k - half + 1 - a.dc0;
    float2         v   = buf[bin];
    if (a.norm != 1.0f) {
      v = make_float2(v.x * a.norm, v.y * a.norm);
    }
    dst[k] = v;
  }
}

// OFDM modulator (ofdm_tx_slot, ofdm.c:585-674, as srsran_enb_dl configures it: no normalisation,
// DC left empty, no frequency shift): the nre subcarriers go to bins 1.. nre/2 (upper half of the
// grid) and N - nre/2 .. N-1 (lower half), a backward DFT computed as conj(FFT(conj(X))) with the
// receiver's Stockham stages, then the cyclic prefix.  in: [sf][port][14][nre], out: [sf][port][sf_len];
// a.norm scales the grid first (srsran_enb_dl_gen_signal's 0.05 / sqrt(nof_prb)).
template <uint32_t NC>
__global__ __launch_bounds__(OFDM_THREADS) void ofdm_tx_kernel(OfdmArgs a)
{
  __shared__ float2 buf[OFDM_MAX_N];
  const uint32_t    sym = blockIdx.x, port = blockIdx.y, sf = blockIdx.z;
  const uint32_t    N = NC ? NC : a.N, ns = a.nsymb, slot = sym / ns, i = sym % ns, half = a.nre / 2;
  const float2*     src = a.in + (((size_t)sf * a.nrx + port) * 2 * ns + sym) * a.nre;
  for (uint32_t n = threadIdx.x; n < N; n += OFDM_THREADS) {
    buf[n] = make_float2(0.f, 0.f);
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < a.nre; k += OFDM_THREADS) {
    const uint32_t bin = k < half ? N - half + k : k - half + 1 - a.dc0;
    const float2   v   = src[k];
    buf[bin]           = make_float2(v.x * a.norm, -(v.y * a.norm));
  }
  __syncthreads();
  fft_n<NC>(buf, a);
  const uint32_t slot_sz = ns * N + a.cp0 + (ns - 1) * a.cp;
  const uint32_t off     = slot * slot_sz + a.cp0 + i * (N + a.cp);
  const uint32_t cpl     = i == 0 ? a.cp0 : a.cp;
  float2*        dst     = a.out + ((size_t)sf * a.nrx + port) * a.sf_len;
  for (uint32_t n = threadIdx.x; n < N; n += OFDM_THREADS) {
    const float2 v = buf[n];
    const float2 x = make_float2(v.x, -v.y);
    dst[off + n]   = x;
    if (n >= N - cpl) {
      dst[off - cpl + (n - (N - cpl))] = x;
    }
  }
}

// ---- N = 2048 / 1536 on one wave per symbol (ofdm_rx_wave_kernel) ----
// N = 64 x M (M = 32 / 24): lane l holds x[l + 64 m], m < M, and takes their M-point DFT in registers (4 x 8 /
// 3 x 8), twiddles it by W_N^(l k2), writes it to a wave-private LDS tile [k2][l], and reads back every second
// element of row k2 = lane / 2 from parity p = lane & 1: a 32-point DFT of those is half of row k2's 64-point DFT,
// the other half sits in the neighbour lane, and one radix-2 step across the pair (a DPP swap) gives
// X[k2 + M k1].  Two register FFTs and one LDS transpose a symbol instead of four LDS stages and eight workgroup
// barriers; the same forward DFT as the Stockham kernels, rounded in another order.  (M = 24: lanes 48..63 idle in
// the second half.)  The tile holds one float plane at a time -- real parts, then imaginary parts -- in rows of 64
// floats with the column index XOR-swizzled by 2 k2 (both the row writes and the column reads conflict-free), so a
// wave needs 8 KB of LDS: the 16 KB a CU keeps free beside the turbo decoder's two 72 KB workgroups (C3,
// K = 5824) take two, so the next batch's OFDM runs beside the decoder instead of waiting for it.
static constexpr int WV_ROW = 64;  // LDS row length of the transpose tile (floats)

// natural-order M-point DFT in place (M = 32: m = 8 m1 + m2, k = k1 + 4 k2; M = 24: k = k1 + 3 k2); the inner
// twiddles W_M^j = W_N^(TS j), TS = N / M, come from the symbol's table
template <int M, int TS>
__device__ __forceinline__ void dft_reg(float2 (&a)[M], const float2* __restrict__ tw)
{
  constexpr int R = M / 8;  // 4 or 3
  float2        b[M];
#pragma unroll
  for (int m2 = 0; m2 < 8; m2++) {
    float2 t[R];
#pragma unroll
    for (int m1 = 0; m1 < R; m1++) {
      t[m1] = a[8 * m1 + m2];
    }
    if constexpr (R == 4) {
      dft4(t);
    } else {
      dft3(t);
    }
#pragma unroll
    for (int k1 = 0; k1 < R; k1++) {
      b[k1 * 8 + m2] = (m2 * k1 == 0) ? t[k1] : cmul(t[k1], tw[TS * m2 * k1]);
    }
  }
#pragma unroll
  for (int k1 = 0; k1 < R; k1++) {
    float2 u[8];
#pragma unroll
    for (int m2 = 0; m2 < 8; m2++) {
      u[m2] = b[k1 * 8 + m2];
    }
    dft8(u);
#pragma unroll
    for (int k2 = 0; k2 < 8; k2++) {
      a[k1 + R * k2] = u[k2];
    }
  }
}

// the value of lane ^ 1 (quad_perm [1, 0, 3, 2])
__device__ __forceinline__ float swap1(float v)
{
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
}

template <uint32_t N, bool CFO>
__global__ __launch_bounds__(64) void ofdm_rx_wave_kernel(OfdmArgs a)
{
  constexpr int      M = (int)(N / 64);
  __shared__ float   T[M * WV_ROW];
  const uint32_t     sym = blockIdx.x, rx = blockIdx.y, sf = blockIdx.z, l = threadIdx.x;
  const uint32_t     ns = a.nsymb, slot = sym / ns, i = sym % ns;
  const uint32_t     slot_sz = ns * N + a.cp0 + (ns - 1) * a.cp;
  const uint32_t     off = a.mbsfn && slot == 0 ? a.mbsfn_off[i] : slot * slot_sz + a.cp0 + i * (N + a.cp) - a.win;
  const size_t       s0      = ((size_t)sf * a.nrx + rx) * a.sf_len + off;
  const float2*      src     = a.in + s0;
  const float2*      tw      = a.tw;
  float2             v[M];
  if (a.in16) {
    const short2* q16 = a.in16 + s0;
#pragma unroll
    for (int m = 0; m < M; m++) {
      const short2 q = q16[l + 64 * m];
      v[m]           = make_float2((float)q.x * a.in_scale, (float)q.y * a.in_scale);
    }
  } else {
#pragma unroll
    for (int m = 0; m < M; m++) {
      v[m] = src[l + 64 * m];
    }
  }
  if constexpr (CFO) {
    float2 c[M];
#pragma unroll
    for (int m = 0; m < M; m++) {
      c[m] = a.cfo_tab[off + l + 64 * m];
    }
#pragma unroll
    for (int m = 0; m < M; m++) {
      v[m] = ref_cprod(v[m], c[m]);  // srsran_cfo_correct on the subframe buffer
    }
  }
  dft_reg<M, 64>(v, tw);
  {
    float2 w[M];
#pragma unroll
    for (int k2 = 1; k2 < M; k2++) {
      w[k2] = tw[l * k2];  // l k2 <= 63 (M - 1) < N
    }
#pragma unroll
    for (int k2 = 1; k2 < M; k2++) {
      v[k2] = cmul(v[k2], w[k2]);
    }
  }
  const uint32_t kk = l >> 1, p = l & 1, row = kk < (uint32_t)M ? kk : 0;
  float2         y[32];
  // the real plane, then the imaginary one
#pragma unroll
  for (int k2 = 0; k2 < M; k2++) {
    T[k2 * WV_ROW + (l ^ (2 * k2))] = v[k2].x;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < 32; j++) {
    y[j].x = T[row * WV_ROW + ((2 * j + p) ^ (2 * row))];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront", "local");  // the real plane read out
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k2 = 0; k2 < M; k2++) {
    T[k2 * WV_ROW + (l ^ (2 * k2))] = v[k2].y;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < 32; j++) {
    y[j].y = T[row * WV_ROW + ((2 * j + p) ^ (2 * row))];
  }
  dft_reg<32, (int)(N / 32)>(y, tw);
  // X[kk + M k] = Y0[k] + W_64^k Y1[k], X[kk + M (k + 32)] = Y0[k] - W_64^k Y1[k]; W_64^k = W_N^(M k)
  const uint32_t half = a.nre / 2;
  float2*        dst  = a.out + (((size_t)sf * a.nrx + rx) * 2 * ns + sym) * a.nre;
#pragma unroll
  for (int k = 0; k < 32; k++) {
    const float2   t = (p && k) ? cmul(y[k], tw[M * k]) : y[k];  // lane 1: W_64^k Y1[k]; lane 0: Y0[k]
    const float2   o = make_float2(swap1(t.x), swap1(t.y));      // the pair's other value
    float2         x = p ? csub(o, t) : cadd(t, o);               // lane 0: Y0 + W Y1; lane 1: Y0 - W Y1
    const uint32_t b = kk + (uint32_t)M * ((uint32_t)k + 32 * p);
    if (a.norm != 1.0f) {
      x = make_float2(x.x * a.norm, x.y * a.norm);
    }
    if (kk >= (uint32_t)M) {
      continue;
    }
    if (b >= N - half) {
      dst[b - (N - half)] = x;
    } else if (b + a.dc0 >= 1 && b + a.dc0 <= half) {
      dst[b + half - 1 + a.dc0] = x;
    }
  }
}

hipError_t ofdm_tx_launch(const OfdmArgs& a, uint32_t nsf, hipStream_t stream)
{
  if (a.N > OFDM_MAX_N || a.nstages <= 0 || nsf == 0 || (a.nsymb != 7 && a.nsymb != 6)) {
    return hipErrorInvalidValue;
  }
  const dim3 grid(2 * a.nsymb, a.nrx, nsf);
  switch (fixed_plan(a)) {
    case 2048:
      hipLaunchKernelGGL(ofdm_tx_kernel<2048>, grid, dim3(OFDM_THREADS), 0, stream, a);
      break;
    case 1536:
      hipLaunchKernelGGL(ofdm_tx_kernel<1536>, grid, dim3(OFDM_THREADS), 0, stream, a);
      break;
    default:
      hipLaunchKernelGGL(ofdm_tx_kernel<0>, grid, dim3(OFDM_THREADS), 0, stream, a);
  }
  return hipGetLastError();
}

int ofdm_plan(uint32_t N, int* radix, uint32_t* ns_magic)
{
  const int n = ofdm_plan(N, radix);
  uint32_t  Ns = 1;
  for (int st = 0; st < n; st++) {
    ns_magic[st] = Ns > 1 ? (uint32_t)((((uint64_t)1 << 32) + Ns - 1) / Ns) : 0u;
    Ns *= (uint32_t)radix[st];
  }
  return n;
}

int ofdm_plan(uint32_t N, int* radix)
{
  int n = 0;
  while (N > 1 && n < OFDM_MAX_STAGES) {
    if (N % 8 == 0 && N != 16) {  // 16 = 4 x 4 keeps every stage at >= radix 4
      radix[n++] = 8;
      N /= 8;
    } else if (N % 4 == 0) {
      radix[n++] = 4;
      N /= 4;
    } else if (N % 3 == 0) {
      radix[n++] = 3;
      N /= 3;
    } else if (N % 2 == 0) {
      radix[n++] = 2;
      N /= 2;
    } else {
      return -1;
    }
  }
  return N == 1 ? n : -1;
}

hipError_t ofdm_rx_launch(const OfdmArgs& a, uint32_t nsf, hipStream_t stream)
{
  StageScope timing_scope(ST_OFDM, stream);
  if (a.N > OFDM_MAX_N || a.nstages <= 0 || nsf == 0 || (a.nsymb != 7 && a.nsymb != 6)) {
    return hipErrorInvalidValue;
  }
  // N = 2048 / 1536: the one-wave-per-symbol kernel (r05s: 29.1 against 34.1 us for the compile-time Stockham
  // plan under the 3-worker chain, 41 % fewer VALU, 69 % fewer wave cycles); SRSRAN_AMD_OFDM_WAVE=0 (read once)
  // keeps the workgroup-per-symbol Stockham kernel
  static const bool wave = [] {
    const char* v = getenv("SRSRAN_AMD_OFDM_WAVE");
    return !(v && v[0] == '0');
  }();
  const dim3     grid(2 * a.nsymb, a.nrx, nsf);
  const uint32_t plan = fixed_plan(a);
  if (wave && plan == 2048) {
    if (a.cfo_tab) {
      hipLaunchKernelGGL((ofdm_rx_wave_kernel<2048, true>), grid, dim3(64), 0, stream, a);
    } else {
      hipLaunchKernelGGL((ofdm_rx_wave_kernel<2048, false>), grid, dim3(64), 0, stream, a);
    }
  } else if (wave && plan == 1536) {
    if (a.cfo_tab) {
      hipLaunchKernelGGL((ofdm_rx_wave_kernel<1536, true>), grid, dim3(64), 0, stream, a);
    } else {
      hipLaunchKernelGGL((ofdm_rx_wave_kernel<1536, false>), grid, dim3(64), 0, stream, a);
    }
  } else if (plan == 2048) {
    hipLaunchKernelGGL(ofdm_rx_kernel<2048>, grid, dim3(OFDM_THREADS), 0, stream, a);
  } else if (plan == 1536) {
    hipLaunchKernelGGL(ofdm_rx_kernel<1536>, grid, dim3(OFDM_THREADS), 0, stream, a);
  } else {
    hipLaunchKernelGGL(ofdm_rx_kernel<0>, grid, dim3(OFDM_THREADS), 0, stream, a);
  }
  return hipGetLastError();
}

__global__ void ofdm_rx_post_kernel(float2* __restrict__ grid, uint32_t rows, OfdmArgs a, const float2* __restrict__ wo,
                                    const float2* __restrict__ ph)
{
  const uint32_t row = blockIdx.y, sym = row % (2 * a.nsymb);
  if (row >= rows || (a.mbsfn && sym < a.nsymb)) {
    return;
  }
  const uint32_t half = a.nre / 2;
  float2*        g    = grid + (size_t)row * a.nre;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < a.nre; k += gridDim.x * blockDim.x) {
    float2 x = g[k];
    if (wo) {
      x = cmul(x, wo[k < half ? a.N - half + k : k - half + 1 - a.dc0]);
    }
    if (ph) {
      x = cmul(x, ph[sym]);
    }
    g[k] = x;
  }
}

hipError_t ofdm_rx_post_launch(float2* grid, uint32_t rows, const OfdmArgs& a, const float2* wo, const float2* ph,
                               hipStream_t stream)
{
  if (rows == 0 || (!wo && !ph)) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(ofdm_rx_post_kernel, dim3((a.nre + 255) / 256, rows), dim3(256), 0, stream, grid, rows, a, wo, ph);
  return hipGetLastError();
}

__global__ void ofdm_tx_post_kernel(float2* __restrict__ out, uint32_t rows, OfdmArgs a, const float2* __restrict__ ph,
                                    const float2* __restrict__ shift)
{
  const uint32_t slot_sz = a.nsymb * a.N + a.cp0 + (a.nsymb - 1) * a.cp;
  float2*        o       = out + (size_t)blockIdx.y * a.sf_len;
  for (uint32_t n = blockIdx.x * blockDim.x + threadIdx.x; n < a.sf_len; n += gridDim.x * blockDim.x) {
    float2 x = o[n];
    if (ph) {
      const uint32_t slot = n / slot_sz, r = n - slot * slot_sz;
      const uint32_t i    = r < a.cp0 + a.N ? 0 : 1 + (r - a.cp0 - a.N) / (a.cp + a.N);
      x                   = cmul(x, ph[slot * a.nsymb + i]);
    }
    if (shift) {
      x = cmul(x, shift[n]);
    }
    o[n] = x;
  }
}

hipError_t ofdm_tx_post_launch(float2* out, uint32_t rows, const OfdmArgs& a, const float2* ph, const float2* shift,
                               hipStream_t stream)
{
  if (rows == 0 || (!ph && !shift)) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(ofdm_tx_post_kernel, dim3((a.sf_len + 255) / 256, rows), dim3(256), 0, stream, out, rows, a, ph,
                     shift);
  return hipGetLastError();
}

// One wave: lanes 0..7 carry the reference's 8 SIMD phases through the len / 8 blocks (a serial
// recurrence: every block's phase is the previous one times w^8, rounded -- it cannot be re-associated
// without changing the result), lane 0 then the scalar tail.  Run once per (f, len) and cached by the host.
__global__ __launch_bounds__(64) void cfo_table_kernel(float c, float s, float2* __restrict__ tab, uint32_t len)
{
  const uint32_t k = threadIdx.x;
  if (k >= 8) {
    return;
  }
  const float2 w = make_float2(c, s);
  float2       p = make_float2(1.0f, 0.0f);  // _phase[k] = _phase[k - 1] * osc, _phase[0] = 1
  for (uint32_t j = 0; j < k; j++) {
    p = ref_cprod(p, w);
  }
  float2 w8 = make_float2(1.0f, 0.0f);  // _phase[7] * osc, computed as the same chain
  for (uint32_t j = 0; j < 8; j++) {
    w8 = ref_cprod(w8, w);
  }
  const uint32_t nblk = len / 8;  // for (; i < len - 8 + 1; i += 8)
  for (uint32_t m = 0; m < nblk; m++) {
    tab[8 * m + k] = p;
    p              = ref_cprod(p, w8);
  }
  if (k == 0) {  // phase = _phase[0] after the SIMD loop; the scalar tail advances by osc
    for (uint32_t i = 8 * nblk; i < len; i++) {
      tab[i] = p;
      p      = ref_cprod(p, w);
    }
  }
}

void cfo_phasor(float f, float* c, float* s)
{
  const float twopi = 2.0f * (float)M_PI;  // TWOPI of vector_simd.c:1725
  sincosf(twopi * f, s, c);                // cexpf(_Complex_I * TWOPI * cfo): the real part is 0
}

hipError_t cfo_table_launch(float c, float s, float2* tab, uint32_t len, hipStream_t stream)
{
  if (len == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(cfo_table_kernel, dim3(1), dim3(64), 0, stream, c, s, tab, len);
  return hipGetLastError();
}

__global__ void cfo_kernel(const float2* __restrict__ in, float2* __restrict__ out, const float2* __restrict__ tab,
                           uint32_t n)
{
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) {
    out[k] = ref_cprod(in[k], tab[k]);
  }
}

hipError_t cfo_launch(const float2* in, float2* out, const float2* tab, uint32_t n, hipStream_t stream)
{
  StageScope timing_scope(ST_OFDM, stream);
  if (n == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(cfo_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, in, out, tab, n);
  return hipGetLastError();
}

}  // namespace srsran_amd
