// srsran_4g_amd/csrc/chest_kernel.hip -- DL CRS channel estimation for CDNA4.
//
// srsUE's default estimator (AVERAGE, Gauss smoothing order 4 / sigma 1, REFS noise):
//   LS at the CRS            estimate_port         chest_dl.c:806-834
//   noise (REFS)             estimate_noise_pilots chest_dl.c:325-400
//   time average + smoothing average_pilots        chest_dl.c:557-600, convolution.c:182-218
//   linear interpolation     srsran_interp_linear_offset interp.c:258-285 (then every symbol)
//   CFO from pilot phases    chest_estimate_cfo    chest_dl.c:621-641
// One workgroup per (port, rx antenna): the 4 x 200 pilots, the noise residuals and the
// 400-point smoothed comb live in LDS; the estimate row (1200 subcarriers at 100 PRB) is
// written once, or 2 nsymb times (14 normal CP, 12 extended) for the full srsran_chest_dl_res_t grid.
// Float operations follow the reference's order (no contraction) so the result matches
// oracle/phy_oracle.c up to the order of the power/phase reductions.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "chest_kernel.h"
#include "stage_timing.h"

#pragma clang fp contract(off)

namespace srsran_amd {

#ifndef CH_THREADS_CFG
#define CH_THREADS_CFG 256
#endif
static constexpr int CH_THREADS = CH_THREADS_CFG;  // a workgroup per (port, rx, subframe)

struct cx {
  float r, i;
};
__device__ __forceinline__ cx ld2(const float2* p, uint32_t k)
{
  const float2 v = p[k];
  return {v.x, v.y};
}
__device__ __forceinline__ cx add(cx a, cx b) { return {a.r + b.r, a.i + b.i}; }
__device__ __forceinline__ cx sub(cx a, cx b) { return {a.r - b.r, a.i - b.i}; }
__device__ __forceinline__ cx mul(cx a, cx b) { return {a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r}; }
__device__ __forceinline__ cx conj(cx a) { return {a.r, -a.i}; }
__device__ __forceinline__ cx scl(cx a, float s) { return {a.r * s, a.i * s}; }
__device__ __forceinline__ cx divs(cx a, float s) { return {a.r / s, a.i / s}; }

__device__ __forceinline__ uint32_t crs_v(uint32_t port, uint32_t l)
{
  return port == 0 ? ((l & 1) ? 3u : 0u) : port == 1 ? ((l & 1) ? 0u : 3u) : port == 2 ? (l == 0 ? 0u : 3u) : (l == 0 ? 3u : 0u);
}
// srsran_refsignal_cs_nsymbol (refsignal_dl.c:254-266), ns = symbols per slot
__device__ __forceinline__ uint32_t crs_nsymbol(uint32_t l, uint32_t port, uint32_t ns)
{
  return port < 2 ? ((l & 1) ? (l / 2 + 1) * ns - 3 : (l / 2) * ns) : 1 + l * ns;
}

// block-wide sum of one float (all threads get the result)
__device__ float block_sum(float v, float* red)
{
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    v += __shfl_xor(v, off, 64);
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = v;
  }
  __syncthreads();
  float s = 0.f;
  for (int w = 0; w < CH_THREADS / 64; w++) {
    s += red[w];
  }
  return s;
}

// block-wide sums of two floats under one pair of barriers (red: 2 CH_THREADS / 64 floats); each sum in
// block_sum's order
__device__ void block_sum2(float& a, float& b, float* red)
{
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off, 64);
    b += __shfl_xor(b, off, 64);
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6]                     = a;
    red[CH_THREADS / 64 + (threadIdx.x >> 6)] = b;
  }
  __syncthreads();
  float sa = 0.f, sb = 0.f;
  for (int w = 0; w < CH_THREADS / 64; w++) {
    sa += red[w];
    sb += red[CH_THREADS / 64 + w];
  }
  a = sa;
  b = sb;
}

// srsran_conv_same_cf (convolution.c:182-218): out[i] = sum_k f[k] x[i - M/2 + k] over the sequence extended
// linearly at both ends (first[] / last[])
__device__ void conv_row(const cx* comb, cx* avg, uint32_t nr, const float* filt, uint32_t M)
{
  for (uint32_t i = threadIdx.x; i < nr; i += CH_THREADS) {
    cx acc = {0.f, 0.f};
    for (uint32_t k = 0; k < M; k++) {
      const int j = (int)i - (int)(M / 2) + (int)k;  // index into the extended sequence
      cx        x;
      if (j < 0) {  // first[]: (2 + M/2 - m) * in[1] - (1 + M/2 - m) * in[0], m = j + M/2
        const uint32_t m = (uint32_t)(j + (int)(M / 2));
        x = sub(scl(comb[1], (float)(2 + M / 2 - m)), scl(comb[0], (float)(1 + M / 2 - m)));
      } else if (j >= (int)nr) {  // last[]: m = j - (nr - M + 1) counts into last[], i >= M - 1
        const uint32_t m = (uint32_t)(j - (int)(nr - M + 1));
        x = sub(scl(comb[nr - 1], (float)(2 + m - M / 2)), scl(comb[nr - 2], (float)(1 + m - M / 2)));
      } else {
        x = comb[j];
      }
      acc = add(acc, scl(x, filt[k]));
    }
    avg[i] = acc;
  }
}

// srsran_interp_linear_offset (interp.c:258-285) of the nr-point comb `av` (spacing `step`, first pilot at
// subcarrier `off`), value at subcarrier j
__device__ __forceinline__ cx interp_at(const cx* av, uint32_t nr, uint32_t step, uint32_t off, uint32_t j)
{
  const float rM = (float)1 / step;
  if (j < off) {
    const uint32_t jj = off - 1 - j;
    return sub(av[0], divs(scl(sub(av[1], av[0]), (float)(jj + 1)), (float)step));
  }
  if (j < off + step * (nr - 1)) {
    const uint32_t i = (j - off) / step, r = (j - off) % step;
    return add(av[i], scl(scl(sub(av[i + 1], av[i]), rM), (float)r));
  }
  const uint32_t r = j - off - step * (nr - 1);
  return add(av[nr - 1], divs(scl(sub(av[nr - 1], av[nr - 2]), (float)r), (float)step));
}

// srsran_interp_linear_vector3 (interp.c:158-188) for one subcarrier: rows[first .. first + M) from in0 / in1
// rows are written straight into the estimate column col (row stride `stride`): a per-lane rows[] array would
// live in scratch
__device__ __forceinline__ void ivec(float2* col, uint32_t stride, cx in0, cx in1, const cx* start, uint32_t d,
                                     uint32_t M, uint32_t first)
{
  const cx diff = scl(sub(in1, in0), (float)1 / d);
  cx       b    = add(start ? *start : in0, diff);
  col[(size_t)first * stride] = make_float2(b.r, b.i);
  for (uint32_t i = 1; i < M; i++) {
    b                                 = add(b, diff);
    col[(size_t)(first + i) * stride] = make_float2(b.r, b.i);
  }
}

// estimate_noise_pilots (chest_dl.c:356-399) for nsym >= 3 rows of nref LS estimates at pe (first pilot of row 0 at
// subcarrier fidx0): each inner row against its neighbours, the residual power averaged over the inner rows
__device__ float noise_rows(const cx* pe, uint32_t nsym, uint32_t nref, uint32_t fidx0, float* red)
{
  float noise = 0.f;
  for (uint32_t i = 1; i < nsym - 1; i++) {
    const uint32_t off = ((fidx0 < 3) ^ (i & 1)) ? 0 : 1;
    const cx*      cur = pe + i * nref;
    float          p   = 0.f;
    for (uint32_t k = threadIdx.x; k < nref; k += CH_THREADS) {
      cx t = cur[k];
#pragma unroll
      for (int nb = 0; nb < 2; nb++) {
        const cx* o = pe + (nb == 0 ? i - 1 : i + 1) * nref;
        if (k >= off) {
          t = add(o[k - off], t);
        }
        if (k < nref + off - 1) {
          t = add(o[1 - off + k], t);
        }
        if (off && k == 0) {
          t = add(t, sub(scl(o[0], 2.0f), o[1]));
        }
        if (!off && k == nref - 1) {
          t = add(t, sub(scl(o[nref - 2], 2.0f), o[nref - 1]));
        }
      }
      t = sub(cur[k], scl(t, 1.0f / 5.0f));
      p += t.r * t.r + t.i * t.i;
    }
    noise += block_sum(p, red) / (float)nref;
  }
  return noise / (float)(nsym - 2);
}

// the smoothing filter into LDS filt[] (all threads see it after the barrier inside): srsran_chest_set_smooth_filter_
// gauss(filter, 4, noise * 200) when automatic (chest_common.c:70-95), else the host's taps; returns the length
__device__ uint32_t load_filter(const ChestArgs& a, float noise, float* filt)
{
  uint32_t M = a.filter_len;
  if (a.filter_auto) {
    const float sd  = noise * 200.0f;
    float       sum = 0.f;
#pragma unroll
    for (int k = 0; k < 5; k++) {
      sum += expf(-powf((float)(k - 2), 2) / (2.0f * powf(sd, 2)));
    }
    M = isnormal(sum) ? 5 : 0;  // srsran_conv_same_cf with an empty filter yields zeros
    if (threadIdx.x < 5) {
      filt[threadIdx.x] = expf(-powf((float)((int)threadIdx.x - 2), 2) / (2.0f * powf(sd, 2))) * (1.0f / sum);
    }
  } else if (threadIdx.x == 0) {  // constant indices: a dynamic index into the by-value kernarg copies it to scratch
#pragma unroll
    for (int k = 0; k < 8; k++) {
      filt[k] = a.filter[k];
    }
  }
  __syncthreads();
  return M;
}

// fill_res (chest_dl.c:962-986) of one subframe from its per-(rx, port) stats st -> o[4]: every stat of the
// subframe loaded first (one round trip, not one a loop step), then the reference's sums in its order
__device__ bool finalize_sf(const float* st, uint32_t np, uint32_t nrx, uint32_t nof_prb, float sz, float nsymb,
                            float* o)
{
  float v[4][4][5];  // [rx][port][noise, rsrp, rssi, cfo re, cfo im]
  bool  has_cfo = false;  // the (rx, port) the CFO comes from had 4 CRS symbols (not a TDD special subframe)
#pragma unroll
  for (uint32_t rx = 0; rx < 4; rx++) {
#pragma unroll
    for (uint32_t p = 0; p < 4; p++) {
      if (rx < nrx && p < np) {
#pragma unroll
        for (int f = 0; f < 5; f++) {
          v[rx][p][f] = st[(rx * np + p) * 8 + f];
        }
      }
    }
  }
  float n = 0, best = -1e9f, rssi = 0, cfo = 0;
#pragma unroll
  for (uint32_t rx = 0; rx < 4; rx++) {
    if (rx < nrx) {
      float s = 0;
#pragma unroll
      for (uint32_t p = 0; p < 4; p++) {
        if (p < np) {
          s += v[rx][p][0];
        }
      }
      n += s / (float)np;
      rssi += 4 * v[rx][0][2] / (float)nof_prb / 12.0f;
    }
  }
#pragma unroll
  for (uint32_t p = 0; p < 4; p++) {
    if (p < np) {
      float s = 0;
#pragma unroll
      for (uint32_t rx = 0; rx < 4; rx++) {
        if (rx < nrx) {
          s += v[rx][p][1];
        }
      }
      s /= (float)nrx;
      best = s > best ? s : best;
    }
  }
  // chest_estimate_cfo (chest_dl.c:618-641): the last (rx, port < 2) wins -- rx = nrx - 1, port = min(np, 2) - 1;
  // ns = SRSRAN_CP_NSYMB, ng = SRSRAN_CP_LEN_NORM(1, n) for both CPs
  float cre = 0, cim = 0;
#pragma unroll
  for (uint32_t rx = 0; rx < 4; rx++) {
#pragma unroll
    for (uint32_t p = 0; p < 2; p++) {
      if (rx == nrx - 1 && p == min(np, 2u) - 1) {
        cre     = v[rx][p][3];
        cim     = v[rx][p][4];
        has_cfo = st[(rx * np + p) * 8 + 6] != 0.0f;
      }
    }
  }
  if (nrx * np > 0) {
    const float ng = (float)(int)ceilf(144.0f * sz / 2048.0f);
    cfo            = -atan2f(cim, cre) * sz / (nsymb * (sz + ng)) / 2 / 3.14159265358979f;
  }
  o[0]     = n / (float)nrx;
  o[1]     = best;
  o[2]     = rssi / (float)nrx;
  o[3]     = cfo;
  return has_cfo && nrx * np > 0;
}


// Diagnostic build only (-DCHEST_STAMPS, tools/chest_stamps.py): thread 0 of every workgroup writes the
// device clock (wall_clock64, 100 MHz) at the phase boundaries below into g_chest_stamps[workgroup][16]
#ifdef CHEST_STAMPS
__device__ unsigned long long* g_chest_stamps = nullptr;
#define CH_STAMP(k)                                                                                         \
  do {                                                                                                      \
    if (threadIdx.x == 0 && g_chest_stamps) {                                                               \
      g_chest_stamps[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 + (k)] = wall_clock64();            \
    }                                                                                                       \
  } while (0)
#else
#define CH_STAMP(k) \
  do {              \
  } while (0)
#endif

__global__ __launch_bounds__(CH_THREADS) void chest_kernel(ChestArgs a)
{
  CH_STAMP(0);
  // pe [4 nref] in dynamic LDS sized by chest_launch; AVERAGE builds its comb in place over pe's first rows and
  // smooths it into the last two, so a workgroup needs 6.4 KB at 100 PRB (INTERPOLATE with a filter: avg [4 nref]
  // after pe, 12.8 KB) -- two fit in the 16 KB a CU keeps free beside the turbo decoder's two workgroups (C3), so
  // the next batch's estimate runs beside the decoder
  extern __shared__ __attribute__((aligned(16))) cx chest_lds[];
  __shared__ float red[2 * CH_THREADS / 64];

  const uint32_t port = blockIdx.x / a.nrx, rx = blockIdx.x % a.nrx, b = blockIdx.y;
  const uint32_t tid  = threadIdx.x;
  const bool     bat  = a.sf_inl || a.sf_idx;  // per-subframe indices: pilots of each subframe's index
  const uint32_t sfi  = a.sf_inl ? (uint32_t)a.sf_inline[b] : a.sf_idx ? a.sf_idx[b] : a.sf_index;
  // CRS symbols of the port: 4 / 2, fewer in the DwPTS of a TDD special subframe
  const uint32_t nsym = chest_crs_nsym(a, sfi, port), nref = 2 * a.nof_prb, np = nsym * nref, nre = 12 * a.nof_prb;
  cx* const      pe   = chest_lds;
  cx* const      comb = pe;  // AVERAGE: over pe's first 2 nref entries, written after the averages are taken
  cx* const      avg  = a.filter_none ? pe : a.estimator == 1 ? pe + 4 * nref : pe + 2 * nref;
  static_assert(2 * CHEST_MAX_PRB <= CH_THREADS, "one comb position a thread");
  const float2*  in   = a.grid + b * a.grid_sf_stride + (size_t)rx * 2 * a.nsymb * nre;
  const float2*  pil  = a.pilots + (bat ? sfi * CHEST_PILOTS_PER_SF : 0) + (size_t)(port / 2) * 4 * CHEST_MAX_NREF;
  const uint32_t fidx0 = (crs_v(port, 0) + a.cell_id % 6) % 6;
  const bool     kept_noise = a.noise_alg != 0;  // PSS / EMPTY: the REFS residuals are not the estimate

  // ---- LS estimates at the CRS and RSRP / RSSI ----
  float rsrp = 0.f;
  {  // all of a thread's pilot loads first (np <= 4 CH_THREADS), then the products: one HBM round trip
    constexpr int PU = (4 * CHEST_MAX_NREF + CH_THREADS - 1) / CH_THREADS;
    cx            r[PU], p[PU];
#pragma unroll
    for (int u = 0; u < PU; u++) {
      const uint32_t k = tid + u * CH_THREADS;
      if (k < np) {
        const uint32_t l = k / nref, i = k % nref;
        const uint32_t f = (crs_v(port, l) + a.cell_id % 6) % 6 + 6 * i;
        r[u]             = ld2(in, crs_nsymbol(l, port, a.nsymb) * nre + f);
        p[u]             = ld2(pil, k);
      }
    }
#pragma unroll
    for (int u = 0; u < PU; u++) {
      const uint32_t k = tid + u * CH_THREADS;
      if (k < np) {
        pe[k] = mul(r[u], conj(p[u]));
        rsrp += r[u].r * r[u].r + r[u].i * r[u].i;
      }
    }
  }
  float rssi = 0.f;
  {  // every RSSI sample of the thread loaded at once (<= 21 at 110 PRB), then summed in k order
    constexpr int RU = (4 * 12 * CHEST_MAX_PRB + CH_THREADS - 1) / CH_THREADS;
    const uint32_t nk = nsym * nre;
    cx             r[RU];
    uint32_t       row = tid / nre, col = tid % nre;  // k = row nre + col, stepped without divisions
#pragma unroll
    for (int u = 0; u < RU; u++) {
      if (tid + u * CH_THREADS < nk) {
        r[u] = ld2(in, crs_nsymbol(row, port, a.nsymb) * nre + col);
      }
      col += CH_THREADS;
      while (col >= nre) {
        col -= nre;
        row++;
      }
    }
#pragma unroll
    for (int u = 0; u < RU; u++) {
      if (tid + u * CH_THREADS < nk) {
        rssi += r[u].r * r[u].r + r[u].i * r[u].i;
      }
    }
  }
  CH_STAMP(1);
  block_sum2(rsrp, rssi, red);  // pe[] complete after its barriers
  rsrp = rsrp / (float)np;
  rssi = rssi / (float)nsym;
  CH_STAMP(2);
  // the fused staging copies' PCIe reads go out here, after the grid loads have been consumed: issued first, they
  // held up every vmcnt wait behind them (loads retire in order); the LDS phases below cover their latency
  const uint32_t bid = blockIdx.y * gridDim.x + blockIdx.x, nblk = gridDim.x * gridDim.y;
  CopyRegs       cr;
  copy_jobs_issue(a.jobs, cr, bid);

  // ---- CFO phase sum (port-0 geometry, chest_dl.c:630-636) ----
  float cre = 0.f, cim = 0.f;
  if (nsym == 4) {
    for (uint32_t k = tid; k < np / 2; k += CH_THREADS) {
      const uint32_t ii = k / (np / 4), kk = k % (np / 4);
      const cx       t  = mul(pe[ii * np / 4 + kk], conj(pe[(ii + 2) * np / 4 + kk]));
      cre += t.r;
      cim += t.i;
    }
    block_sum2(cre, cim, red);
  }

  CH_STAMP(3);
  // ---- noise from the pilot residuals (REFS) ----
  float noise = 0.f;
  if (kept_noise) {
    noise = a.noise_in[rx * 4 + port];
  } else if (nsym >= 3) {
    noise = noise_rows(pe, nsym, nref, fidx0, red);
  } else {
    float p = 0.f;
    for (uint32_t k = tid; k + 2 < nref; k += CH_THREADS) {
      cx t = add(add(pe[k], pe[k + 1]), pe[k + 2]);
      t    = sub(pe[k + 1], scl(t, 1.0f / 3.0f));
      p += t.r * t.r + t.i * t.i;
    }
    noise = block_sum(p, red) / (float)(nref - 2);
  }

  CH_STAMP(4);
  // ---- time average into a 3-subcarrier comb (AVERAGE), then smoothing (average_pilots) ----
  uint32_t nr = nref;
  if (a.estimator == 1) {
    // INTERPOLATE: every CRS symbol smoothed on its own (below)
  } else if (a.filter_none) {
    // no average_pilots: AVERAGE interpolates the raw LS estimates -- with more than one CRS symbol the first 4 N_RB
    // of them as one comb of spacing 3 (interp_lin_3 over pilot_estimates, chest_dl.c:476-481, 724-725): pe itself
    nr = nsym > 1 ? 2 * nref : nref;
  } else if (nsym > 1) {
    // the averages in registers first: the comb then overwrites the pe rows they came from
    const uint32_t k  = tid;
    cx             e0 = {0.f, 0.f}, e1 = {0.f, 0.f};
    if (k < nref) {
      e0 = pe[(fidx0 < 3 ? 0 : 1) * nref + k];
      e1 = pe[(fidx0 < 3 ? 1 : 0) * nref + k];
      for (uint32_t l = 2; l + 1 < nsym; l += 2) {
        e0 = add(e0, pe[(fidx0 < 3 ? l : l + 1) * nref + k]);
        e1 = add(e1, pe[(fidx0 < 3 ? l + 1 : l) * nref + k]);
      }
    }
    __syncthreads();
    if (k < nref) {
      comb[2 * k]     = scl(e0, 2.0f / (float)nsym);
      comb[2 * k + 1] = scl(e1, 2.0f / (float)nsym);
    }
    nr = 2 * nref;
  }  // (one CRS symbol: the comb is pe's first row as it is)
  __syncthreads();
  // the smoothing filter lives in LDS: a private array indexed by the tap loop would spill to scratch
  __shared__ float filt[8];
  const uint32_t   M = load_filter(a, noise, filt);
  if (a.filter_none) {
    // the estimates as they are (a 1-tap unit filter would give the same values): avg is pe
  } else if (a.estimator == 1) {
    for (uint32_t l = 0; l < nsym; l++) {
      conv_row(pe + l * nref, avg + l * nref, nref, filt, M);
    }
  } else {
    conv_row(comb, avg, nr, filt, M);
  }
  __syncthreads();
  CH_STAMP(5);

  // ---- interpolation to every subcarrier (interp_linear_offset) and, for INTERPOLATE, between the CRS
  // symbols (interpolate_pilots, chest_dl.c:510-554); PSS noise on row nsymb - 1 (estimate_noise_pss) ----
  const uint32_t step = nsym > 1 ? 3 : 6;  // AVERAGE
  const uint32_t off  = nsym > 1 ? a.cell_id % 3 : fidx0;
  const uint32_t ns   = a.nsymb, nrows = 2 * ns;
  const bool     noise_sf = kept_noise && (sfi == 0 || sfi == 5);
  const uint32_t kp   = nre / 2 - 31;  // PSS / SSS subcarriers kp .. kp + 61 of rows ns - 1 / ns - 2
  float2*        ce   = a.ce + b * a.ce_sf_stride + (size_t)(port * a.nrx + rx) * a.ce_stride;
  float          pss_err = 0.f;
  for (uint32_t j = tid; j < nre; j += CH_THREADS) {
    if (a.estimator == 1 && nsym == 1) {  // one CRS symbol (special subframe): its row everywhere (chest_dl.c:511-515)
      const cx     v = interp_at(avg, nref, 6, fidx0, j);
      const float2 o = make_float2(v.r, v.i);
      for (uint32_t l = 0; l < nrows; l++) {
        ce[(size_t)l * nre + j] = o;
      }
      if (noise_sf && a.noise_alg == 1 && j >= kp && j < kp + 62) {
        const cx t = sub(mul(v, ld2(a.pss, j - kp)), ld2(in, (ns - 1) * nre + j));
        pss_err += t.r * t.r + t.i * t.i;
      }
    } else if (a.estimator == 1) {
      float2* col = ce + j;
      const auto vi = [&](uint32_t l) {
        return interp_at(avg + l * nref, nref, 6, (crs_v(port, l) + a.cell_id % 6) % 6, j);
      };
      const cx v0 = vi(0), v1 = vi(1);
      const auto put = [&](uint32_t l, cx x) { col[(size_t)l * nre] = make_float2(x.r, x.i); };
      if (port < 2 && nsym == 3) {  // special subframe, normal CP: CRS rows 0, 4, 7; rows 8 .. 13 extrapolated
        const cx       v2 = vi(2);
        const uint32_t r1 = ns - 3, r2 = ns;
        put(0, v0), put(r1, v1), put(r2, v2);
        ivec(col, nre, v0, v1, nullptr, r1, r1 - 1, 1);
        ivec(col, nre, v1, v2, nullptr, r2 - r1, r2 - r1 - 1, r1 + 1);
        ivec(col, nre, v1, v2, &v2, r2 - r1, nrows - 1 - r2, r2 + 1);
      } else if (port < 2) {  // CRS rows 0, ns - 3, ns, 2 ns - 3
        const cx       v2 = vi(2), v3 = vi(3);
        const uint32_t r1 = ns - 3, r2 = ns, r3 = 2 * ns - 3;
        put(0, v0), put(r1, v1), put(r2, v2), put(r3, v3);
        ivec(col, nre, v0, v1, nullptr, r1, r1 - 1, 1);
        ivec(col, nre, v1, v2, nullptr, r2 - r1, r2 - r1 - 1, r1 + 1);
        ivec(col, nre, v2, v3, nullptr, r3 - r2, r3 - r2 - 1, r2 + 1);
        ivec(col, nre, v2, v3, &v3, r3 - r2, nrows - 1 - r3, r3 + 1);
      } else {  // CRS rows 1, ns + 1 (the reference fills rows ns + 2 .. from row 1 as well)
        put(1, v0), put(ns + 1, v1);
        ivec(col, nre, v1, v0, &v0, ns, 1, 0);
        ivec(col, nre, v0, v1, nullptr, ns, ns - 1, 2);
        ivec(col, nre, v0, v1, nullptr, ns, ns - 2, ns + 2);
      }
      if (noise_sf && a.noise_alg == 1 && j >= kp && j < kp + 62) {  // row ns - 1 as this lane just wrote it
        const float2 w = col[(size_t)(ns - 1) * nre];
        const cx t = sub(mul(cx{w.x, w.y}, ld2(a.pss, j - kp)), ld2(in, (ns - 1) * nre + j));
        pss_err += t.r * t.r + t.i * t.i;
      }
    } else {
      const cx     v = interp_at(avg, nr, step, off, j);
      const float2 o = make_float2(v.r, v.i);
      if (a.full_grid) {
        for (uint32_t l = 0; l < nrows; l++) {
          ce[l * nre + j] = o;
        }
      } else {
        ce[j] = o;
      }
      if (noise_sf && a.noise_alg == 1 && j >= kp && j < kp + 62) {
        const cx t = sub(mul(v, ld2(a.pss, j - kp)), ld2(in, (ns - 1) * nre + j));
        pss_err += t.r * t.r + t.i * t.i;
      }
    }
  }
  if (noise_sf) {
    if (a.noise_alg == 1) {  // nof_ports * srsran_vec_avg_power_cf(62) * M_SQRT1_2
      noise = (float)a.nports * (block_sum(pss_err, red) / 62.0f) * (float)0.70710678118654752440;
    } else {  // estimate_noise_empty_sc: 5 empty subcarriers either side of the SSS and of the PSS
      noise = 0.f;
#pragma unroll
      for (int g = 0; g < 4; g++) {  // SSS left/right, then PSS left/right
        const uint32_t base = (ns - 2 + (g >> 1)) * nre + ((g & 1) ? kp + 62 : kp - 5);
        float          p    = 0.f;
        for (int k = 0; k < 5; k++) {
          const cx x = ld2(in, base + k);
          p += x.r * x.r + x.i * x.i;
        }
        noise += p / 5.0f;
      }
    }
  }
  if (tid == 0) {
    float* s = a.stats + b * CHEST_STATS_PER_SF + (size_t)(rx * a.nports + port) * 8;
    s[0]     = noise;
    s[1]     = rsrp;
    s[2]     = rssi;
    s[3]     = cre;
    s[4]     = cim;
    s[5]     = noise_sf ? 1.0f : 0.0f;
    s[6]     = nsym == 4 ? 1.0f : 0.0f;  // CFO phase sums present (4 CRS symbols)
  }
  CH_STAMP(6);
  copy_jobs_finish(a.jobs, cr, bid, nblk);
  CH_STAMP(7);
}

// MBSFN subframe (estimate_port_mbsfn, chest_dl.c:836-865), one workgroup per (port, rx), ports 0 / 1 only:
//   LS           the CRS of symbol 0 (2 N_RB, the subframe's CRS of the port pair) and the MBSFN reference signals
//                of symbols 2 / 6 / 10 of the extended-CP grid (6 N_RB each, every 2nd subcarrier from 0 / 1 / 0:
//                srsran_refsignal_mbsfn_get_sf, refsignal_dl.c:474-502) in one array of 20 N_RB
//   noise (REFS) estimate_noise_pilots with npilots = 20 N_RB over 3 "symbols" (chest_dl.c:325-399): the array cut
//                into rows of floor(20 N_RB / 3), the middle one against the other two, fidx 1
//   smoothing    average_pilots (557-600): the CRS row copied, each MBSFN row filtered on its own
//   interpolation interpolate_pilots (444-521): the CRS row into ce row 0 (spacing 6), the MBSFN rows into rows
//                2 / 6 / 10 (spacing 2), then rows 1, 3-5, 7-9 between them and row 11 extrapolated
__global__ __launch_bounds__(CH_THREADS) void chest_mbsfn_kernel(ChestArgs a)
{
  __shared__ cx    pe[20 * CHEST_MAX_PRB];
  __shared__ cx    avg[20 * CHEST_MAX_PRB];
  __shared__ float red[2 * CH_THREADS / 64];
  __shared__ float filt[8];
  const uint32_t   port = blockIdx.x / a.nrx, rx = blockIdx.x % a.nrx, tid = threadIdx.x;
  const uint32_t   nref = 2 * a.nof_prb, nm = 6 * a.nof_prb, np = 20 * a.nof_prb, nre = 12 * a.nof_prb;
  const float2*    in    = a.grid + (size_t)rx * 2 * a.nsymb * nre;
  const float2*    pil   = a.pilots + (size_t)(port / 2) * 4 * CHEST_MAX_NREF;  // symbol 0's CRS first
  const uint32_t   fidx0 = (crs_v(port, 0) + a.cell_id % 6) % 6;
  for (uint32_t k = tid; k < np; k += CH_THREADS) {
    cx r, p;
    if (k < nref) {
      r = ld2(in, crs_nsymbol(0, port, a.nsymb) * nre + fidx0 + 6 * k);
      p = ld2(pil, k);
    } else {
      const uint32_t m = k - nref, l = m / nm, i = m % nm;
      r                = ld2(in, (2 + 4 * l) * nre + (l == 1 ? 1u : 0u) + 2 * i);
      p                = ld2(a.mbsfn_pilots, m);
    }
    pe[k] = mul(r, conj(p));
  }
  __syncthreads();
  const float    noise = a.noise_alg == 0 ? noise_rows(pe, 3, np / 3, 1, red) : a.noise_in[rx * 4 + port];
  const uint32_t M     = load_filter(a, noise, filt);
  for (uint32_t k = tid; k < np; k += CH_THREADS) {
    if (k < nref || a.filter_none) {
      avg[k] = pe[k];
    }
  }
  if (!a.filter_none) {
    for (uint32_t l = 0; l < 3; l++) {
      conv_row(pe + nref + l * nm, avg + nref + l * nm, nm, filt, M);
    }
  }
  __syncthreads();
  float2* ce = a.ce + (size_t)(port * a.nrx + rx) * a.ce_stride;
  for (uint32_t j = tid; j < nre; j += CH_THREADS) {
    float2*  col = ce + j;
    const cx c0  = interp_at(avg, nref, 6, fidx0, j);
    const cx m0  = interp_at(avg + nref, nm, 2, 0, j);
    const cx m1  = interp_at(avg + nref + nm, nm, 2, 1, j);
    const cx m2  = interp_at(avg + nref + 2 * nm, nm, 2, 0, j);
    col[0]                = make_float2(c0.r, c0.i);
    col[(size_t)2 * nre]  = make_float2(m0.r, m0.i);
    col[(size_t)6 * nre]  = make_float2(m1.r, m1.i);
    col[(size_t)10 * nre] = make_float2(m2.r, m2.i);
    ivec(col, nre, c0, m0, nullptr, 2, 1, 1);
    ivec(col, nre, m0, m1, nullptr, 4, 3, 3);
    ivec(col, nre, m1, m2, nullptr, 4, 3, 7);
    ivec(col, nre, m1, m2, &m2, 4, 1, 11);
  }
  if (tid == 0) {
    float* s = a.stats + (size_t)(rx * a.nports + port) * 8;
    s[0]     = noise;
    s[1] = s[2] = s[3] = s[4] = s[5] = 0.f;
  }
}

hipError_t chest_mbsfn_launch(const ChestArgs& a, hipStream_t stream)
{
  StageScope timing_scope(ST_CHEST, stream);
  if (a.nports > 2 || a.nof_prb > CHEST_MAX_PRB || !a.mbsfn_pilots) {
    return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(chest_mbsfn_kernel, dim3(a.nports * a.nrx), dim3(CH_THREADS), 0, stream, a);
  return hipGetLastError();
}

hipError_t chest_set_stamps(void* d_buf)
{
#ifdef CHEST_STAMPS
  unsigned long long* p = (unsigned long long*)d_buf;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_chest_stamps), &p, sizeof(p));
#else
  (void)d_buf;
  return hipErrorNotSupported;
#endif
}

hipError_t chest_launch(const ChestArgs& a, hipStream_t stream, uint32_t nsf)
{
  StageScope timing_scope(ST_CHEST, stream);
  if (a.nsymb != 7 && a.nsymb != 6) {
    return hipErrorInvalidValue;
  }
  if (nsf == 0) {
    return hipSuccess;
  }
  const size_t lds = (size_t)(a.estimator == 1 && !a.filter_none ? 8 : 4) * 2 * a.nof_prb * sizeof(cx);
  hipLaunchKernelGGL(chest_kernel, dim3(a.nports * a.nrx, nsf), dim3(CH_THREADS), lds, stream, a);
  return hipGetLastError();
}

// One workgroup, a thread per subframe (in turns of 256).  A subframe without a CFO estimate of its own (a TDD special
// subframe: fewer than 4 CRS symbols) reports the last estimate before it -- of this batch, or *cfo_state, the last of
// the batches before -- as the host-synchronous path keeps q->cfo (chest_api.cpp); *cfo_state holds the batch's last
// value afterwards.
constexpr uint32_t FIN_THREADS = 256;
__global__ __launch_bounds__(FIN_THREADS) void chest_finalize_kernel(const float* stats, uint32_t np, uint32_t nrx,
                                                                     uint32_t nof_prb, float sz, float nsymb, float* out,
                                                                     uint32_t nsf, float* cfo_state)
{
  __shared__ int last_est[FIN_THREADS];  // per turn: the highest subframe with its own estimate, per thread
  __shared__ float carry;
  if (threadIdx.x == 0) {
    carry = cfo_state ? *cfo_state : 0.f;
  }
  for (uint32_t base = 0; base < nsf; base += FIN_THREADS) {
    const uint32_t b   = base + threadIdx.x;
    const bool     own = b < nsf && finalize_sf(stats + b * CHEST_STATS_PER_SF, np, nrx, nof_prb, sz, nsymb, out + 4 * b);
    last_est[threadIdx.x] = own ? (int)threadIdx.x : -1;
    __syncthreads();  // carry (first turn) and the turn's outputs
    for (uint32_t off = 1; off < FIN_THREADS; off <<= 1) {  // inclusive prefix max: the last estimate at or before
      const int v = threadIdx.x >= off ? last_est[threadIdx.x - off] : -1;
      __syncthreads();
      last_est[threadIdx.x] = max(last_est[threadIdx.x], v);
      __syncthreads();
    }
    if (b < nsf && !own) {
      const int j = last_est[threadIdx.x];
      out[4 * b + 3] = j >= 0 ? out[4 * (base + j) + 3] : carry;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t n = min(nsf - base, FIN_THREADS);
      const int      j = last_est[n - 1];
      carry            = j >= 0 ? out[4 * (base + j) + 3] : carry;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && cfo_state) {
    *cfo_state = carry;
  }
}

// PSS / EMPTY over a batch: one thread walks the subframes in order, carrying each (rx, port)'s kept estimate
__global__ void chest_keep_kernel(float* stats, uint32_t np, uint32_t nrx, float* state, uint32_t nsf)
{
  if (threadIdx.x != 0 || blockIdx.x != 0) {
    return;
  }
  for (uint32_t b = 0; b < nsf; b++) {
    float* st = stats + b * CHEST_STATS_PER_SF;
    for (uint32_t rx = 0; rx < nrx; rx++) {
      for (uint32_t p = 0; p < np; p++) {
        float* v = st + (rx * np + p) * 8;
        if (v[5] != 0.0f) {
          state[rx * 4 + p] = v[0];
        } else {
          v[0] = state[rx * 4 + p];
        }
      }
    }
  }
}

hipError_t chest_finalize_kept_launch(float* stats, uint32_t np, uint32_t nrx, uint32_t nof_prb, float symbol_sz,
                                      uint32_t nsymb, float* state, float* out, uint32_t nsf, hipStream_t stream,
                                      float* cfo_state)
{
  if (nsf == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(chest_keep_kernel, dim3(1), dim3(64), 0, stream, stats, np, nrx, state, nsf);
  return chest_finalize_launch(stats, np, nrx, nof_prb, symbol_sz, nsymb, out, nsf, stream, cfo_state);
}

// correct_sync_error's device part: one workgroup per (port, rx) and subframe (blockIdx.y; batches: the subframe
// indices as chest_kernel takes them)
__global__ __launch_bounds__(CH_THREADS) void chest_sync_kernel(ChestArgs a, float* out)
{
  __shared__ float red[2 * CH_THREADS / 64];
  const uint32_t   port = blockIdx.x / a.nrx, rx = blockIdx.x % a.nrx, b = blockIdx.y;
  const bool       bat  = a.sf_inl || a.sf_idx;
  const uint32_t   sfi  = a.sf_inl ? (uint32_t)a.sf_inline[b] : a.sf_idx ? a.sf_idx[b] : a.sf_index;
  const uint32_t   nsym = chest_crs_nsym(a, sfi, port), nref = 2 * a.nof_prb, nre = 12 * a.nof_prb;
  const float2*    in   = a.grid + b * a.grid_sf_stride + (size_t)rx * 2 * a.nsymb * nre;
  const float2*    pil  = a.pilots + (bat ? sfi * CHEST_PILOTS_PER_SF : 0) + (size_t)(port / 2) * 4 * CHEST_MAX_NREF;
  float*           o    = out + (size_t)b * CHEST_SYNC_PER_SF + (rx * 4 + port) * 10;
  float            pwr  = 0.f;
  for (uint32_t l = 0; l < nsym; l++) {
    const uint32_t row = crs_nsymbol(l, port, a.nsymb) * nre, f0 = (crs_v(port, l) + a.cell_id % 6) % 6;
    float          sr = 0.f, si = 0.f;
    for (uint32_t i = threadIdx.x; i < nref; i += CH_THREADS) {
      const cx x = mul(ld2(in, row + f0 + 6 * i), conj(ld2(pil, l * nref + i)));
      pwr += x.r * x.r + x.i * x.i;
      if (i > 0) {  // x[i] conj(x[i - 1])
        const cx y = mul(ld2(in, row + f0 + 6 * (i - 1)), conj(ld2(pil, l * nref + i - 1)));
        const cx t = mul(x, conj(y));
        sr += t.r;
        si += t.i;
      }
    }
    block_sum2(sr, si, red);
    if (threadIdx.x == 0) {
      o[2 * l]     = sr;
      o[2 * l + 1] = si;
    }
  }
  pwr = block_sum(pwr, red);
  if (threadIdx.x == 0) {
    o[8] = pwr;
  }
}

hipError_t chest_sync_sums_launch(const ChestArgs& a, float* out, hipStream_t stream, uint32_t nsf)
{
  if (nsf == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(chest_sync_kernel, dim3(a.nports * a.nrx, nsf), dim3(CH_THREADS), 0, stream, a, out);
  return hipGetLastError();
}

// srsran_vec_apply_cfo's complex product (simd.h:898-901, AVX2 + FMA build)
__device__ __forceinline__ float2 cfo_prod(float2 x, float2 p)
{
  return make_float2(__fmaf_rn(x.x, p.x, -__fmul_rn(x.y, p.y)), __fmaf_rn(x.x, p.y, __fmul_rn(x.y, p.x)));
}

// correct_sync_error of a batch (chest_dl.c:750-804), one workgroup per (rx, subframe): the reference's scalar
// arithmetic on the phase sums of chest_sync_kernel (thread 0), then -- where the error exceeds 0.05 samples -- the
// phasor table of srsran_vec_apply_cfo (8 lanes carry the SIMD phases, lane 0 the tail) in LDS and every row of the
// rx grid rotated in place.  The phasor's sincosf / the phase atan2f are the device's (the host-synchronous path
// uses the host's libm), so corrected grids can differ from it in the last bit of a rotated sample.
__global__ __launch_bounds__(CH_THREADS) void chest_sync_apply_kernel(ChestArgs a, const float* __restrict__ sums,
                                                                      float* __restrict__ serr, float2* grid, float sz)
{
  __shared__ float2 tab[12 * CHEST_MAX_PRB];
  __shared__ float2 w_sh;
  __shared__ int    rot_sh;
  const uint32_t rx = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const uint32_t sfi = a.sf_inl ? (uint32_t)a.sf_inline[b] : a.sf_idx ? a.sf_idx[b] : a.sf_index;
  const uint32_t nre = 12 * a.nof_prb, rows = 2 * a.nsymb;
  if (tid == 0) {
    float pwr_sum = 0.0f, err = 0.0f;
    for (uint32_t port = 0; port < a.nports; port++) {
      const float*   o    = sums + (size_t)b * CHEST_SYNC_PER_SF + (rx * 4 + port) * 10;
      const uint32_t nsym = chest_crs_nsym(a, sfi, port), npilots = nsym * 2 * a.nof_prb;
      const float    k    = sz / 6.0f;
      float          sum  = 0.0f;
      for (uint32_t l = 0; l < nsym; l++) {  // srsran_vec_estimate_frequency: -cargf(sum) * M_1_PI * 0.5f
        const float f = (float)((double)-atan2f(o[2 * l + 1], o[2 * l]) * 0.31830988618379067154 * 0.5f);
        sum += f * k;
      }
      const float pwr = o[8] / (float)npilots;
      const float se  = sum / (float)nsym;
      serr[(size_t)b * 16 + rx * 4 + port] = se;
      if (!isinf(sum) && !isnan(sum) && !isinf(pwr) && !isnan(pwr)) {
        err += se * pwr;
        pwr_sum += pwr;
      }
    }
    if (isnormal(pwr_sum)) {
      err /= pwr_sum;
    }
    rot_sh = isnormal(err) && fabsf(err) > 0.05f;
    float c, s;
    sincosf((2.0f * 3.14159265358979323846f) * (err / sz), &s, &c);  // cfo_phasor of err / symbol size
    w_sh = make_float2(c, s);
  }
  __syncthreads();
  if (!rot_sh) {
    return;
  }
  if (tid < 8) {  // srsran_vec_apply_cfo's phasors over nre samples (as cfo_table_kernel)
    const float2 w = w_sh;
    float2       p = make_float2(1.0f, 0.0f);
    for (uint32_t j = 0; j < tid; j++) {
      p = cfo_prod(p, w);
    }
    float2 w8 = make_float2(1.0f, 0.0f);
    for (uint32_t j = 0; j < 8; j++) {
      w8 = cfo_prod(w8, w);
    }
    const uint32_t nblk = nre / 8;
    for (uint32_t m = 0; m < nblk; m++) {
      tab[8 * m + tid] = p;
      p                = cfo_prod(p, w8);
    }
    if (tid == 0) {
      for (uint32_t i = 8 * nblk; i < nre; i++) {
        tab[i] = p;
        p      = cfo_prod(p, w);
      }
    }
  }
  __syncthreads();
  float2* g = grid + b * a.grid_sf_stride + (size_t)rx * rows * nre;
  for (uint32_t i = tid; i < rows * nre; i += CH_THREADS) {
    g[i] = cfo_prod(g[i], tab[i % nre]);
  }
}

hipError_t chest_sync_apply_launch(const ChestArgs& a, const float* sums, float* serr, float2* grid, float symbol_sz,
                                   uint32_t nsf, hipStream_t stream)
{
  if (nsf == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(chest_sync_apply_kernel, dim3(a.nrx, nsf), dim3(CH_THREADS), 0, stream, a, sums, serr, grid,
                     symbol_sz);
  return hipGetLastError();
}

// srsran_vec_apply_cfo's product (simd.h:898-901): re = fma(x.re, p.re, -(x.im p.im)), im = fma(x.re, p.im, x.im p.re)
__global__ void grid_rotate_kernel(float2* grid, const float2* __restrict__ tab, uint32_t nre, uint32_t total)
{
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < total) {
    const float2 x = grid[k], p = tab[k % nre];
    grid[k] = make_float2(__fmaf_rn(x.x, p.x, -__fmul_rn(x.y, p.y)), __fmaf_rn(x.x, p.y, __fmul_rn(x.y, p.x)));
  }
}

hipError_t grid_rotate_launch(float2* grid, const float2* tab, uint32_t nre, uint32_t nrows, hipStream_t stream)
{
  const uint32_t total = nre * nrows;
  if (total == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(grid_rotate_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, grid, tab, nre, total);
  return hipGetLastError();
}

hipError_t chest_finalize_launch(const float* stats, uint32_t np, uint32_t nrx, uint32_t nof_prb, float symbol_sz,
                                 uint32_t nsymb, float* out, uint32_t nsf, hipStream_t stream, float* cfo_state)
{
  StageScope timing_scope(ST_CHEST, stream);
  if (nsf == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(chest_finalize_kernel, dim3(1), dim3(FIN_THREADS), 0, stream, stats, np, nrx, nof_prb, symbol_sz,
                     (float)nsymb, out, nsf, cfo_state);
  return hipGetLastError();
}

}  // namespace srsran_amd
