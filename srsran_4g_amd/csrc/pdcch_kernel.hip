// srsran_4g_amd/csrc/pdcch_kernel.hip -- PCFICH / PDCCH receive kernels for gfx950.
//
// RE extraction fused into the predecoding: 2-port TX diversity in ctrl_diversity_kernel (the
// reference's SSE / generic arithmetic split), 1 port in the PDSCH predecoder (eq_kernel.hip, MMSE).
// Then:
//   pcfich_kernel      QPSK soft demodulation (demod_soft.c:120-123: x * -sqrt(2)), descrambling
//                      (scrambling.c: x * c, c = +-1) and the CFI correlation (pcfich.c:113-134)
//   pdcch_llr_kernel   the same demodulation / descrambling over the control region
//                      (pdcch.c:449-516, srsran_scrambling_f_offset at offset 0)
//   pdcch_cand_kernel  one wave per candidate (location x format): the |LLR| mean gate
//                      (pdcch.c:371-378), rate de-matching (rm_conv.c:120-175, every soft-buffer
//                      position gathers its contributions in the reference's order: no atomics),
//                      quantisation (viterbi.c:546-585), the 16-bit tail-biting Viterbi decoder of
//                      the AVX2 build (viterbi37_avx2_16bit.c) with lane = trellis state, decisions
//                      as 64-bit ballots in LDS, chainback, CRC16 / RNTI (pdcch.c:313-350), and the
//                      re-encoding correlation of srsran_pdcch_msg_corr (pdcch.c:418-437).
// Restated step by step in oracle/pdcch_oracle.c, which is pinned to the compiled reference.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pdcch_kernel.h"
#include "viterbi_dev.h"

namespace srsran_amd {
namespace {

#pragma clang fp contract(off)

constexpr float   NSQRT2  = -1.41421356237309504880f;  // (float)(-M_SQRT2)
constexpr float   RX_NULL = 10000.0f;                  // SRSRAN_RX_NULL
constexpr int     NCOLS   = 32;
__constant__ uint8_t kPerm[NCOLS] = {1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
                                     0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30};
__constant__ uint8_t kPermInv[NCOLS] = {16, 0, 24, 8, 20, 4, 28, 12, 18, 2, 26, 10, 22, 6, 30, 14,
                                        17, 1, 25, 9, 21, 5, 29, 13, 19, 3, 27, 11, 23, 7, 31, 15};
// PCFICH codewords (36.212 Table 5.3.4-1) as bits: cfi c -> 32-bit word, bit i = codeword bit i
__constant__ uint32_t kCfiWords[3] = {0xB6DB6DB6u, 0x6DB6DB6Du, 0xDB6DB6DBu};

__device__ __forceinline__ float qpsk_llr(const float2* x, uint32_t i, const uint32_t* seq)
{
  const float2 s = x[i >> 1];
  float        v = ((i & 1) ? s.y : s.x) * NSQRT2;
  if ((seq[i >> 5] >> (i & 31)) & 1u) {
    v = v * -1.0f;
  }
  return v;
}

__global__ void pcfich_kernel(const float2* __restrict__ x, const uint32_t* __restrict__ seq, float* __restrict__ data_f,
                              uint32_t* __restrict__ cfi_out, float* __restrict__ corr_out)
{
  __shared__ float llr[32];
  const int t = threadIdx.x;
  if (t < 32) {
    llr[t]    = qpsk_llr(x, (uint32_t)t, seq);
    data_f[t] = llr[t];
  }
  __syncthreads();
  if (t == 0) {
    float best = 0.0f;
    int   idx  = 0;
    for (int c = 0; c < 3; c++) {
      float acc = 0.0f;
      for (int i = 0; i < 32; i++) {
        const float cb = ((kCfiWords[c] >> i) & 1u) ? 1.0f : -1.0f;  // 2 b - 1
        acc            = acc + cb * llr[i];
      }
      if (acc > best) {
        best = acc;
        idx  = c;
      }
    }
    *cfi_out  = (uint32_t)idx + 1;
    *corr_out = best;
  }
}

__global__ void pdcch_llr_kernel(const float2* __restrict__ x, uint32_t nbits, const uint32_t* __restrict__ seq,
                                 float* __restrict__ llr)
{
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nbits; i += gridDim.x * blockDim.x) {
    llr[i] = qpsk_llr(x, i, seq);
  }
}

// ---- control-channel TX-diversity predecoding (2 ports) with the RE gather fused ----
// srsran_predecoding_diversity_multi without CSI (precoding.c:780-800): the SSE body
// (srsran_predecoding_diversity2_sse, precoding.c:518-643) for the first 4 * (n / 4) symbols when
// n > 32, the generic loop (precoding.c:428-503) for the rest; the layer demapping
// (srsran_layerdemap_diversity) is the codeword order d[2k + l] = x_l[k].
struct cpx {
  float r, i;
};
__device__ __forceinline__ cpx ldc(const float2* p, uint32_t k)
{
  const float2 v = p[k];
  return {v.x, v.y};
}
__device__ __forceinline__ cpx cmulf(cpx a, cpx b) { return {a.r * b.r - a.i * b.i, a.i * b.r + a.r * b.i}; }
__device__ __forceinline__ cpx conjf(cpx a) { return {a.r, -a.i}; }

__global__ void ctrl_diversity_kernel(CtrlEqArgs a)
{
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;  // symbol pair
  if (k >= a.n / 2) {
    return;
  }
  const uint32_t g0 = a.idx[2 * k], g1 = a.idx[2 * k + 1];
  cpx            x0 = {0.f, 0.f}, x1 = {0.f, 0.f};
  float          hh = 0.f;
  const bool     sse = 2 * k < a.sse_symbols;
  for (int p = 0; p < a.nrx; p++) {
    const cpx h00 = ldc(a.h[0][p], g0), h01 = ldc(a.h[0][p], g1), h10 = ldc(a.h[1][p], g0), h11 = ldc(a.h[1][p], g1);
    const cpx r0 = ldc(a.y[p], g0), r1 = ldc(a.y[p], g1);
    if (sse) {
      const float h  = (h00.r * h00.r + h00.i * h00.i) + (h11.r * h11.r + h11.i * h11.i);
      hh             = p == 0 ? h : hh + h;
      const cpx a0 = cmulf(conjf(h00), r0), b0 = cmulf(h11, conjf(r1));
      const cpx a1 = cmulf(conjf(h01), r1), b1 = cmulf(h10, conjf(r0));
      const cpx t0 = {a0.r + b0.r, a0.i + b0.i}, t1 = {a1.r - b1.r, a1.i - b1.i};
      x0           = p == 0 ? t0 : cpx{x0.r + t0.r, x0.i + t0.i};
      x1           = p == 0 ? t1 : cpx{x1.r + t1.r, x1.i + t1.i};
    } else {
      hh = hh + (((h00.r * h00.r + h00.i * h00.i) + h11.r * h11.r) + h11.i * h11.i);  // hh += ...
      if (hh == 0.f) {
        hh = 1e-4f;
      }
      const cpx a0 = cmulf(conjf(h00), r0), b0 = cmulf(h11, conjf(r1));
      const cpx a1 = cmulf(cpx{-h10.r, -h10.i}, conjf(r0)), b1 = cmulf(conjf(h01), r1);
      x0           = {x0.r + (a0.r + b0.r), x0.i + (a0.i + b0.i)};
      x1           = {x1.r + (a1.r + b1.r), x1.i + (a1.i + b1.i)};
    }
  }
  float2 o0, o1;
  if (sse) {  // x / hh * (float)(M_SQRT2 / scaling), scaling = 1
    const float s2 = 1.41421356237309504880f;
    o0             = make_float2(__fdiv_rn(x0.r, hh) * s2, __fdiv_rn(x0.i, hh) * s2);
    o1             = make_float2(__fdiv_rn(x1.r, hh) * s2, __fdiv_rn(x1.i, hh) * s2);
  } else {  // x / hh * M_SQRT2 in double
    const double s2 = 1.41421356237309504880;
    o0 = make_float2((float)((double)__fdiv_rn(x0.r, hh) * s2), (float)((double)__fdiv_rn(x0.i, hh) * s2));
    o1 = make_float2((float)((double)__fdiv_rn(x1.r, hh) * s2), (float)((double)__fdiv_rn(x1.i, hh) * s2));
  }
  a.d[2 * k]     = o0;
  a.d[2 * k + 1] = o1;
}

__device__ __forceinline__ uint32_t parity32(uint32_t v) { return vit_parity32(v); }

// Rank of soft-buffer position p (stream s, column col, row r) among the non-dummy positions of
// the circular buffer (rm_conv.c bit collection order); -1 for a dummy position.  Only row 0 of a
// column whose permuted index is below ndummy (< 32) is a dummy.
__device__ __forceinline__ int cb_rank(int p, int nrows, int Kp, int ndummy, const uint8_t* dcols_before)
{
  const int s = p / Kp, q = p - s * Kp, col = q / nrows, r = q - col * nrows;
  const bool dcol = kPerm[col] < ndummy;
  if (r == 0 && dcol) {
    return -1;
  }
  return s * (Kp - ndummy) + col * nrows - dcols_before[col] + r - (dcol ? 1 : 0);
}

// Soft-buffer position of rank k (inverse of cb_rank).
__device__ __forceinline__ int cb_pos(int k, int nrows, int Kp, int ndummy)
{
  const int nv = Kp - ndummy, s = k / nv;
  int       r  = k - s * nv;
  for (int col = 0; col < NCOLS; col++) {
    const int cnt = nrows - (kPerm[col] < ndummy ? 1 : 0);
    if (r < cnt) {
      return s * Kp + col * nrows + r + (kPerm[col] < ndummy ? 1 : 0);
    }
    r -= cnt;
  }
  return -1;
}

}  // namespace

// One 64-lane workgroup per candidate.
__global__ __launch_bounds__(64) void pdcch_cand_kernel(const float* __restrict__ llr, const PdcchCand* __restrict__ cands,
                                                        PdcchCandOut* __restrict__ outs)
{
  __shared__ float    rm[3 * (PDCCH_MAX_BITS + 16)];
  __shared__ uint16_t sym[3 * (PDCCH_MAX_BITS + 16)];
  __shared__ uint64_t dec[5 * (PDCCH_MAX_BITS + 16) + 6];
  __shared__ uint8_t  data[PDCCH_MAX_BITS + 16];
  __shared__ uint8_t  dcb[NCOLS];
  __shared__ int      skip;

  const PdcchCand c    = cands[blockIdx.x];
  PdcchCandOut*   o    = outs + blockIdx.x;
  const int       lane = threadIdx.x;
  const uint32_t  E    = 72u << c.L;
  const float*    e    = llr + 72u * c.ncce;
  const uint32_t  F    = c.nof_bits + 16;  // frame length
  const uint32_t  clen = 3 * F;

  // ---- mean |LLR| gate (pdcch.c:371-378: double accumulation in order, > 0.3f) ----
  if (lane == 0) {
    double mean = 0;
    for (uint32_t i = 0; i < E; i++) {
      mean += fabsf(e[i]);
    }
    mean /= E;
    skip = !(mean > 0.3f);
    o->nof_bits = skip ? 0 : c.nof_bits;
    o->crc_rem  = 0;
    o->corr     = 0.0f;
  }
  __syncthreads();
  if (skip) {
    return;
  }

  // ---- rate de-matching (rm_conv.c:120-175) ----
  const int nrows = (int)((clen / 3 - 1) / NCOLS + 1);
  const int Kp    = nrows * NCOLS;
  const int nd    = max(0, Kp - (int)(clen / 3));
  const int nv    = 3 * (Kp - nd);  // non-dummy positions of the circular buffer
  if (lane == 0) {
    int acc = 0;
    for (int col = 0; col < NCOLS; col++) {
      dcb[col] = (uint8_t)acc;
      acc += kPerm[col] < nd ? 1 : 0;
    }
  }
  __syncthreads();
  for (uint32_t oi = lane; oi < clen; oi += 64) {
    const int i = (int)(oi / 3), j = (int)(oi - 3 * (oi / 3));
    const int di = (i + nd) / NCOLS, dj = (i + nd) % NCOLS;
    const int p  = Kp * j + kPermInv[dj] * nrows + di;
    const int rk = cb_rank(p, nrows, Kp, nd, dcb);
    float     t  = RX_NULL;
    if (rk >= 0) {
      for (int k = rk; k < (int)E; k += nv) {
        if (t == RX_NULL) {
          t = e[k];
        } else if (e[k] != RX_NULL) {
          t = t + e[k];
        }
      }
    }
    rm[oi] = t != RX_NULL ? t : 0.0f;
  }
  __syncthreads();

  // ---- quantisation: gain 500 / max|x|, fused multiply-add as the reference build (viterbi.c:560-575) ----
  float mx = 0.0f;
  for (uint32_t i = lane; i < clen; i += 64) {
    mx = fmaxf(mx, fabsf(rm[i]));
  }
  for (int off = 32; off > 0; off >>= 1) {
    mx = fmaxf(mx, __shfl_xor(mx, off, 64));
  }
  const float mxv  = (mx > 0.0f && __builtin_isnormal(mx)) ? mx : 1e-9f;
  const float gain = __fdiv_rn(500.0f, mxv);
  for (uint32_t i = lane; i < clen; i += 64) {
    int v  = __float2int_rz(__builtin_fmaf(gain, rm[i], 32767.5f));
    sym[i] = (uint16_t)min(max(v, 0), 65535);
  }
  __syncthreads();

  // ---- Viterbi, lane = state (viterbi_dev.h) ----
  viterbi37_tb16(sym, F, dec, data, lane);
  if (lane == 0) {
    // CRC16 of the payload and the received parity (pdcch.c:333-345)
    uint32_t crc = 0;
    for (uint32_t i = 0; i < c.nof_bits; i++) {
      const uint32_t fb = ((crc >> 15) & 1u) ^ data[i];
      crc               = (crc << 1) & 0xffffu;
      if (fb) {
        crc ^= 0x1021u;
      }
    }
    uint32_t p = 0;
    for (int i = 0; i < 16; i++) {
      p = (p << 1) | data[c.nof_bits + i];
    }
    o->crc_rem = (uint16_t)(p ^ crc);
  }
  __syncthreads();
  for (uint32_t i = lane; i < c.nof_bits; i += 64) {
    o->payload[i] = data[i];
  }

  // ---- srsran_pdcch_msg_corr: re-encode (the decoded bits already carry the masked CRC),
  //      rate-match to E, QPSK, correlate with the LLRs as complex pairs ----
  float cr = 0.0f, ci = 0.0f;
  for (uint32_t k = 2 * lane; k < E; k += 128) {  // one QPSK symbol (2 bits) per iteration
    float dv[2];
    for (int h = 0; h < 2; h++) {
      const int pos = cb_pos((int)((k + h) % (uint32_t)nv), nrows, Kp, nd);
      const int st  = pos / Kp, q = pos - st * Kp, col = q / nrows, row = q - col * nrows;
      const int bi  = row * NCOLS + kPerm[col] - nd;  // coded bit index / 3
      uint32_t  sr  = 0;                              // tail-biting encoder register at bit bi
      for (int t = bi - 6; t <= bi; t++) {
        sr = (sr << 1) | data[(t + (int)F) % (int)F];
      }
      const uint32_t poly = st == 0 ? 0x6Du : st == 1 ? 0x4Fu : 0x57u;
      dv[h]               = parity32(sr & poly) ? -0.70710678118654752440f : 0.70710678118654752440f;
    }
    const float lr = e[k], li = e[k + 1];
    cr = cr + (lr * dv[0] + li * dv[1]);  // x * conj(d)
    ci = ci + (li * dv[0] - lr * dv[1]);
  }
  for (int off = 32; off > 0; off >>= 1) {
    cr = cr + __shfl_xor(cr, off, 64);
    ci = ci + __shfl_xor(ci, off, 64);
  }
  if (lane == 0) {
    const float n = (float)(E / 2);
    const float ar = cr / n, ai = ci / n;
    o->corr        = sqrtf(ar * ar + ai * ai) * 0.70710678118654752440f;
  }
}

hipError_t ctrl_diversity_launch(const CtrlEqArgs& a, hipStream_t stream)
{
  if (a.n < 2) {
    return hipSuccess;
  }
  const uint32_t pairs = a.n / 2;
  hipLaunchKernelGGL(ctrl_diversity_kernel, dim3((pairs + 255) / 256), dim3(256), 0, stream, a);
  return hipGetLastError();
}

hipError_t pcfich_launch(const float2* d_x, const uint32_t* d_seq, float* d_data_f, uint32_t* d_cfi, float* d_corr,
                         hipStream_t stream)
{
  hipLaunchKernelGGL(pcfich_kernel, dim3(1), dim3(64), 0, stream, d_x, d_seq, d_data_f, d_cfi, d_corr);
  return hipGetLastError();
}

hipError_t pdcch_llr_launch(const float2* d_x, uint32_t nbits, const uint32_t* d_seq, float* d_llr, hipStream_t stream)
{
  if (nbits == 0) {
    return hipSuccess;
  }
  const uint32_t grid = (nbits + 255) / 256;
  hipLaunchKernelGGL(pdcch_llr_kernel, dim3(grid), dim3(256), 0, stream, d_x, nbits, d_seq, d_llr);
  return hipGetLastError();
}

hipError_t pdcch_cand_launch(const float* d_llr, const PdcchCand* d_cands, uint32_t n, PdcchCandOut* d_outs,
                             hipStream_t stream)
{
  if (n == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(pdcch_cand_kernel, dim3(n), dim3(64), 0, stream, d_llr, d_cands, d_outs);
  return hipGetLastError();
}

}  // namespace srsran_amd
