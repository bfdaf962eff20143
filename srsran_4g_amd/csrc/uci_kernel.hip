// srsran_4g_amd/csrc/uci_kernel.hip -- UCI on PUSCH, receive side, for gfx950.
//
// The control information is a few hundred soft bits per TB, so each kernel runs one 64-lane wave
// per TB (grid = TBs of the batch) and keeps everything in LDS:
//   uci_ack_ri_kernel  HARQ-ACK: gather the Q'_ACK Qm soft bits at their interleaver positions
//                      (uci.c:364-388) into the circular accumulator of srsran_uci_decode_ack_ri
//                      (uci.c:641-714: 16-bit wrap, clamp to +-16383 after every add, the 1-bit
//                      repetition descrambling from the sequence), decide (1 bit: sum; 2 bits:
//                      parity-checked sums; 3..10 bits: (32, O) block code ML), threshold; zero
//                      the ACK positions (sch.c:1083-1086); then RI the same way (sch.c:1089-1110).
//   uci_cqi_kernel     CQI from the front of the de-interleaved LLRs: <= 11 bits the (32, O) block
//                      code ML over the wrap-summed copies (block.c:240-259), otherwise the 16-bit
//                      rate de-matcher (rm_conv.c:159-217, RX_NULL = 10000 semantics), the
//                      quantiser of srsran_viterbi_decode_s (viterbi.c:579-605: 32767 + x), the
//                      tail-biting Viterbi (viterbi_dev.h) and the CRC8 check (uci.c:268-296).
// The block-code ML runs the 2^O hypotheses across the lanes; the reference's strict ">" from a
// zero start is kept by reducing (correlation, -hypothesis) and mapping a non-positive best to 0.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "uci_kernel.h"
#include "viterbi_dev.h"

namespace srsran_amd {
namespace {

// (32, O) basis sequences, 36.212 Table 5.2.2.6.4-1; bit n of word i is M_{i,n} (block.c:37-43)
__constant__ uint16_t kBlockBasis[32] = {0x403, 0x607, 0x749, 0x50D, 0x48F, 0x5D3, 0x755, 0x599, 0x69B, 0x65D, 0x6E5,
                                         0x567, 0x7A9, 0x6AB, 0x4B1, 0x6F3, 0x277, 0x139, 0x0FB, 0x061, 0x445, 0x60B,
                                         0x591, 0x717, 0x3DF, 0x4E3, 0x32D, 0x3AF, 0x175, 0x1FD, 0x7FF, 0x001};
// interleaver column sets (36.212 Tables 5.2.2.8-1 / -2), normal and extended CP
__constant__ uint8_t kAckCols[2][4] = {{2, 3, 8, 9}, {1, 2, 6, 7}};
__constant__ uint8_t kRiCols[2][4]  = {{1, 4, 7, 10}, {0, 3, 5, 8}};
constexpr int        NCOLS          = 32;
__constant__ uint8_t kPerm[NCOLS]    = {1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
                                        0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30};
__constant__ uint8_t kPermInv[NCOLS] = {16, 0, 24, 8, 20, 4, 28, 12, 18, 2, 26, 10, 22, 6, 30, 14,
                                        17, 1, 25, 9, 21, 5, 29, 13, 19, 3, 27, 11, 23, 7, 31, 15};
constexpr int        RX_NULL         = 10000;  // SRSRAN_RX_NULL
constexpr uint32_t   CQI_MAX_CODED   = 3 * (UCI_MAX_CQI_BITS + 8);

__device__ __forceinline__ uint32_t uci_pos(uint32_t idx, uint32_t k, const UciDesc& d, bool ri)
{
  const uint32_t row = d.rows - 1 - idx / 4, c = (3 * idx) % 4, ext = d.cols > 10 ? 0 : 1;
  const uint32_t col = ri ? kRiCols[ext][c] : kAckCols[ext][c];
  return row * d.Qm + d.rows * col * d.Qm + k;
}

// srsran_block_decode over 32 accumulated soft bits (block.c:196-232): returns the correlation,
// writes min(nbits, 11) bits
__device__ int32_t block_ml(const int16_t* llr32, uint32_t nbits, uint8_t* data, int lane)
{
  nbits               = min(nbits, 11u);
  const uint32_t ng   = 1u << nbits;
  int32_t        best = INT32_MIN;
  uint32_t       bw   = 0;
  for (uint32_t w = (uint32_t)lane; w < ng; w += 64) {
    int32_t corr = 0;
    for (int i = 0; i < 32; i++) {
      const int32_t e = (int32_t)(__builtin_popcount(w & kBlockBasis[i]) & 1) * 2 - 1;
      corr += (int32_t)llr32[i] * e;
    }
    if (corr > best) {  // ascending w: the first maximum of the lane
      best = corr;
      bw   = w;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const int32_t  ob = __shfl_xor(best, off, 64);
    const uint32_t ow = (uint32_t)__shfl_xor((int)bw, off, 64);
    if (ob > best || (ob == best && ow < bw)) {
      best = ob;
      bw   = ow;
    }
  }
  if (best <= 0) {  // max_corr starts at 0 with word 0 and only a strictly larger one replaces it
    best = 0;
    bw   = 0;
  }
  if (lane == 0) {
    for (uint32_t i = 0; i < nbits; i++) {
      data[i] = (uint8_t)((bw >> i) & 1u);
    }
  }
  return best;
}

// srsran_uci_decode_ack_ri (uci.c:641-714) for one wave; returns corr > thr
__device__ bool decode_ack_ri(const UciDesc& d, uint32_t nbits, uint32_t Qp, bool ri, int16_t* acc, uint8_t* data,
                              int32_t* corr_out, int32_t* thr_out, int lane)
{
  const uint32_t Qm    = d.Qm;
  const uint32_t nacc  = nbits == 1 ? Qm : nbits == 2 ? Qm * 3 : 32;
  const uint32_t count = Qp * Qm;
  if (lane < 32) {
    int16_t a = 0;
    if ((uint32_t)lane < nacc) {
      for (uint32_t c = (uint32_t)lane; c < count; c += nacc) {
        const uint32_t pos = uci_pos(c / Qm, c % Qm, d, ri);
        int16_t        v   = d.q[pos];
        if (nbits == 1 && lane == 1 && pos > 0) {
          v = d.c[pos] == d.c[pos - 1] ? v : (int16_t)(-v);
        }
        a = (int16_t)(a + v);
        a = (int16_t)min((int)a, 16383);
        a = (int16_t)max((int)a, -16383);
      }
    }
    acc[lane] = a;
  }
  __syncthreads();
  int32_t corr = 0;
  if (nbits == 1) {
    const int32_t sum = (int32_t)acc[0] + (int32_t)acc[1];
    if (lane == 0) {
      data[0] = sum > 0 ? 1 : 0;
    }
    corr = abs(sum);
  } else if (nbits == 2) {
    const int16_t s1 = (int16_t)(acc[0] + acc[Qm + 1]);
    const int16_t s2 = (int16_t)(acc[1] + acc[2 * Qm]);
    const int16_t s3 = (int16_t)(acc[Qm] + acc[2 * Qm + 1]);
    const uint8_t d0 = s1 > 0 ? 1 : 0, d1 = s2 > 0 ? 1 : 0;
    if (lane == 0) {
      data[0] = d0;
      data[1] = d1;
    }
    corr = ((s3 > 0) == ((d0 ^ d1) != 0)) ? abs((int)s1) + abs((int)s2) + abs((int)s3) : 0;
  } else {
    corr = block_ml(acc, nbits, data, lane);
  }
  const uint32_t f   = Qm < 4 ? 100u : Qm < 6 ? 200u : Qm < 8 ? 700u : 1000u;
  const int32_t  thr = (int32_t)(count * f / Qm);
  if (corr_out) {
    *corr_out = corr;
    *thr_out  = thr;
  }
  __syncthreads();
  return corr > thr;
}

}  // namespace

__global__ __launch_bounds__(64) void uci_ack_ri_kernel(const UciDesc* __restrict__ desc)
{
  __shared__ int16_t acc[32];
  __shared__ uint8_t bits[16];
  const UciDesc      d    = desc[blockIdx.x];
  const int          lane = threadIdx.x;
  if (d.ack_bits > 0) {
    int32_t    corr = 0, thr = 0;
    const bool ok   = decode_ack_ri(d, d.ack_bits, d.ack_Qp, false, acc, bits, &corr, &thr, lane);
    __syncthreads();
    if (lane == 0) {
      for (uint32_t i = 0; i < min(d.ack_bits, 11u) && i < 16; i++) {
        d.out->ack[i] = bits[i];
      }
      d.out->ack_corr  = corr;
      d.out->ack_thr   = thr;
      d.out->ack_valid = ok ? 1u : 0u;
    }
    // zero the HARQ positions (the data around them is punctured, not rate matched)
    for (uint32_t c = (uint32_t)lane; c < d.ack_Qp * d.Qm; c += 64) {
      d.q[uci_pos(c / d.Qm, c % d.Qm, d, false)] = 0;
    }
    __syncthreads();
  }
  if (d.ri_bits > 0) {
    decode_ack_ri(d, d.ri_bits, d.ri_Qp, true, acc, bits, nullptr, nullptr, lane);
    __syncthreads();
    if (lane == 0) {
      for (uint32_t i = 0; i < min(d.ri_bits, 4u); i++) {
        d.out->ri[i] = bits[i];
      }
    }
  }
}

__global__ __launch_bounds__(64) void uci_cqi_kernel(const UciDesc* __restrict__ desc)
{
  __shared__ int16_t  acc[32];
  __shared__ int16_t  rm[CQI_MAX_CODED];
  __shared__ uint16_t sym[CQI_MAX_CODED];
  __shared__ uint64_t dec[5 * (UCI_MAX_CQI_BITS + 8) + 6];
  __shared__ uint8_t  data[UCI_MAX_CQI_BITS + 8];
  __shared__ uint8_t  dcb[NCOLS];
  const UciDesc       d    = desc[blockIdx.x];
  const int           lane = threadIdx.x;
  const uint32_t      Q    = d.cqi_Qp * d.Qm;
  if (d.cqi_bits == 0) {
    return;
  }
  if (d.cqi_bits <= 11) {
    // block.c:240-259: the 32-periodic copies summed with 16-bit wrap (srsran_vec_sum_sss)
    if (lane < 32) {
      int16_t a = 0;
      for (uint32_t t = (uint32_t)lane; t < Q; t += 32) {
        a = (int16_t)(a + d.g[t]);
      }
      acc[lane] = a;
    }
    __syncthreads();
    block_ml(acc, d.cqi_bits, data, lane);
    __syncthreads();
    if (lane == 0) {
      for (uint32_t i = 0; i < UCI_MAX_CQI_BITS; i++) {
        d.out->cqi[i] = i < d.cqi_bits ? data[i] : 0;
      }
      d.out->cqi_crc = 1;
    }
    return;
  }
  // ---- srsran_rm_conv_rx_s (rm_conv.c:159-217) ----
  const uint32_t F    = d.cqi_bits + 8;
  const uint32_t clen = 3 * F;
  const int      nrows = (int)((clen / 3 - 1) / NCOLS + 1);
  const int      Kp    = nrows * NCOLS;
  const int      nd    = max(0, Kp - (int)(clen / 3));
  const int      nv    = 3 * (Kp - nd);
  if (lane == 0) {
    int a = 0;
    for (int col = 0; col < NCOLS; col++) {
      dcb[col] = (uint8_t)a;
      a += kPerm[col] < nd ? 1 : 0;
    }
  }
  __syncthreads();
  for (uint32_t oi = (uint32_t)lane; oi < clen; oi += 64) {
    const int i = (int)(oi / 3), j = (int)(oi - 3 * (oi / 3));
    const int di = (i + nd) / NCOLS, dj = (i + nd) % NCOLS;
    const int p  = Kp * j + kPermInv[dj] * nrows + di;
    // rank of p among the non-dummy circular-buffer positions (only row 0 of a dummy column is dummy)
    const int  s = p / Kp, qq = p - s * Kp, col = qq / nrows, r = qq - col * nrows;
    const bool dcol = kPerm[col] < nd;
    int16_t    t    = (int16_t)RX_NULL;
    if (!(r == 0 && dcol)) {
      const int rk = s * (Kp - nd) + col * nrows - dcb[col] + r - (dcol ? 1 : 0);
      for (int k = rk; k < (int)Q; k += nv) {
        const int16_t x = d.g[k];
        if (t == RX_NULL) {
          t = x;
        } else if (x != RX_NULL) {
          t = (int16_t)(t + x);
        }
      }
    }
    rm[oi] = t != RX_NULL ? t : 0;
  }
  __syncthreads();
  // ---- srsran_vec_quant_sus(x, 1, 32767, 65535) ----
  for (uint32_t i = (uint32_t)lane; i < clen; i += 64) {
    sym[i] = (uint16_t)min(max(32767 + (int)rm[i], 0), 65535);
  }
  __syncthreads();
  viterbi37_tb16(sym, F, dec, data, lane);
  if (lane == 0) {
    // CRC8 (SRSRAN_LTE_CRC8 = 0x19B) over the payload and its parity: zero remainder = match
    uint32_t crc = 0;
    for (uint32_t i = 0; i < F; i++) {
      const uint32_t fb = ((crc >> 7) & 1u) ^ data[i];
      crc               = (crc << 1) & 0xffu;
      if (fb) {
        crc ^= 0x9Bu;
      }
    }
    const bool ok = crc == 0;
    for (uint32_t i = 0; i < UCI_MAX_CQI_BITS; i++) {
      d.out->cqi[i] = (ok && i < d.cqi_bits) ? data[i] : 0;
    }
    d.out->cqi_crc = ok ? 1u : 0u;
  }
}

hipError_t uci_ack_ri_launch(const UciDesc* d_desc, uint32_t ntb, hipStream_t stream)
{
  if (ntb == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(uci_ack_ri_kernel, dim3(ntb), dim3(64), 0, stream, d_desc);
  return hipGetLastError();
}

hipError_t uci_cqi_launch(const UciDesc* d_desc, uint32_t ntb, hipStream_t stream)
{
  if (ntb == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(uci_cqi_kernel, dim3(ntb), dim3(64), 0, stream, d_desc);
  return hipGetLastError();
}

}  // namespace srsran_amd
