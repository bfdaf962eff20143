// srsran_4g_amd/csrc/enc_kernel.hip -- DL-SCH transmit side for CDNA4:
//
//   enc_tb_crc_kernel  TB CRC24A (sch.c:240-359 through srsran_tcod_encode_lut's crc_tb): one
//                      workgroup per TB, the payload staged in LDS by coalesced loads, each thread the
//                      CRC of a contiguous chunk from zero, moved into place by x^(8 bytes_after) mod P
//                      and XOR-reduced (crc24_dev.h).
//   enc_cb_kernel      one workgroup of two waves per code block: the block's bits in LDS, CRC24B
//                      (C > 1) the same way, then the two constituent encoders of the PCCC
//                      (turbocoder.c: g0 = 13, g1 = 15 octal, 36.212 5.1.3.2), wave 0 on c(k),
//                      wave 1 on c(pi(k)) with pi the QPP interleaver.  The 8-state recursion is
//                      linear over GF(2), so each lane encodes a chunk of ceil(K/64) bits from the
//                      zero state, lane 0 chains the chunks' true start states through the
//                      zero-input transition of one chunk (an 8-entry table), and every lane
//                      re-encodes its chunk from its start state: 2 x ceil(K/64) dependent steps
//                      instead of K (the QPP index stepped incrementally, no division).  Trellis termination appends the 12 tail bits (natural
//                      3K+12 order).  Rate matching reads the circular buffer through the
//                      transmitter's read-out table (the inverse of the receive table): e(j) =
//                      coded(fwd(j mod (3K+12))), coalesced writes.
//   enc_pack_kernel    unpacked e bits -> bytes, MSB first (the packed e_bits of srsran_dlsch_encode).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc24_dev.h"
#include "enc_kernel.h"

namespace srsran_amd {

static constexpr uint32_t kCrc24A = 0x1864CFBu, kCrc24B = 0x1800063u;

// x^(8 n) mod P
__device__ __forceinline__ uint32_t xpow8(uint32_t n, uint32_t poly)
{
  uint32_t r = 1, b = 0x100u;  // x^8
  while (n) {
    if (n & 1u) {
      r = clmul_mod24(r, b, poly);
    }
    b = clmul_mod24(b, b, poly);
    n >>= 1;
  }
  return r;
}

// CRC (zero init, no final xor) of bytes [0, n) given by get(i), over one wave; result in every lane
template <typename F>
__device__ __forceinline__ uint32_t wave_crc(uint32_t n, uint32_t poly, F get)
{
  const uint32_t lane = threadIdx.x & 63, ch = (n + 63) / 64;
  const uint32_t b0 = min(lane * ch, n), b1 = min(b0 + ch, n);
  uint32_t       c  = 0;
  for (uint32_t i = b0; i < b1; i++) {
    c = crc24_byte(c, get(i), poly);
  }
  uint32_t part = b1 > b0 ? clmul_mod24(c, xpow8(n - b1, poly), poly) : 0u;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    part ^= (uint32_t)__shfl_xor((int)part, off, 64);
  }
  return part;
}

// 256 threads per TB: thread t CRCs bytes [t ch, (t+1) ch) from zero (the chunk is first copied to
// LDS with coalesced loads), moves it into place with x^(8 bytes_after), XOR-reduce
__global__ __launch_bounds__(256) void enc_tb_crc_kernel(const EncTb* __restrict__ tbs)
{
  const EncTb&       t = tbs[blockIdx.x];
  __shared__ uint8_t buf[12800];
  __shared__ uint32_t red[4];
  const uint32_t     n = t.nbytes, tid = threadIdx.x;
  uint32_t           part = 0;
  for (uint32_t base = 0; base < n; base += 12800) {  // <= 12800 bytes per pass (TBS <= 102400 bits)
    const uint32_t m = min(12800u, n - base);
    for (uint32_t i = tid; i < m; i += 256) {
      buf[i] = t.data[base + i];
    }
    __syncthreads();
    const uint32_t ch = (m + 255) / 256, b0 = min(tid * ch, m), b1 = min(b0 + ch, m);
    uint32_t       c  = 0;
    for (uint32_t i = b0; i < b1; i++) {
      c = crc24_byte(c, buf[i], kCrc24A);
    }
    if (b1 > b0) {
      part ^= clmul_mod24(c, xpow8(n - base - b1, kCrc24A), kCrc24A);
    }
    __syncthreads();
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    part ^= (uint32_t)__shfl_xor((int)part, off, 64);
  }
  if ((tid & 63) == 0) {
    red[tid >> 6] = part;
  }
  __syncthreads();
  if (tid == 0) {
    *t.crc = red[0] ^ red[1] ^ red[2] ^ red[3];
  }
}

hipError_t enc_tb_crc_launch(const EncTb* d_tbs, uint32_t ntb, hipStream_t stream)
{
  if (ntb == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(enc_tb_crc_kernel, dim3(ntb), dim3(256), 0, stream, d_tbs);
  return hipGetLastError();
}

// one step of a constituent encoder: state s = r0 | r1 << 1 | r2 << 2 (r0 newest); returns parity
__device__ __forceinline__ uint32_t rsc_step(uint32_t& s, uint32_t u)
{
  const uint32_t r0 = s & 1u, r1 = (s >> 1) & 1u, r2 = (s >> 2) & 1u;
  const uint32_t in = u ^ r2 ^ r1;
  const uint32_t p  = r2 ^ r0 ^ in;
  s                 = (in | (r0 << 1) | (r1 << 2));
  return p;
}

// The PCCC of one code block (turbocoder.c:77-185) by a 128-thread workgroup: wave w runs constituent encoder w
// (w = 1 on the QPP-interleaved bits), its 64 lanes on 64 chunks of the block chained through the zero-input
// transition; c = the K information bits (LDS, 0 / 1), coded = 3 K + 12 bits in srsran_tcod_encode's order
// (x_k, z_k, z'_k, then the two encoders' tail pairs).  Every thread of the workgroup calls it.
struct PcccLds {
  uint8_t e_end[2][64], s_start[2][64], T[2][8];
};
__device__ __forceinline__ void pccc_encode(const uint8_t* c, uint32_t K, uint32_t f1, uint32_t f2, uint8_t* coded, PcccLds& sh)
{
  const uint32_t tid = threadIdx.x, w = tid >> 6, lane = tid & 63;

  // pass 1: every chunk from the zero state; the zero-input transition of a whole chunk
  const uint32_t L = (K + 63) / 64, k0 = lane * L, k1 = min(k0 + L, K);
  // QPP pi(k) = (f1 k + f2 k^2) mod K stepped incrementally: pi(k+1) = pi(k) + g(k),
  // g(k+1) = g(k) + 2 f2 (mod K)
  const uint32_t pi0 = k0 < K ? (uint32_t)(((uint64_t)f1 * k0 + (uint64_t)f2 * k0 * k0) % K) : 0u;
  const uint32_t g0  = k0 < K ? (uint32_t)(((uint64_t)f1 + (uint64_t)f2 * (2 * (uint64_t)k0 + 1)) % K) : 0u;
  const uint32_t d2  = (uint32_t)((2 * (uint64_t)f2) % K);
  auto           adv = [&](uint32_t& p, uint32_t& g) {
    p += g;
    p -= p >= K ? K : 0u;
    g += d2;
    g -= g >= K ? K : 0u;
  };
  uint32_t s = 0, p = pi0, g = g0;
  for (uint32_t k = k0; k < k1; k++) {
    rsc_step(s, w ? c[p] : c[k]);
    adv(p, g);
  }
  sh.e_end[w][lane] = (uint8_t)s;
  if (lane < 8) {
    uint32_t t = lane;
    for (uint32_t k = 0; k < L; k++) {
      rsc_step(t, 0);
    }
    sh.T[w][lane] = (uint8_t)t;
  }
  __syncthreads();
  if (lane == 0) {
    uint32_t st = 0;
    for (uint32_t l = 0; l < 64; l++) {
      sh.s_start[w][l] = (uint8_t)st;
      st               = sh.T[w][st] ^ sh.e_end[w][l];
    }
  }
  __syncthreads();

  // pass 2: parity from the true start states; tail bits from the final state (natural order:
  // encoder 1's three (x, z) pairs, then encoder 2's)
  s = sh.s_start[w][lane];
  p = pi0;
  g = g0;
  for (uint32_t k = k0; k < k1; k++) {
    const uint32_t u = w ? c[p] : c[k];
    adv(p, g);
    coded[3 * k + 1 + w] = (uint8_t)rsc_step(s, u);
    if (w == 0) {
      coded[3 * k] = (uint8_t)u;
    }
  }
  if (k0 < K && k1 == K) {
    for (uint32_t j = 0; j < 3; j++) {
      const uint32_t x  = ((s >> 2) ^ (s >> 1)) & 1u;  // the feedback: the register input becomes 0
      const uint32_t pz = rsc_step(s, x);
      coded[3 * K + 6 * w + 2 * j]     = (uint8_t)x;
      coded[3 * K + 6 * w + 2 * j + 1] = (uint8_t)pz;
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(128) void enc_cb_kernel(const EncCb* __restrict__ cbs)
{
  const EncCb& b = cbs[blockIdx.x];
  __shared__ uint8_t  cbytes[768];
  __shared__ uint8_t  c[6144];
  __shared__ uint8_t  coded[3 * 6144 + 12];
  __shared__ PcccLds  sh;
  const uint32_t      K = b.K, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const uint32_t      nB = b.rlen / 8;

  // the block's info bytes: payload, then the TB CRC bytes
  const uint32_t tcrc = *b.tb_crc;
  for (uint32_t m = tid; m < nB; m += 128) {
    const uint32_t x = b.rp / 8 + m;
    cbytes[m]        = x < b.tb_bytes ? b.data[x] : (uint8_t)(tcrc >> (8 * (2 - (x - b.tb_bytes))));
  }
  __syncthreads();
  if (b.cb_crc && w == 0) {
    const uint32_t cc = wave_crc(nB, kCrc24B, [&](uint32_t i) { return (uint32_t)cbytes[i]; });
    if (lane < 3) {
      cbytes[nB + lane] = (uint8_t)(cc >> (8 * (2 - lane)));
    }
  }
  __syncthreads();
  for (uint32_t k = tid; k < K; k += 128) {
    c[k] = (cbytes[k >> 3] >> (7 - (k & 7))) & 1u;
  }
  __syncthreads();
  pccc_encode(c, K, b.f1, b.f2, coded, sh);

  // rate matching: the read-out table streamed 8 entries a thread ahead of the LDS gathers
  const uint16_t* __restrict__ fwd = b.fwd;
  uint8_t* __restrict__ eo         = b.e;
  const uint32_t N = b.N, E = b.E;
  for (uint32_t j0 = 0; j0 < E; j0 += 128 * 8) {
    uint16_t f[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const uint32_t j = j0 + u * 128 + tid;
      const uint32_t r = j - (j / N) * N;
      f[u]             = j < E ? fwd[r] : (uint16_t)0;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const uint32_t j = j0 + u * 128 + tid;
      if (j < E) {
        eo[j] = coded[f[u]];
      }
    }
  }
}

hipError_t enc_cb_launch(const EncCb* d_cbs, uint32_t ncb, hipStream_t stream)
{
  if (ncb == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(enc_cb_kernel, dim3(ncb), dim3(128), 0, stream, d_cbs);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void enc_pack_kernel(const EncTb* __restrict__ tbs)
{
  const EncTb&   t = tbs[blockIdx.y];
  const uint32_t m = blockIdx.x * 256 + threadIdx.x;
  if (8 * m >= t.nof_e_bits) {
    return;
  }
  uint32_t v = 0;
#pragma unroll
  for (uint32_t k = 0; k < 8; k++) {
    const uint32_t j = 8 * m + k;
    v |= (j < t.nof_e_bits ? (uint32_t)t.e_bits[j] & 1u : 0u) << (7 - k);
  }
  t.packed[m] = (uint8_t)v;
}

hipError_t enc_pack_launch(const EncTb* d_tbs, uint32_t ntb, uint32_t max_bytes, hipStream_t stream)
{
  if (ntb == 0 || max_bytes == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(enc_pack_kernel, dim3((max_bytes + 255) / 256, ntb), dim3(256), 0, stream, d_tbs);
  return hipGetLastError();
}

}  // namespace srsran_amd

namespace srsran_amd {

// srsran_tcod_encode (turbocoder.c:77-185) of one code block: K unpacked input bits (SRSRAN_TX_NULL = 100 marks
// filler bits: encoded as 0, passed through to the systematic output and blanking encoder 1's parity) -> 3 K + 12
// unpacked output bits
__global__ __launch_bounds__(128) void tcod_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint32_t K,
                                                   uint32_t f1, uint32_t f2)
{
  __shared__ uint8_t c[6144];
  __shared__ uint8_t coded[3 * 6144 + 12];
  __shared__ PcccLds sh;
  for (uint32_t k = threadIdx.x; k < K; k += 128) {
    const uint8_t x = in[k];
    c[k]            = x == kTxNull ? 0u : x;
  }
  __syncthreads();
  pccc_encode(c, K, f1, f2, coded, sh);
  for (uint32_t k = threadIdx.x; k < K; k += 128) {
    const uint8_t x = in[k];
    out[3 * k]      = x;
    out[3 * k + 1]  = x == kTxNull ? kTxNull : coded[3 * k + 1];
    out[3 * k + 2]  = coded[3 * k + 2];
  }
  for (uint32_t k = threadIdx.x; k < 12; k += 128) {
    out[3 * K + k] = coded[3 * K + k];
  }
}

hipError_t tcod_launch(const uint8_t* d_in, uint8_t* d_out, uint32_t K, uint32_t f1, uint32_t f2, hipStream_t stream)
{
  if (K == 0 || K > 6144) {
    return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(tcod_kernel, dim3(1), dim3(128), 0, stream, d_in, d_out, K, f1, f2);
  return hipGetLastError();
}

// srsran_rm_turbo_tx_lut (rm_turbo.c:345-388) of one code block, one workgroup: for rv 0 the circular buffer w
// (sub-block interleaving and bit collection, 3 K + 12 bits packed MSB first, no dummy bits) from the packed
// systematic (K + 4 bits) and parity (2 (K + 4) bits) streams through the reference's interleaver tables, into
// w_buff; otherwise w from w_buff.  Then out_len bits of w from r_ptr (wrapping) into output at bit w_offset: the
// bits before w_offset in its byte kept, those after the last bit kept -- or cleared when the reference's last
// srsran_bit_copy was byte-aligned (zero_tail, bit.c:685-698)
__global__ __launch_bounds__(256) void rm_tx_lut_kernel(RmTxLut a)
{
  extern __shared__ uint8_t w[];
  const uint32_t in_len = 3 * a.K + 12, nwb = (in_len + 7) / 8, nsys = a.K + 4;
  for (uint32_t b = threadIdx.x; b < nwb; b += 256) {
    uint8_t v = 0;
    if (a.rv == 0) {
#pragma unroll
      for (uint32_t j = 0; j < 8; j++) {
        const uint32_t pos = 8 * b + j;
        uint32_t       bit = 0;
        if (pos < nsys) {
          const uint32_t i = a.tsys[pos];
          bit              = (a.sys[i >> 3] >> (7 - (i & 7))) & 1u;
        } else if (pos < in_len) {
          const uint32_t i = a.tpar[pos - nsys];
          bit              = (a.par[i >> 3] >> (7 - (i & 7))) & 1u;
        }
        v |= (uint8_t)(bit << (7 - j));
      }
      a.w_buff[b] = v;
    } else {
      v = a.w_buff[b];
    }
    w[b] = v;
  }
  __syncthreads();
  if (a.out_len == 0) {
    return;
  }
  const uint32_t first = a.w_offset / 8, last = (a.w_offset + a.out_len - 1) / 8;
  for (uint32_t ob = first + threadIdx.x; ob <= last; ob += 256) {
    uint8_t v = a.output[ob];
#pragma unroll
    for (uint32_t j = 0; j < 8; j++) {
      const uint32_t pos = 8 * ob + j;
      const uint8_t  m   = (uint8_t)(0x80u >> j);
      if (pos >= a.w_offset && pos < a.w_offset + a.out_len) {
        uint32_t src = a.r_ptr + (pos - a.w_offset);
        src %= in_len;
        v = (uint8_t)((v & ~m) | (((w[src >> 3] >> (7 - (src & 7))) & 1u) ? m : 0u));
      } else if (pos >= a.w_offset + a.out_len && a.zero_tail) {
        v = (uint8_t)(v & ~m);
      }
    }
    a.output[ob] = v;
  }
}

hipError_t rm_tx_lut_launch(const RmTxLut& a, hipStream_t stream)
{
  const size_t lds = (3 * (size_t)a.K + 12 + 7) / 8;
  hipLaunchKernelGGL(rm_tx_lut_kernel, dim3(1), dim3(256), lds, stream, a);
  return hipGetLastError();
}

}  // namespace srsran_amd
