// srsran_4g_amd/csrc/sch_kernel.hip -- DL-SCH rate de-matching and TB assembly for CDNA4.
//
// rm_rx_kernel: the reference scatters E LLRs into the soft buffer
//   output[deinter[i % N]] += input[i]           (rm_turbo.c:440-447, AVX body 707-811)
// with a per-(K, rv, layout) permutation table.  Here the table is inverted once on
// the host, so every soft-buffer position gathers its own contributions:
//   sb[p] += e[inv[p]] + e[inv[p] + N] + ...      (all < E; int16 wrap, order-free)
// which gives coalesced soft-buffer reads/writes, no atomics and no write conflicts;
// the E-vector gather hits L2 (E <= ~20 KB per CB).
//
// tb_kernel: one workgroup per transport block performs the tail of decode_tb_cb and
// decode_tb (sch.c:458-573): payload assembly in CB order (later CBs overwrite the
// 3 CRC bytes earlier ones wrote, skipped CBs come from the soft buffer's saved copy),
// the CB CRC bookkeeping, saving of good CBs on failure, the TB CRC24A and the
// reset of the CB flags when the TB CRC fails.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc24_dev.h"
#include "sch_kernel.h"
#include "tdec_kernel.h"
#include "stage_timing.h"

namespace srsran_amd {

static constexpr int RM_THREADS    = 256;
static constexpr int RM_PER_THREAD = 16;  // positions per thread: 2 x 16-byte table loads, 16 gathers

__global__ __launch_bounds__(RM_THREADS) void rm_rx_kernel(const RmSlot* __restrict__ slots)
{
  const RmSlot   s = slots[blockIdx.y];
  const uint32_t p = (blockIdx.x * RM_THREADS + threadIdx.x) * RM_PER_THREAD;
  if (p >= s.len || (!s.overwrite && *s.skip)) {
    return;
  }
  // len is a multiple of 4 (3K+12 / 3K+108 with 8 | K); buffers are 8-byte aligned, so
  // work in 4-position (8-byte) groups
  const int ng = (int)min((uint32_t)RM_PER_THREAD, s.len - p) / 4;
  uint2     iv[RM_PER_THREAD / 4], v[RM_PER_THREAD / 4];
#pragma unroll
  for (int g = 0; g < RM_PER_THREAD / 4; g++) {
    if (g < ng) {
      iv[g] = *reinterpret_cast<const uint2*>(s.inv + p + 4 * g);
      v[g]  = s.overwrite ? make_uint2(0, 0) : *reinterpret_cast<const uint2*>(s.sb + p + 4 * g);
    }
  }
  short e0[RM_PER_THREAD];  // first contribution of every position, gathered together
#pragma unroll
  for (int g = 0; g < RM_PER_THREAD / 4; g++) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t idx = k == 0 ? (iv[g].x & 0xffffu) : k == 1 ? (iv[g].x >> 16) : k == 2 ? (iv[g].y & 0xffffu) : (iv[g].y >> 16);
      e0[4 * g + k]      = (g < ng && idx != 0xffffu && idx < s.E) ? s.e[idx] : (short)0;
    }
  }
#pragma unroll
  for (int g = 0; g < RM_PER_THREAD / 4; g++) {
    if (g < ng) {
      short acc[4] = {(short)(v[g].x & 0xffffu), (short)(v[g].x >> 16), (short)(v[g].y & 0xffffu), (short)(v[g].y >> 16)};
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t idx = k == 0 ? (iv[g].x & 0xffffu) : k == 1 ? (iv[g].x >> 16) : k == 2 ? (iv[g].y & 0xffffu) : (iv[g].y >> 16);
        acc[k] = (short)(acc[k] + e0[4 * g + k]);
        if (idx != 0xffffu) {  // repetitions past one period (E > N): rare
          for (uint32_t i = idx + s.N; i < s.E; i += s.N) {
            acc[k] = (short)(acc[k] + s.e[i]);
          }
        }
      }
      v[g].x = (uint32_t)(uint16_t)acc[0] | ((uint32_t)(uint16_t)acc[1] << 16);
      v[g].y = (uint32_t)(uint16_t)acc[2] | ((uint32_t)(uint16_t)acc[3] << 16);
      *reinterpret_cast<uint2*>(s.sb + p + 4 * g) = v[g];
    }
  }
}

static constexpr int TB_THREADS = 1024;
static constexpr int TB_WAVES   = TB_THREADS / 64;

// x^(8 * 2^k) mod CRC24A for k = 0..16, built at compile time.
constexpr uint32_t ce_clmul_mod24(uint32_t a, uint32_t b, uint32_t poly)
{
  uint64_t r = 0;
  for (int i = 0; i < 24; i++) {
    if ((b >> i) & 1u) {
      r ^= (uint64_t)a << i;
    }
  }
  for (int i = 46; i >= 24; i--) {
    if ((r >> i) & 1ull) {
      r ^= (uint64_t)poly << (i - 24);
    }
  }
  return (uint32_t)r;
}
struct XpTable {
  uint32_t v[17];
};
constexpr XpTable make_xp()
{
  XpTable  t{};
  uint32_t x = 0x100u;  // x^8
  for (int k = 0; k < 17; k++) {
    t.v[k] = x;
    x      = ce_clmul_mod24(x, x, LTE_CRC24A);
  }
  return t;
}
__constant__ XpTable kXpA = make_xp();

// x^(8m) mod CRC24A
__device__ __forceinline__ uint32_t xpow8(uint32_t m)
{
  uint32_t r = 1;
  for (int k = 0; m; k++, m >>= 1) {
    if (m & 1u) {
      r = clmul24(r, kXpA.v[k], LTE_CRC24A);
    }
  }
  return r;
}

// Zero (as srsran_softbuffer_rx_reset_cb does) CB soft buffers [sb0, n), saved payloads
// [0, n) except those in `keep`, and CB flags [f0, max_cb).
__device__ void reset_range(const SchTb& t, uint32_t sb0, uint32_t n, uint32_t f0, uint32_t keep)
{
  const int tid = threadIdx.x;
  if (sb0 < n) {  // soft buffers are 8-byte aligned, sb_stride a multiple of 4
    uint2*         p   = reinterpret_cast<uint2*>(t.sbuf + (size_t)sb0 * t.sb_stride);
    const uint32_t n64 = (n - sb0) * t.sb_stride / 4;
    for (uint32_t i = tid; i < n64; i += TB_THREADS) {
      p[i] = make_uint2(0, 0);
    }
  }
  if (keep == 0) {  // one contiguous range
    const uint32_t nb = n * t.saved_stride;
    for (uint32_t i = tid; i < nb; i += TB_THREADS) {
      t.saved[i] = 0;
    }
  } else {
    for (uint32_t c = 0; c < n; c++) {
      if (c < 32 && ((keep >> c) & 1u)) {
        continue;
      }
      for (uint32_t i = tid; i < t.saved_stride; i += TB_THREADS) {
        t.saved[(size_t)c * t.saved_stride + i] = 0;
      }
    }
  }
  for (uint32_t c = f0 + tid; c < t.max_cb; c += TB_THREADS) {
    t.cb_crc[c] = 0;
  }
}

__global__ __launch_bounds__(TB_THREADS) void tb_kernel(const SchTb* __restrict__ tbs)
{
  const SchTb t   = tbs[blockIdx.x];
  const int   tid = threadIdx.x;
  if (t.status != 1) {
    if (t.new_data && t.cb_crc) {  // the reset still happened (softbuffer.c:146-169)
      reset_range(t, 0, t.nof_cb_reset, 0, 0);
      if (tid == 0) {
        *t.tb_crc = 0;
      }
    }
    if (tid == 0) {
      *t.result = t.status;
      *t.avg    = 0.0f;
    }
    return;
  }
  __shared__ uint8_t        pay[SCH_MAX_CB * SCH_SLOT_BYTES];  // the TB payload as decode_tb leaves it
  __shared__ uint32_t       start[SCH_MAX_CB], len[SCH_MAX_CB], rlen8[SCH_MAX_CB];
  __shared__ const uint8_t* src[SCH_MAX_CB];
  __shared__ uint32_t       okf[SCH_MAX_CB];
  __shared__ uint32_t       noi_sum, end_max, wave_crc[TB_WAVES];

  const uint32_t C = t.C;
  if (tid == 0) {
    noi_sum = 0;
    end_max = 0;
  }
  __syncthreads();
  if (tid < (int)C) {
    const uint32_t K    = tid < (int)t.C1 ? t.K1 : t.K2;
    const uint32_t rlen = C == 1 ? K : K - 24;
    const uint32_t slot = t.slot0 + tid;
    const uint32_t n    = t.noi[slot];
    const bool     skip = n == 0;  // CB CRC was already OK: copy the saved payload (sch.c:476-480)
    start[tid]          = tid * rlen / 8;
    rlen8[tid]          = rlen / 8;
    len[tid]            = skip ? rlen / 8 : K / 8;
    src[tid]            = skip ? t.saved + (size_t)tid * t.saved_stride : t.cbout + (size_t)slot * SCH_SLOT_BYTES;
    okf[tid]            = skip ? 1u : t.crc_ok[slot];
    atomicAdd(&noi_sum, n);
    atomicMax(&end_max, start[tid] + len[tid]);
  }
  __syncthreads();
  bool all_ok = true;
  for (uint32_t c = 0; c < C; c++) {
    all_ok = all_ok && okf[c];
  }
  // payload: byte p comes from the last CB (in decode order) whose write covered it
  // (sch.c:425-431: each CB writes K/8 bytes at cb*rlen/8, over the previous CB's CRC).
  // Four independent global loads per thread in flight.
  const uint32_t end     = end_max;
  const bool     uniform = t.C1 == C || t.K1 == t.K2;  // one rlen: owner = min(p / rlen8, C-1)
  const uint32_t r8      = rlen8[0];
  for (uint32_t p0 = tid; p0 < end; p0 += 4 * TB_THREADS) {
    uint8_t v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t p = p0 + u * TB_THREADS;
      v[u]             = 0;
      if (p < end) {
        int c;
        if (uniform) {
          c = (int)min(p / r8, C - 1);
        } else {
          c = (int)C - 1;
          while (c > 0 && !(p >= start[c] && p < start[c] + len[c])) {
            c--;
          }
        }
        v[u] = src[c][p - start[c]];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t p = p0 + u * TB_THREADS;
      if (p < end) {
        pay[p] = v[u];
      }
    }
  }
  __syncthreads();
  for (uint32_t p = tid; p < end; p += TB_THREADS) {
    t.data[p] = pay[p];
  }

  bool     tb_fail = false;
  uint32_t keep    = 0;
  if (!all_ok) {
    // keep the good CBs for the next retransmission (sch.c:465-474)
    for (uint32_t c = 0; c < C; c++) {
      if (okf[c]) {
        keep |= 1u << c;
        for (uint32_t i = tid; i < rlen8[c]; i += TB_THREADS) {
          t.saved[(size_t)c * t.saved_stride + i] = pay[start[c] + i];
        }
      }
    }
  } else if (C > 1) {
    // TB CRC24A over tbs + 24 bits (srsran_crc_match_byte, sch.c:560): 256 equal chunks
    // aligned to the END of the message (leading zero bytes do not change a zero-init CRC),
    // then a shuffle tree: crc(A|B) = crc(A) * x^(8|B|) + crc(B).
    const int      nbytes = (int)((t.tbs + 24) / 8);
    const int      per    = (nbytes + TB_THREADS - 1) / TB_THREADS;
    const int      b1     = nbytes - (TB_THREADS - 1 - tid) * per;
    const int      b0     = b1 - per;
    uint32_t       crc    = 0;
    for (int b = max(b0, 0); b < b1; b++) {
      crc = crc24_byte(crc, b >= 0 ? pay[b] : 0u, LTE_CRC24A);
    }
    uint32_t M = xpow8((uint32_t)per);  // multiplier for a span of 2^l chunks, l = level
    const int lane = tid & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t other = (uint32_t)__shfl_xor((int)crc, off, 64);
      crc = (lane & off) ? (clmul24(other, M, LTE_CRC24A) ^ crc) : (clmul24(crc, M, LTE_CRC24A) ^ other);
      M   = clmul24(M, M, LTE_CRC24A);
    }
    if (lane == 0) {
      wave_crc[tid >> 6] = crc;
    }
    __syncthreads();
    if (tid < 64) {  // M = x^(8 * per * 64): one wave's span; same tree over the wave CRCs
      crc = lane < TB_WAVES ? wave_crc[lane] : 0u;
#pragma unroll
      for (int off = 1; off < TB_WAVES; off <<= 1) {
        const uint32_t other = (uint32_t)__shfl_xor((int)crc, off, 64);
        crc = (lane & off) ? (clmul24(other, M, LTE_CRC24A) ^ crc) : (clmul24(crc, M, LTE_CRC24A) ^ other);
        M   = clmul24(M, M, LTE_CRC24A);
      }
      if (lane == 0) {
        wave_crc[0] = crc;
      }
    }
    __syncthreads();
    tb_fail = wave_crc[0] != 0;  // srsran_softbuffer_rx_reset_cb_crc (sch.c:567)
  }
  if (tid < (int)C) {
    t.cb_crc[tid] = (okf[tid] && !tb_fail) ? 1 : 0;
  }
  if (t.new_data) {
    // what reset_tbs cleared and this decode did not rewrite: flags past C, soft
    // buffers past C, saved payloads that were not saved just now
    reset_range(t, C, t.nof_cb_reset, C, keep);
  }
  if (tid == 0) {
    *t.tb_crc = all_ok ? 1 : 0;
    *t.result = (all_ok && !tb_fail) ? 0 : -1;
    *t.avg    = (float)noi_sum / (float)C;
  }
}

hipError_t rm_rx_launch(const RmSlot* d_slots, uint32_t nslots, uint32_t max_len, hipStream_t stream)
{
  StageScope timing_scope(ST_RM, stream);
  const uint32_t per_block = RM_THREADS * RM_PER_THREAD;
  const uint32_t gx        = (max_len + per_block - 1) / per_block;
  for (uint32_t s0 = 0; s0 < nslots; s0 += 65535) {
    const uint32_t n = nslots - s0 < 65535 ? nslots - s0 : 65535;
    hipLaunchKernelGGL(rm_rx_kernel, dim3(gx, n), dim3(RM_THREADS), 0, stream, d_slots + s0);
  }
  return hipGetLastError();
}

hipError_t tb_launch(const SchTb* d_tbs, uint32_t ntb, hipStream_t stream)
{
  StageScope timing_scope(ST_TB, stream);
  if (ntb == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(tb_kernel, dim3(ntb), dim3(TB_THREADS), 0, stream, d_tbs);
  return hipGetLastError();
}

}  // namespace srsran_amd
