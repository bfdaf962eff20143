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

namespace srsran_amd {

static constexpr int RM_THREADS = 256;
static constexpr int RM_PER_THREAD = 4;

__global__ __launch_bounds__(RM_THREADS) void rm_rx_kernel(const RmSlot* __restrict__ slots)
{
  const RmSlot s  = slots[blockIdx.y];
  const uint32_t p = (blockIdx.x * RM_THREADS + threadIdx.x) * RM_PER_THREAD;
  if (p >= s.len || (!s.overwrite && *s.skip)) {
    return;
  }
  // len is a multiple of 4 (3K+12 / 3K+108 with 8 | K) and buffers are 8-byte aligned
  const uint2 iv = *reinterpret_cast<const uint2*>(s.inv + p);
  uint2       v  = *reinterpret_cast<const uint2*>(s.sb + p);
  const uint32_t idx[4] = {iv.x & 0xffffu, iv.x >> 16, iv.y & 0xffffu, iv.y >> 16};
  if (s.overwrite) {
    v = make_uint2(0, 0);
  }
  short acc[4] = {(short)(v.x & 0xffffu), (short)(v.x >> 16), (short)(v.y & 0xffffu), (short)(v.y >> 16)};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (idx[k] != 0xffffu) {
      for (uint32_t i = idx[k]; i < s.E; i += s.N) {
        acc[k] = (short)(acc[k] + s.e[i]);
      }
    }
  }
  v.x = (uint32_t)(uint16_t)acc[0] | ((uint32_t)(uint16_t)acc[1] << 16);
  v.y = (uint32_t)(uint16_t)acc[2] | ((uint32_t)(uint16_t)acc[3] << 16);
  *reinterpret_cast<uint2*>(s.sb + p) = v;
}

static constexpr int TB_THREADS = 256;

// Zero (as srsran_softbuffer_rx_reset_cb does) CB soft buffers [sb0, n), saved payloads
// [0, n) except those in *keep, and CB flags [f0, max_cb).
__device__ void reset_range(const SchTb& t, uint32_t sb0, uint32_t n, uint32_t f0, const uint32_t* keep)
{
  const int tid = threadIdx.x;
  for (uint32_t c = sb0; c < n; c++) {
    for (uint32_t i = tid; i < t.sb_stride; i += TB_THREADS) {
      t.sbuf[(size_t)c * t.sb_stride + i] = 0;
    }
  }
  for (uint32_t c = 0; c < n; c++) {
    if (keep && c < 32 && ((*keep >> c) & 1u)) {
      continue;
    }
    for (uint32_t i = tid; i < t.saved_stride; i += TB_THREADS) {
      t.saved[(size_t)c * t.saved_stride + i] = 0;
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
      reset_range(t, 0, t.nof_cb_reset, 0, nullptr);
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
  __shared__ uint32_t start[SCH_MAX_CB], len[SCH_MAX_CB], rlen8[SCH_MAX_CB];
  __shared__ const uint8_t* src[SCH_MAX_CB];
  __shared__ uint32_t okf[SCH_MAX_CB];
  __shared__ uint32_t noi_sum, end_max, crc_part[TB_THREADS / 64];
  __shared__ uint32_t xp[17];  // x^(8*2^k) mod CRC24A

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
  const uint32_t end = end_max;
  for (uint32_t p = tid; p < end; p += TB_THREADS) {
    for (int c = (int)C - 1; c >= 0; c--) {
      if (p >= start[c] && p < start[c] + len[c]) {
        t.data[p] = src[c][p - start[c]];
        break;
      }
    }
  }
  __syncthreads();

  bool tb_fail = false;
  if (!all_ok) {
    // keep the good CBs for the next retransmission (sch.c:465-474)
    for (uint32_t c = 0; c < C; c++) {
      if (okf[c]) {
        for (uint32_t i = tid; i < rlen8[c]; i += TB_THREADS) {
          t.saved[(size_t)c * t.saved_stride + i] = t.data[start[c] + i];
        }
      }
    }
  } else if (C > 1) {
    // TB CRC24A over tbs + 24 bits (srsran_crc_match_byte, sch.c:560)
    if (tid == 0) {
      uint32_t v = 0x100u;  // x^8
      for (int k = 0; k < 17; k++) {
        xp[k] = v;
        v     = clmul_mod24(v, v, LTE_CRC24A);
      }
    }
    __syncthreads();
    const uint32_t nbytes = (t.tbs + 24) / 8;
    const uint32_t per    = (nbytes + TB_THREADS - 1) / TB_THREADS;
    const uint32_t b0     = min(nbytes, tid * per);
    const uint32_t b1     = min(nbytes, b0 + per);
    uint32_t       crc    = 0;
    for (uint32_t b = b0; b < b1; b++) {
      crc = crc24_byte(crc, t.data[b], LTE_CRC24A);
    }
    uint32_t after = nbytes - b1;
    for (int k = 0; after; k++, after >>= 1) {
      if (after & 1u) {
        crc = clmul_mod24(crc, xp[k], LTE_CRC24A);
      }
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      crc ^= (uint32_t)__shfl_xor((int)crc, off, 64);
    }
    if ((tid & 63) == 0) {
      crc_part[tid >> 6] = crc;
    }
    __syncthreads();
    uint32_t total = 0;
    for (int w = 0; w < TB_THREADS / 64; w++) {
      total ^= crc_part[w];
    }
    tb_fail = total != 0;  // srsran_softbuffer_rx_reset_cb_crc (sch.c:567)
  }
  if (tid < (int)C) {
    t.cb_crc[tid] = (okf[tid] && !tb_fail) ? 1 : 0;
  }
  if (t.new_data) {
    // what reset_tbs cleared and this decode did not rewrite: flags past C, soft
    // buffers past C, saved payloads that were not saved just now
    const uint32_t saved_now = all_ok ? 0u : 0xffffffffu;
    uint32_t       mask      = 0;
    for (uint32_t c = 0; c < C; c++) {
      mask |= (okf[c] && saved_now) ? (1u << c) : 0u;
    }
    reset_range(t, C, t.nof_cb_reset, C, &mask);
  }
  if (tid == 0) {
    *t.tb_crc = all_ok ? 1 : 0;
    *t.result = (all_ok && !tb_fail) ? 0 : -1;
    *t.avg    = (float)noi_sum / (float)C;
  }
}

hipError_t rm_rx_launch(const RmSlot* d_slots, uint32_t nslots, uint32_t max_len, hipStream_t stream)
{
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
  if (ntb == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(tb_kernel, dim3(ntb), dim3(TB_THREADS), 0, stream, d_tbs);
  return hipGetLastError();
}

}  // namespace srsran_amd
