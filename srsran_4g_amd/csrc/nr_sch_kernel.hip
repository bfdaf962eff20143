// srsran_4g_amd/csrc/nr_sch_kernel.hip -- NR SCH receive kernels for CDNA4 (gfx950).
//
// nr_rm_kernel: srsran_ldpc_rm_rx_c (ldpc_rm.c:297-338, 396-410, 675-706) for every code block of
//   a batch, one workgroup per block.  The reference de-interleaves (tmp[i cols + j] = e[j Qm + i]),
//   walks the circular buffer from k0 skipping the filler range, and adds each LLR into the soft
//   buffer position it lands on, clipping to +-63 after every add; filler positions get 127.  Here
//   every soft-buffer position gathers its own contributions instead: position p is the rank-th
//   non-filler position after k0, so it receives LLRs i = rank, rank + L, rank + 2L, ... (L = Ncb
//   minus the fillers inside it), added in that order with the same clipping -- the sequential
//   result, without atomics.  The block's LLR offset in the TB reproduces sch_nr.c: blocks whose CRC
//   already passed are skipped and do not advance the read pointer (sch_nr.c:633-636 vs 682).
//   With `fresh` (new data) the TB's blocks behave as after srsran_softbuffer_rx_reset_cb (softbuffer.c:
//   150-169) restricted to what the TB can observe: no block is skipped, accumulation starts from zero
//   over the whole circular buffer, and the block's CRC flag and saved payload are cleared.
// nr_tb_kernel: sch_nr.c:692-748 -- if every block passed, concatenate the blocks' packed bits into
//   the payload and (C > 1) check the TB CRC over the payload against the CRC bits the last block
//   carries; chunk CRCs are shifted into place with x^(8 bytes after) mod P and XOR-combined.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nr_sch_kernel.h"
#include "stage_timing.h"

namespace srsran_amd {

__device__ __forceinline__ uint32_t cb_E(const NrRmCb& d, uint32_t r) { return r <= d.jthr ? d.E0 : d.E1; }

// |[a0, a1) ∩ [b0, b1)|
__device__ __forceinline__ uint32_t overlap(uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1)
{
  const uint32_t lo = max(a0, b0), hi = min(a1, b1);
  return hi > lo ? hi - lo : 0u;
}

__global__ __launch_bounds__(256) void nr_rm_kernel(const NrRmCb* __restrict__ cbs)
{
  const NrRmCb d = cbs[blockIdx.x];
  if (d.fresh) {
    for (uint32_t b = threadIdx.x; b < d.data_bytes; b += blockDim.x) {
      d.data[b] = 0;
    }
    if (threadIdx.x == 0) {
      d.flags[d.r] = 0;  // read by no other block of a fresh TB
    }
  } else if (d.flags[d.r]) {
    return;  // already decoded: the reference skips the block (and its rate de-matching)
  }
  uint32_t off = 0;  // LLR read offset of this block in the TB
  for (uint32_t q = 0; q < d.r; ++q) {
    off += (!d.fresh && d.flags[q]) ? 0u : cb_E(d, q);
  }
  const uint32_t E    = cb_E(d, d.r);
  const uint32_t cols = E / d.Qm;
  const int8_t*  e    = d.e + off;
  const uint32_t Ncb  = d.Ncb;
  const uint32_t fi = min(d.ini, Ncb), fe = min(d.end, Ncb);  // filler positions inside the circle
  const uint32_t L  = Ncb - (fe - fi);
  // de-interleaver: the i-th selected bit is e[(i mod cols) Qm + i / cols]
  const uint64_t inv = ((1ull << 40) + cols - 1) / cols;  // i / cols exact for i, cols < 2^20
  auto           div = [&](uint32_t i) { return (uint32_t)(((uint64_t)i * inv) >> 40); };
  // rank of a non-filler position: its distance from k0 along the circle, minus the fillers passed
  auto rank_of = [&](uint32_t p) {
    const uint32_t dist = p >= d.k0 ? p - d.k0 : p + Ncb - d.k0;
    uint32_t       nf;
    if (d.k0 + dist <= Ncb) {
      nf = overlap(d.k0, d.k0 + dist, fi, fe);
    } else {
      nf = overlap(d.k0, Ncb, fi, fe) + overlap(0, d.k0 + dist - Ncb, fi, fe);
    }
    return dist - nf;
  };
  // one position, any case (region boundaries, the tail, repetitions when E > L)
  auto one = [&](uint32_t p) {
    if (p >= d.ini && p < d.end) {
      d.buf[p] = 127;  // filler bit: infinity8 (ldpc_rm.c:327-329)
      return;
    }
    const uint32_t rank = rank_of(p);
    if (rank >= E) {
      if (d.fresh) {
        d.buf[p] = 0;
      }
      return;
    }
    int acc = d.fresh ? 0 : (int)d.buf[p];
    for (uint32_t i = rank; i < E; i += L) {  // in order, clipped after every add
      const uint32_t j = div(i);
      acc              = min(max(acc + (int)e[(i - j * cols) * d.Qm + j], -63), 63);
    }
    d.buf[p] = (int8_t)acc;
  };
  if (E <= L) {
    // Every position receives at most one LLR.  Pass 1 writes what no LLR reaches (fillers, and on
    // new data zeros); pass 2 gives each thread a de-interleaver column m: its Qm LLRs
    // e[m Qm .. m Qm + Qm) are contiguous, and rank j cols + m lands on position pos(rank) -- for a
    // fixed row j the lanes' positions are consecutive, so both the loads and the stores coalesce.
    uint32_t* b4 = reinterpret_cast<uint32_t*>(d.buf);  // soft buffers are 8-byte aligned
    for (uint32_t q = threadIdx.x; q < Ncb / 4; q += blockDim.x) {
      const uint32_t p0 = 4 * q;
      if (!d.fresh && (p0 + 4 <= fi || p0 >= fe)) {
        continue;  // no filler in this dword
      }
      uint32_t w = 0;
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) {
        w |= (p0 + k >= fi && p0 + k < fe ? 0x7Fu : 0u) << (8 * k);  // filler bits: infinity8 (ldpc_rm.c:327-329)
      }
      if (d.fresh) {
        b4[q] = w;
      } else {
        for (uint32_t k = 0; k < 4; ++k) {
          if (p0 + k >= fi && p0 + k < fe) {
            d.buf[p0 + k] = 127;
          }
        }
      }
    }
    for (uint32_t p = 4 * (Ncb / 4) + threadIdx.x; p < Ncb; p += blockDim.x) {
      if (p >= fi && p < fe) {
        d.buf[p] = 127;
      } else if (d.fresh) {
        d.buf[p] = 0;
      }
    }
    __syncthreads();
    // non-filler positions in circle order from k0: lap 1 runs k0 .. Ncb - 1, lap 2 runs 0 .. k0 - 1
    const uint32_t a1   = d.k0 < fi ? fi - d.k0 : 0u;  // lap 1 before the fillers
    const uint32_t s1   = max(d.k0, fe);               // lap 1 after them
    const uint32_t lap1 = a1 + (Ncb > s1 ? Ncb - s1 : 0u);
    const uint32_t b2   = min(fi, d.k0);               // lap 2 before the fillers
    auto           pos  = [&](uint32_t i) -> uint32_t {
      if (i < lap1) {
        return i < a1 ? d.k0 + i : s1 + (i - a1);
      }
      const uint32_t i2 = i - lap1;
      return i2 < b2 ? i2 : fe + (i2 - b2);
    };
    for (uint32_t m = threadIdx.x; m < cols; m += blockDim.x) {
      int x[8];
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) {
        x[j] = j < d.Qm ? (int)e[m * d.Qm + j] : 0;
      }
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) {
        if (j < d.Qm) {
          const uint32_t p = pos(j * cols + m);
          const int      v = d.fresh ? 0 : (int)d.buf[p];
          d.buf[p]         = (int8_t)min(max(v + x[j], -63), 63);
        }
      }
    }
    return;
  }
  // E > L (repetition): every position gathers its contributions in the reference's order (one())
  for (uint32_t p = threadIdx.x; p < Ncb; p += blockDim.x) {
    one(p);
  }
}

// a * b mod P, P of degree `order` <= 24 given with its x^order bit, a, b < 2^order (Horner over
// the 24 low bits of b: leading zero bits leave r = 0)
__host__ __device__ constexpr uint32_t mulmod(uint32_t a, uint32_t b, uint32_t poly, int order)
{
  uint32_t r = 0;
#pragma unroll
  for (int i = 23; i >= 0; i--) {
    r = (r << 1) ^ (((b >> i) & 1u) ? a : 0u);
    r ^= ((r >> order) & 1u) ? poly : 0u;
  }
  return r;
}

// Shift factors of the TB CRCs ([0] CRC24A, [1] CRC16, phy_common.h:72-74): thread[t] = x^(8 16 t)
// and slice[s] = x^(8 NR_TB_SLICE s) mod P -- the bytes after a thread's chunk inside its slice and
// after the slice
struct TbCrcShift {
  uint32_t thread[2][NR_TB_THREADS];
  uint32_t slice[2][16];
  constexpr TbCrcShift() : thread(), slice()
  {
    const uint32_t polys[2] = {0x1864CFBu, 0x11021u};
    const int      ords[2]  = {24, 16};
    for (int t = 0; t < 2; t++) {
      uint32_t x128 = 1u << 8;  // x^8 -> x^128
      for (int k = 0; k < 4; k++) {
        x128 = mulmod(x128, x128, polys[t], ords[t]);
      }
      thread[t][0] = 1u;
      for (uint32_t i = 1; i < NR_TB_THREADS; i++) {
        thread[t][i] = mulmod(thread[t][i - 1], x128, polys[t], ords[t]);
      }
      const uint32_t xs = mulmod(thread[t][NR_TB_THREADS - 1], x128, polys[t], ords[t]);  // x^(8 16 256)
      slice[t][0]       = 1u;
      for (int i = 1; i < 16; i++) {
        slice[t][i] = mulmod(slice[t][i - 1], xs, polys[t], ords[t]);
      }
    }
  }
};
static_assert(NR_TB_SLICE == 16 * NR_TB_THREADS, "slice = threads x 16 bytes");
__constant__ TbCrcShift c_tb_shift = TbCrcShift();

// Grid (TB, slice).  Every slice checks the blocks' flags itself.  Counted from the end of the payload,
// thread t of slice s owns the 16 bytes that end 16 t + NR_TB_SLICE s bytes before it: it copies them
// from the blocks' saved payloads and folds their CRC, times x^(8 16 t) (a constexpr table), into the
// slice's sum, which thread 0 multiplies by x^(8 NR_TB_SLICE s) into the TB's accumulator.  The last
// slice to finish compares it with the CRC bits the last block carries and clears the scratch.
__global__ __launch_bounds__(NR_TB_THREADS) void nr_tb_kernel(const NrTb* __restrict__ tbs)
{
  __shared__ uint32_t s_tab[256];
  __shared__ uint32_t s_ok, s_iters, s_crc, s_last;
  const NrTb     d     = tbs[blockIdx.x];
  const uint32_t slice = blockIdx.y;
  if (threadIdx.x == 0) {
    s_ok    = 0;
    s_iters = 0;
    s_crc   = 0;
  }
  __syncthreads();
  for (uint32_t r = threadIdx.x; r < d.C; r += blockDim.x) {
    atomicAdd(&s_ok, d.flags[r] ? 1u : 0u);
    atomicAdd(&s_iters, (uint32_t)d.iters[r]);
  }
  __syncthreads();
  const bool all_ok = s_ok == d.C;
  if (threadIdx.x == 0 && slice == 0) {
    *d.avg_out = d.C ? (float)s_iters / (float)d.C : __builtin_nanf("");
    if (!all_ok || d.C == 1) {
      *d.crc_out = all_ok ? 1 : 0;  // C == 1: the block's CRC was the TB CRC (sch_nr.c:729-731)
    }
  }
  if (!all_ok) {
    return;  // not all blocks decoded: no TB union, crc false (sch_nr.c:694-696)
  }
  // concatenation: block r contributes its first cb_bytes bytes (the last one cb_bytes_last)
  const uint32_t cb_bytes      = (d.Kp - d.L_cb) / 8;
  const uint32_t cb_bytes_last = (d.Kp - d.L_cb - d.L_tb) / 8;
  const uint32_t nbytes        = (d.C - 1) * cb_bytes + cb_bytes_last;
  const uint32_t nslices       = (nbytes + NR_TB_SLICE - 1) / NR_TB_SLICE;
  if (slice >= nslices) {
    return;
  }
  const bool     tbcrc = d.C > 1;
  const uint32_t poly  = d.L_tb == 24 ? 0x1864CFBu : 0x11021u;  // CRC24A / CRC16 (sch_nr.c:596)
  const int      order = (int)d.L_tb;
  const uint32_t mask  = (1u << order) - 1u;
  if (tbcrc) {
    for (uint32_t v = threadIdx.x; v < 256; v += blockDim.x) {
      uint32_t c = v << (order - 8);
#pragma unroll
      for (int k = 0; k < 8; k++) {
        c = (c & (1u << (order - 1))) ? ((c << 1) ^ poly) : (c << 1);
      }
      s_tab[v] = c & mask;
    }
  }
  // chunks are counted from the end of the payload: thread t of slice s holds the 16 bytes that end
  // 16 t + NR_TB_SLICE s bytes before it (the first chunk of the payload may be shorter)
  const uint32_t back = slice * NR_TB_SLICE + threadIdx.x * NR_TB_BYTES;  // bytes after the chunk
  const uint32_t b1   = back < nbytes ? nbytes - back : 0u;
  const uint32_t b0   = b1 > NR_TB_BYTES ? b1 - NR_TB_BYTES : 0u;
  uint8_t        v[NR_TB_BYTES];
  if (b0 < b1) {
    uint32_t r = min(b0 / cb_bytes, d.C - 1), o = b0 - r * cb_bytes;
#pragma unroll
    for (uint32_t k = 0; k < NR_TB_BYTES; ++k) {  // independent loads, issued back to back
      const bool in = k < b1 - b0;
      v[k]          = in ? d.data[(size_t)r * d.data_stride + o] : 0;
      if (in && ++o == cb_bytes && r + 1 < d.C) {
        o = 0;
        ++r;
      }
    }
#pragma unroll
    for (uint32_t k = 0; k < NR_TB_BYTES; ++k) {
      if (k < b1 - b0) {
        d.payload[b0 + k] = v[k];
      }
    }
  }
  if (!tbcrc) {
    return;
  }
  __syncthreads();  // tables
  if (b0 < b1) {
    uint32_t crc = 0;  // srsran_crc_checksum_byte: MSB first, zero init
#pragma unroll
    for (uint32_t k = 0; k < NR_TB_BYTES; ++k) {  // fixed trip count: v[] stays in registers
      if (k < b1 - b0) {
        crc = ((crc << 8) & mask) ^ s_tab[((crc >> (order - 8)) ^ v[k]) & 0xFFu];
      }
    }
    // * x^(8 16 t): the bytes after the chunk inside the slice
    crc = mulmod(crc, c_tb_shift.thread[order == 24 ? 0 : 1][threadIdx.x], poly, order);
    atomicXor(&s_crc, crc & mask);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    // * x^(8 NR_TB_SLICE s): the bytes after the slice
    atomicXor(&d.scratch[0], mulmod(s_crc, c_tb_shift.slice[order == 24 ? 0 : 1][slice], poly, order) & mask);
    __threadfence();
    s_last = atomicAdd(&d.scratch[1], 1u) == nslices - 1;
  }
  __syncthreads();
  if (s_last && threadIdx.x == 0) {
    __threadfence();
    const uint32_t acc = atomicExch(&d.scratch[0], 0u);
    d.scratch[1]       = 0;
    // the TB CRC bits follow the data in the last block (sch_nr.c:711-717)
    const uint8_t* t   = d.data + (size_t)(d.C - 1) * d.data_stride + cb_bytes_last;
    uint32_t       chk = 0;
    for (uint32_t b = 0; b < d.L_tb / 8; ++b) {
      chk = (chk << 8) | t[b];
    }
    *d.crc_out = acc == chk ? 1 : 0;
  }
}

hipError_t nr_rm_launch(const NrRmCb* d_cbs, uint32_t ncb, hipStream_t stream)
{
  if (ncb == 0) {
    return hipSuccess;
  }
  StageScope timing_scope(ST_NR_RM, stream);
  hipLaunchKernelGGL(nr_rm_kernel, dim3(ncb), dim3(256), 0, stream, d_cbs);
  return hipGetLastError();
}

hipError_t nr_tb_launch(const NrTb* d_tbs, uint32_t ntb, uint32_t slices, hipStream_t stream)
{
  if (ntb == 0) {
    return hipSuccess;
  }
  StageScope timing_scope(ST_NR_TB, stream);
  hipLaunchKernelGGL(nr_tb_kernel, dim3(ntb, slices > 0 ? slices : 1), dim3(NR_TB_THREADS), 0, stream, d_tbs);
  return hipGetLastError();
}

}  // namespace srsran_amd
