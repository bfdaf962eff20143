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
// tb_kernel performs the tail of decode_tb_cb and decode_tb
// (sch.c:458-573): payload assembly in CB order (later CBs overwrite the 3 CRC bytes earlier
// ones wrote, skipped CBs come from the soft buffer's saved copy) with the TB CRC24A of each
// 1 KB chunk, then per TB the CB CRC bookkeeping, saving of good CBs on failure, the TB CRC
// decision and the reset of the CB flags when it fails.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "crc24_dev.h"
#include "gmem.h"
#include "sch_kernel.h"
#include "tdec_kernel.h"
#include "stage_copy.h"
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

// rm_rx_lds_kernel: one workgroup per code block.  The CB's E LLRs are staged in LDS with
// coalesced loads, then every soft-buffer position gathers its contributions from LDS
// (4 positions per thread per pass: 8-byte table and soft-buffer accesses, coalesced).
static constexpr int RM_LDS_THREADS = 512;

// one 4-position group: the soft-buffer values v plus every contribution es[idx + j N] of each position
__device__ __forceinline__ uint2 rm_group(uint2 iv, uint2 v, const short* es, uint32_t E, uint32_t N)
{
  const uint32_t idx[4] = {iv.x & 0xffffu, iv.x >> 16, iv.y & 0xffffu, iv.y >> 16};
  int16_t        acc[4] = {(int16_t)(v.x & 0xffffu), (int16_t)(v.x >> 16), (int16_t)(v.y & 0xffffu),
                           (int16_t)(v.y >> 16)};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (idx[k] != 0xffffu) {
      int16_t a = acc[k];
      for (uint32_t i = idx[k]; i < E; i += N) {  // one period, plus repetitions when E > N
        a = (int16_t)(a + es[i]);
      }
      acc[k] = a;
    }
  }
  return make_uint2((uint32_t)(uint16_t)acc[0] | ((uint32_t)(uint16_t)acc[1] << 16),
                    (uint32_t)(uint16_t)acc[2] | ((uint32_t)(uint16_t)acc[3] << 16));
}

// the same when E <= N (no repetition: a position has at most one contribution, es[idx] when idx < E -- the
// first transmission of a C3 code block): branch-free, the four positions' sums as two packed 16-bit adds (wrap)
__device__ __forceinline__ uint2 rm_group1(uint2 iv, uint2 v, const short* es, uint32_t E)
{
  const uint32_t idx[4] = {iv.x & 0xffffu, iv.x >> 16, iv.y & 0xffffu, iv.y >> 16};
  uint32_t       c[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t e = (uint32_t)(uint16_t)es[min(idx[k], E - 1)];  // an unused slot (0xffff) reads a valid LLR
    c[k]             = idx[k] < E ? e : 0u;
  }
  const uint32_t lo = c[0] | (c[1] << 16), hi = c[2] | (c[3] << 16);
  typedef short  v2s __attribute__((ext_vector_type(2)));
  const v2s      a  = __builtin_bit_cast(v2s, v.x) + __builtin_bit_cast(v2s, lo);
  const v2s      b  = __builtin_bit_cast(v2s, v.y) + __builtin_bit_cast(v2s, hi);
  return make_uint2(__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b));
}

__global__ __launch_bounds__(RM_LDS_THREADS) void rm_rx_lds_kernel(const RmSlot* __restrict__ slots)
{
  // E LLRs staged as 16-byte words from the aligned address at or below e (es = the E values from `sh` on;
  // the words never cross a page, so reading the partial first / last word stays inside mapped memory).  Dynamic
  // LDS sized to the launch's largest E (rm_rx_launch): 14.4 KB for C3, within the 16 KB a CU keeps free beside
  // the turbo decoder's two workgroups, so another batch's de-matching runs beside the decoder
  extern __shared__ uint4 es4[];
  const RmSlot     s = slots[blockIdx.x];
  if (!s.overwrite && *gptr(s.skip)) {
    return;
  }
  const int                  tid = threadIdx.x;
  const uintptr_t            ea  = (uintptr_t)s.e;
  const uint32_t             sh  = (uint32_t)(ea & 15u) / 2;
  const gptr_t<const uint4>  src = gptr(reinterpret_cast<const uint4*>(ea - 2 * sh));
  const uint32_t             n16 = (sh + s.E + 7) / 8;
  uint32_t                   i   = tid;
  for (; i + 3 * RM_LDS_THREADS < n16; i += 4 * RM_LDS_THREADS) {  // four loads in flight before the LDS stores
    const uint4 w0 = src[i], w1 = src[i + RM_LDS_THREADS], w2 = src[i + 2 * RM_LDS_THREADS],
                w3 = src[i + 3 * RM_LDS_THREADS];
    es4[i]                      = w0;
    es4[i + RM_LDS_THREADS]     = w1;
    es4[i + 2 * RM_LDS_THREADS] = w2;
    es4[i + 3 * RM_LDS_THREADS] = w3;
  }
  for (; i < n16; i += RM_LDS_THREADS) {
    es4[i] = src[i];
  }
  __syncthreads();
  const short*                 es  = reinterpret_cast<const short*>(es4) + sh;
  const gptr_t<const uint2>    inv = gptr(reinterpret_cast<const uint2*>(s.inv));
  const gptr_t<uint2>          sb  = gptr(reinterpret_cast<uint2*>(s.sb));
  constexpr int                UP  = 4;  // 4-position groups per thread whose table / buffer loads go together
  if (s.E <= s.N && s.E > 0) {  // one period at most: every position gathers at most one LLR
    for (uint32_t g0 = tid; 4 * g0 < s.len; g0 += UP * RM_LDS_THREADS) {
      uint2 iv[UP], v[UP];
#pragma unroll
      for (int u = 0; u < UP; u++) {
        const uint32_t g = g0 + u * RM_LDS_THREADS;
        if (4 * g < s.len) {
          iv[u] = inv[g];
          v[u]  = s.overwrite ? make_uint2(0, 0) : sb[g];
        }
      }
#pragma unroll
      for (int u = 0; u < UP; u++) {
        const uint32_t g = g0 + u * RM_LDS_THREADS;
        if (4 * g < s.len) {
          sb[g] = rm_group1(iv[u], v[u], es, s.E);
        }
      }
    }
    return;
  }
  for (uint32_t g0 = tid; 4 * g0 < s.len; g0 += UP * RM_LDS_THREADS) {
    uint2 iv[UP], v[UP];
#pragma unroll
    for (int u = 0; u < UP; u++) {
      const uint32_t g = g0 + u * RM_LDS_THREADS;
      if (4 * g < s.len) {
        iv[u] = inv[g];
        v[u]  = s.overwrite ? make_uint2(0, 0) : sb[g];
      }
    }
#pragma unroll
    for (int u = 0; u < UP; u++) {
      const uint32_t g = g0 + u * RM_LDS_THREADS;
      if (4 * g < s.len) {
        sb[g] = rm_group(iv[u], v[u], es, s.E, s.N);
      }
    }
  }
}

static constexpr int TB_CHUNK       = 16 * 64;  // payload bytes per assembly chunk (one wave, 16 B a lane)
static constexpr int TB_FIN_THREADS = 512;  // 8 waves: 2 a SIMD fit beside the turbo decoder (a C3 TB: ~10 chunks, 2 rounds)
static constexpr int TB_THREADS     = TB_FIN_THREADS;  // reset_range stride

// a * b mod P over GF(2) at compile time (the CRC placement tables below)
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
// zero bytes [0, nbytes) of p with 16-byte stores where aligned (block-cooperative)
__device__ void zero_bytes(uint8_t* p_, uint32_t nbytes, int tid, int nthreads)
{
  const gptr_t<uint8_t> p = gptr(p_);
  const uint32_t head = (uint32_t)((16 - ((uintptr_t)p & 15)) & 15);
  if (nbytes <= head + 16) {
    for (uint32_t i = tid; i < nbytes; i += nthreads) {
      p[i] = 0;
    }
    return;
  }
  const uint32_t nvec = (nbytes - head) / 16;
  for (uint32_t i = tid; i < head; i += nthreads) {
    p[i] = 0;
  }
  const gptr_t<uint4> v = reinterpret_cast<gptr_t<uint4>>(p + head);
  for (uint32_t i = tid; i < nvec; i += nthreads) {
    v[i] = make_uint4(0, 0, 0, 0);
  }
  for (uint32_t i = head + 16 * nvec + tid; i < nbytes; i += nthreads) {
    p[i] = 0;
  }
}

// Zero (as srsran_softbuffer_rx_reset_cb does) CB soft buffers [sb0, n), saved payloads
// [0, n) except those in `keep`, and CB flags [f0, max_cb).
__device__ void reset_range(const SchTb& t, uint32_t sb0, uint32_t n, uint32_t f0, uint32_t keep)
{
  const int tid = threadIdx.x;
  if (sb0 < n) {  // soft buffers are 8-byte aligned, sb_stride a multiple of 4
    const gptr_t<uint2> p = gptr(reinterpret_cast<uint2*>(t.sbuf + (size_t)sb0 * t.sb_stride));
    const uint32_t n64 = (n - sb0) * t.sb_stride / 4;
    for (uint32_t i = tid; i < n64; i += TB_THREADS) {
      p[i] = make_uint2(0, 0);
    }
  }
  if (keep == 0) {  // one contiguous range
    zero_bytes(t.saved, n * t.saved_stride, tid, TB_THREADS);
  } else {
    for (uint32_t c = 0; c < n; c++) {
      if (c < 32 && ((keep >> c) & 1u)) {
        continue;
      }
      zero_bytes(t.saved + (size_t)c * t.saved_stride, t.saved_stride, tid, TB_THREADS);
    }
  }
  for (uint32_t c = f0 + tid; c < t.max_cb; c += TB_THREADS) {
    gptr(t.cb_crc)[c] = 0;
  }
}

// Per-CB geometry of a TB as decode_tb leaves the payload (sch.c:425-431, 476-480): CB c writes
// len[c] bytes at start[c] = c * rlen / 8 (K/8 decoded bytes, or rlen/8 saved bytes when the CB
// was skipped); later CBs overwrite the CRC bytes of earlier ones.
struct TbGeom {
  uint32_t       start[SCH_MAX_CB], len[SCH_MAX_CB], rlen8[SCH_MAX_CB], okf[SCH_MAX_CB];
  const uint8_t* src[SCH_MAX_CB];
  uint32_t       noi_sum, end;
};

__device__ void tb_geometry(const SchTb& t, TbGeom& g)
{
  const int tid = threadIdx.x;
  if (tid == 0) {
    g.noi_sum = 0;
    g.end     = 0;
  }
  __syncthreads();
  if (tid < (int)t.C) {
    const uint32_t K    = tid < (int)t.C1 ? t.K1 : t.K2;
    const uint32_t rlen = t.C == 1 ? K : K - 24;
    const uint32_t slot = t.slot0 + tid;
    const uint32_t n    = gptr(t.noi)[slot];
    const bool     skip = n == 0;  // CB CRC was already OK: copy the saved payload (sch.c:476-480)
    g.start[tid]        = tid * rlen / 8;
    g.rlen8[tid]        = rlen / 8;
    g.len[tid]          = skip ? rlen / 8 : K / 8;
    g.src[tid]          = skip ? t.saved + (size_t)tid * t.saved_stride : t.cbout + (size_t)slot * SCH_SLOT_BYTES;
    g.okf[tid]          = skip ? 1u : gptr(t.crc_ok)[slot];
    atomicAdd(&g.noi_sum, n);
    atomicMax(&g.end, g.start[tid] + g.len[tid]);
  }
  __syncthreads();
}

// byte p of the payload: from the last CB (in decode order) whose write covered it
__device__ __forceinline__ uint8_t tb_byte(const SchTb& t, const TbGeom& g, uint32_t p)
{
  int c;
  if (t.C1 == t.C || t.K1 == t.K2) {  // one rlen: owner = min(p / rlen8, C - 1)
    c = (int)min(p / g.rlen8[0], t.C - 1);
  } else {
    c = (int)t.C - 1;
    while (c > 0 && !(p >= g.start[c] && p < g.start[c] + g.len[c])) {
      c--;
    }
  }
  return gptr(g.src[c])[p - g.start[c]];
}

// CRC24A byte table and x^(128 k) mod CRC24A (k = 0..63), built at compile time
struct Crc24Tables {
  uint32_t byte[256];
  uint32_t xp16[64];
};
constexpr Crc24Tables make_crc24_tables()
{
  Crc24Tables t{};
  for (uint32_t b = 0; b < 256; b++) {
    uint32_t c = b << 16;
    for (int k = 0; k < 8; k++) {
      c = (c & 0x800000u) ? ((c << 1) ^ LTE_CRC24A) : (c << 1);
    }
    t.byte[b] = c & 0xFFFFFFu;
  }
  uint32_t x128 = 1;
  for (int k = 0; k < 16; k++) {  // x^128 = (x^8)^16
    x128 = ce_clmul_mod24(x128, 0x100u, LTE_CRC24A);
  }
  uint32_t m = 1;
  for (int k = 0; k < 64; k++) {
    t.xp16[k] = m;
    m         = ce_clmul_mod24(m, x128, LTE_CRC24A);
  }
  return t;
}
__device__ const Crc24Tables kCrcT = make_crc24_tables();

// x^(8 TB_CHUNK c) mod CRC24A for c < TB_MAX_CHUNKS (the placement of chunk c's CRC at the message end)
struct ChunkPow {
  uint32_t v[TB_MAX_CHUNKS];
};
constexpr ChunkPow make_chunk_pow()
{
  ChunkPow t{};
  uint32_t m = 0x100u;  // x^8, squared up to x^(8 TB_CHUNK)
  for (int k = 1; k < TB_CHUNK; k <<= 1) {
    m = ce_clmul_mod24(m, m, LTE_CRC24A);
  }
  uint32_t p = 1;
  for (int c = 0; c < TB_MAX_CHUNKS; c++) {
    t.v[c] = p;
    p      = ce_clmul_mod24(p, m, LTE_CRC24A);
  }
  return t;
}
__device__ const ChunkPow kChunkPow = make_chunk_pow();
static_assert((TB_CHUNK & (TB_CHUNK - 1)) == 0, "TB_CHUNK a power of two (repeated squaring above)");

// One assembly chunk of a TB, by one wave (lane = 0..63).  Chunk c covers payload bytes
// [nbytes - (c+1) * TB_CHUNK, nbytes - c * TB_CHUNK), nbytes = (tbs + 24) / 8 -- aligned to the END
// of the CRC'd message so leading out-of-range bytes act as zeros, which do not change a
// zero-initialised CRC.  Lane j gathers 16 consecutive bytes, writes them to the payload and
// CRCs them (LDS byte table); its CRC moves to the chunk end with one multiply by
// x^(128 (63 - j)) and the lanes XOR-reduce: the chunk's CRC, placed later with x^(8 * TB_CHUNK * c).
// Chunk 0 also writes the bytes past nbytes (the last CB's CRC24B, sch.c:425-431).
__device__ uint32_t assemble_chunk(const SchTb& t, const TbGeom& g, const uint32_t* ctab, int chunk, int lane)
{
  const int nbytes = (int)((t.tbs + 24) / 8);
  const int c1     = nbytes - chunk * TB_CHUNK;  // one past the chunk's last byte
  const bool uniform = t.C1 == t.C || t.K1 == t.K2;
  const int  p0      = c1 - TB_CHUNK + 16 * lane;
  // the lane's 16 bytes: owners first (ALU / LDS), then every gather in flight at once, then the CRC
  uint32_t v[16];
  int      c = -1;
#pragma unroll
  for (int u = 0; u < 16; u++) {
    const int p = p0 + u;
    v[u]        = 0;
    if (p >= 0 && (uint32_t)p < g.end) {
      if (uniform) {
        if (c < 0) {
          c = (int)min((uint32_t)p / g.rlen8[0], t.C - 1);
        } else if (c + 1 < (int)t.C && (uint32_t)p >= g.start[c + 1]) {
          c++;
        }
        v[u] = gptr(g.src[c])[p - g.start[c]];
      } else {
        v[u] = tb_byte(t, g, (uint32_t)p);
      }
    }
  }
  uint32_t crc = 0;
#pragma unroll
  for (int u = 0; u < 16; u++) {
    const int p = p0 + u;
    if (p >= 0 && (uint32_t)p < g.end) {
      gptr(t.data)[p] = (uint8_t)v[u];
    }
    crc = ((crc << 8) ^ ctab[((crc >> 16) ^ v[u]) & 0xFFu]) & 0xFFFFFFu;
  }
  if (chunk == 0) {  // bytes past the CRC'd message
    for (uint32_t p = (uint32_t)nbytes + lane; p < g.end; p += 64) {
      gptr(t.data)[p] = tb_byte(t, g, p);
    }
  }
  crc = clmul24(crc, kCrcT.xp16[63 - lane], LTE_CRC24A);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    crc ^= (uint32_t)__shfl_xor((int)crc, off, 64);
  }
  return crc;
}

// tb_kernel: one workgroup per TB (4 waves) -- the payload assembly with the TB CRC24A of each 1 KB chunk
// (the waves take the chunks in turn), then the CB bookkeeping, the TB CRC from the chunk CRCs, saving of
// good CBs on failure, new-transmission resets (sch.c:458-573).  One launch for the whole tail of decode_tb.
__global__ __launch_bounds__(TB_FIN_THREADS) void tb_kernel(const SchTb* __restrict__ tbs)
{
  const SchTb t   = tbs[blockIdx.x];
  const int   tid = threadIdx.x;
  __shared__ uint32_t ctab[256];
  __shared__ uint32_t part[TB_MAX_CHUNKS];
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
  __shared__ TbGeom g;
  __shared__ uint32_t tb_crc;
  for (int k = tid; k < 256; k += TB_FIN_THREADS) {
    ctab[k] = kCrcT.byte[k];
  }
  tb_geometry(t, g);  // (its barriers also publish ctab)
  {
    const int nch = (int)(((t.tbs + 24) / 8 + TB_CHUNK - 1) / TB_CHUNK);
    for (int ch = tid >> 6; ch < nch; ch += TB_FIN_THREADS / 64) {
      const uint32_t crc = assemble_chunk(t, g, ctab, ch, tid & 63);
      if ((tid & 63) == 0) {
        part[ch] = crc;
      }
    }
  }
  __syncthreads();  // the payload and the chunk CRCs are complete
  const uint32_t C      = t.C;
  bool           all_ok = true;
  for (uint32_t c = 0; c < C; c++) {
    all_ok = all_ok && g.okf[c];
  }
  bool     tb_fail = false;
  uint32_t keep    = 0;
  if (!all_ok) {
    // keep the good CBs for the next retransmission (sch.c:465-474)
    for (uint32_t c = 0; c < C; c++) {
      if (g.okf[c]) {
        keep |= 1u << c;
        for (uint32_t i = tid; i < g.rlen8[c]; i += TB_FIN_THREADS) {
          gptr(t.saved)[(size_t)c * t.saved_stride + i] = gptr(t.data)[g.start[c] + i];
        }
      }
    }
  } else if (C > 1) {
    // TB CRC24A over tbs + 24 bits (srsran_crc_match_byte, sch.c:560): chunk c's CRC moved to the message end
    // by x^(8 TB_CHUNK c), one lane a chunk, XOR-reduced over the first wave
    if (tid < 64) {
      const uint32_t nch = ((t.tbs + 24) / 8 + TB_CHUNK - 1) / TB_CHUNK;
      uint32_t       r   = tid < (int)nch ? clmul24(part[tid], kChunkPow.v[tid], LTE_CRC24A) : 0u;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        r ^= (uint32_t)__shfl_xor((int)r, off, 64);
      }
      if (tid == 0) {
        tb_crc = r;
      }
    }
    __syncthreads();
    tb_fail = tb_crc != 0;  // srsran_softbuffer_rx_reset_cb_crc (sch.c:567)
  }
  if (tid < (int)C) {
    gptr(t.cb_crc)[tid] = (g.okf[tid] && !tb_fail) ? 1 : 0;
  }
  if (t.new_data) {
    // what reset_tbs cleared and this decode did not rewrite: flags past C, soft
    // buffers past C, saved payloads that were not saved just now
    reset_range(t, C, t.nof_cb_reset, C, keep);
  }
  if (tid == 0) {
    *t.tb_crc = all_ok ? 1 : 0;
    *t.result = (all_ok && !tb_fail) ? 0 : -1;
    *t.avg    = (float)g.noi_sum / (float)C;
  }
}

hipError_t rm_rx_launch(const RmSlot* d_slots, uint32_t nslots, uint32_t max_len, uint32_t max_e, hipStream_t stream)
{
  StageScope timing_scope(ST_RM, stream);
  if (nslots == 0) {
    return hipSuccess;
  }
  if (max_e <= (uint32_t)RM_LDS_MAX_E) {
    for (uint32_t s0 = 0; s0 < nslots; s0 += 65535) {
      const uint32_t n = nslots - s0 < 65535 ? nslots - s0 : 65535;
      hipLaunchKernelGGL(rm_rx_lds_kernel, dim3(n), dim3(RM_LDS_THREADS), ((size_t)(max_e + 7) / 8 + 1) * sizeof(uint4),
                         stream, d_slots + s0);
    }
    return hipGetLastError();
  }
  const uint32_t per_block = RM_THREADS * RM_PER_THREAD;
  const uint32_t gx        = (max_len + per_block - 1) / per_block;
  for (uint32_t s0 = 0; s0 < nslots; s0 += 65535) {
    const uint32_t n = nslots - s0 < 65535 ? nslots - s0 : 65535;
    hipLaunchKernelGGL(rm_rx_kernel, dim3(gx, n), dim3(RM_THREADS), 0, stream, d_slots + s0);
  }
  return hipGetLastError();
}

hipError_t tb_launch(const SchTb* d_tbs, uint32_t ntb, uint32_t max_tbs, hipStream_t stream)
{
  StageScope timing_scope(ST_TB, stream);
  if (ntb == 0) {
    return hipSuccess;
  }
  const uint32_t nch = ((max_tbs + 24) / 8 + TB_CHUNK - 1) / TB_CHUNK;
  if (nch > TB_MAX_CHUNKS) {
    return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(tb_kernel, dim3(ntb), dim3(TB_FIN_THREADS), 0, stream, d_tbs);
  return hipGetLastError();
}

// ulsch_deinterleave (sch.c:994-1021) with no RI bits: ulsch_interleave_gen (sch.c:661-682) numbers
// the input positions (i rows + j) Qm + k in (row j, column i, bit k) order and srsran_vec_lut_sis
// (vector.c:147-152) stores g[number] = q[position] -- a transpose of the rows x N_symb matrix of
// Qm-LLR groups.  One thread per output LLR: the stores are contiguous, the loads stride by rows Qm.
__global__ __launch_bounds__(256) void ul_deint_kernel(const int16_t* __restrict__ q, int16_t* __restrict__ g,
                                                       uint32_t rows, uint32_t cols, uint32_t Qm)
{
  const uint32_t n = rows * cols * Qm;
  for (uint32_t o = blockIdx.x * blockDim.x + threadIdx.x; o < n; o += gridDim.x * blockDim.x) {
    const uint32_t t = o / Qm, k = o - t * Qm;
    const uint32_t j = t / cols, i = t - j * cols;
    g[o]             = q[(i * rows + j) * Qm + k];
  }
}

hipError_t ul_deint_launch(const int16_t* q, int16_t* g, uint32_t Qm, uint32_t H_prime_total, uint32_t N_symb,
                           hipStream_t stream)
{
  if (N_symb == 0 || Qm == 0) {
    return hipErrorInvalidValue;
  }
  const uint32_t rows = H_prime_total / N_symb, n = rows * N_symb * Qm;
  if (n == 0) {
    return hipSuccess;
  }
  StageScope timing_scope(ST_RM, stream);
  hipLaunchKernelGGL(ul_deint_kernel, dim3((n + 255) / 256 < 2048u ? (n + 255) / 256 : 2048u), dim3(256), 0, stream, q, g, rows, N_symb, Qm);
  return hipGetLastError();
}

// Batched form, tiled through LDS: q holds N_symb rows (columns i of the interleaver) of rows Qm
// LLRs, g is its transpose.  A workgroup takes 64 interleaver rows j of one TB: it reads, for every
// i, the contiguous run q[(i rows + j0) Qm ..) and writes the contiguous run g[j0 N_symb Qm ..).
constexpr uint32_t UL_TILE_J = 64, UL_MAX_SYMB = 14, UL_MAX_QM = 8;
__global__ __launch_bounds__(256) void ul_deint_batch_kernel(const UlDeint* __restrict__ desc)
{
  __shared__ int16_t tile[UL_MAX_SYMB * UL_TILE_J * UL_MAX_QM];
  const UlDeint  d  = desc[blockIdx.y];
  const uint32_t j0 = blockIdx.x * UL_TILE_J;
  if (j0 >= d.rows) {
    return;
  }
  const uint32_t nj  = min(UL_TILE_J, d.rows - j0);
  const uint32_t run = nj * d.Qm;  // LLRs of one interleaver column inside the tile
  for (uint32_t x = threadIdx.x; x < d.cols * run; x += blockDim.x) {
    const uint32_t i = x / run, r = x - i * run;
    tile[i * UL_TILE_J * UL_MAX_QM + r] = d.q[(i * d.rows + j0) * d.Qm + r];
  }
  __syncthreads();
  const uint32_t row = d.cols * d.Qm;  // LLRs of one output row j
  if (d.g0_src < 0) {
    for (uint32_t x = threadIdx.x; x < nj * row; x += blockDim.x) {
      const uint32_t jj = x / row, r = x - jj * row, i = r / d.Qm, k = r - i * d.Qm;
      d.g[j0 * row + x] = tile[i * UL_TILE_J * UL_MAX_QM + jj * d.Qm + k];
    }
    return;
  }
  // with RI: row j holds the non-RI cells of that row; the rows before it lost sum_i max(0,
  // j - (rows - ri_rows[i])) cells
  for (uint32_t x = threadIdx.x; x < nj * row; x += blockDim.x) {
    const uint32_t jj = x / row, r = x - jj * row, i = r / d.Qm, k = r - i * d.Qm, j = j0 + jj;
    if (j + d.ri_rows[i] >= d.rows) {
      continue;
    }
    uint32_t lost = 0, before = 0;
    for (uint32_t c = 0; c < d.cols; c++) {
      const uint32_t first = d.rows - d.ri_rows[c];  // first RI row of column c
      lost += j > first ? j - first : 0;
      before += (c < i && j >= first) ? 1 : 0;
    }
    const uint32_t o = (j * d.cols - lost + i - before) * d.Qm + k;
    d.g[o]           = o == 0 ? d.q[d.g0_src] : tile[i * UL_TILE_J * UL_MAX_QM + jj * d.Qm + k];
  }
}

hipError_t ul_deint_batch_launch(const UlDeint* d_desc, uint32_t ntb, uint32_t max_rows, hipStream_t stream)
{
  if (ntb == 0 || max_rows == 0) {
    return hipSuccess;
  }
  StageScope timing_scope(ST_RM, stream);
  hipLaunchKernelGGL(ul_deint_batch_kernel, dim3((max_rows + UL_TILE_J - 1) / UL_TILE_J, ntb), dim3(256), 0, stream,
                     d_desc);
  return hipGetLastError();
}

}  // namespace srsran_amd

// ---------------- descriptor staging (stage_copy.h; host side in stage_copy.cpp) ----------------
namespace srsran_amd {

__global__ __launch_bounds__(256) void stage_copy_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                         uint32_t n16, uint32_t* __restrict__ zero, uint32_t nz,
                                                         uint32_t* __restrict__ fence, uint32_t* __restrict__ count,
                                                         uint32_t seq)
{
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) {
    dst[i] = src[i];
  }
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < nz; i += gridDim.x * 256) {
    zero[i] = 0;
  }
  if (fence) {
    __syncthreads();  // every load of this workgroup has returned (its value was stored above); no fence (stage_jobs.h)
    if (threadIdx.x == 0) {
      if (atomicAdd(count, 1u) == gridDim.x - 1) {  // the last workgroup: the whole slot has been read
        __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(fence, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

hipError_t stage_copy_job(const CopyJob& j, hipStream_t stream)
{
  const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>((std::max(j.n16, j.nz) + 255) / 256, 256));
  hipLaunchKernelGGL(stage_copy_kernel, dim3(blocks), dim3(256), 0, stream, j.dst, j.src, j.n16, j.zero, j.nz, j.fence,
                     j.count, j.seq);
  return hipGetLastError();
}

hipError_t stage_copy_launch(void* dst, const void* src_dev, size_t bytes, hipStream_t stream, uint32_t* zero,
                             uint32_t zero_words, const StageFence* fence, int slot, uint32_t seq)
{
  const uint32_t n16 = (uint32_t)((bytes + 15) / 16);
  const uint32_t nz  = zero ? zero_words : 0;
  if (n16 == 0 && nz == 0 && !fence) {
    return hipSuccess;
  }
  const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>((std::max(n16, nz) + 255) / 256, 256));
  hipLaunchKernelGGL(stage_copy_kernel, dim3(blocks), dim3(256), 0, stream, (uint4*)dst, (const uint4*)src_dev, n16,
                     zero, nz, fence ? fence->d + slot : nullptr, fence ? fence->count : nullptr, seq);
  return hipGetLastError();
}

}  // namespace srsran_amd
