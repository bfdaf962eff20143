// srsran_4g_amd/csrc/sch_api.cpp -- C-ABI host side of the DL-SCH receive path.
//
// Implements include/srsran_sch.h:
//   code block segmentation            cbsegm.c:62-151
//   CRC host utilities                 crc.c:69-195
//   rate de-matching tables + RX       rm_turbo.c:175-317, 390-483 (executed by rm_rx_kernel)
//   HARQ soft buffers in HBM           softbuffer.c:36-178
//   sch object + DL-SCH decode         sch.c:140-230, 371-609
// The decode runs entirely on the GPU (sch_kernel.hip + tdec_kernel.hip); the host
// only segments, builds descriptors and copies.  No CPU fallback.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../../include/srsran_sch.h"
#include "devkey.h"
#include "sch_kernel.h"
#include "tdec_kernel.h"
#include "tdec8bit_kernel.h"
#include "enc_kernel.h"
#include "uci_kernel.h"
#include "pdsch_internal.h"
#include "ulsch_batch.h"
#include "stage_copy.h"
#include "stage_timing.h"

using namespace srsran_amd;

namespace {

// 36.213 Table 7.1.7.2.1-1, I_TBS = 33 (the largest index, 256QAM table), N_PRB = 1..110:
// srsran_softbuffer_rx_init sizes max_cb from it (softbuffer.c:38-46).
const int kTbsMaxIdx[SRSRAN_MAX_PRB] = {
       968,   1992,   2984,   4008,   4968,   5992,   6968,   7992,   8760,   9912,  10680,
     11832,  12960,  13536,  14688,  15840,  16992,  17568,  19080,  19848,  20616,  21384,
     22920,  23688,  24496,  25456,  26416,  27376,  28336,  29296,  30576,  31704,  32856,
     34008,  35160,  35160,  36696,  37888,  39232,  39232,  40576,  40576,  42368,  43816,
     43816,  45352,  46888,  46888,  48936,  48936,  51024,  51024,  52752,  52752,  55056,
     55056,  57336,  57336,  59256,  59256,  59256,  61664,  61664,  63776,  63776,  63776,
     66592,  66592,  68808,  68808,  71112,  71112,  71112,  73712,  75376,  76208,  76208,
     76208,  78704,  78704,  81176,  81176,  81176,  81176,  84760,  84760,  84760,  87936,
     87936,  87936,  90816,  90816,  90816,  93800,  93800,  93800,  93800,  97896,  97896,
     97896,  97896,  97896,  97896,  97896,  97896,  97896,  97896,  97896,  97896,  97896,
};

// Sub-block interleaver inter-column permutation, 36.212 Table 5.1.4-1.
const uint8_t kColPerm[32] = {0, 16, 8,  24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30,
                              1, 17, 9,  25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31};

std::mutex g_mu;
int        g_have_gpu = -1;

bool have_gpu_locked()
{
  if (g_have_gpu < 0) {
    int n      = 0;
    g_have_gpu = (hipGetDeviceCount(&n) == hipSuccess && n > 0) ? 1 : 0;
  }
  return g_have_gpu == 1;
}

bool have_gpu()
{
  std::lock_guard<std::mutex> lk(g_mu);
  return have_gpu_locked();
}

// ---------------- rate de-matching tables (rm_turbo.c:175-317) ----------------
// For one (K, rv, layout): inv[p] = index, in the rv's circular read-out order with
// the dummy bits dropped, of the coded bit stored at soft-buffer position p; that
// order repeats with period N = 3K+12 along the E received LLRs.
struct InvTable {
  uint16_t* d   = nullptr;
  uint32_t  len = 0;  // soft buffer positions of the layout
  uint32_t  N   = 0;  // 3K + 12
};
std::map<uint64_t, InvTable> g_inv;  // (device, cb_idx, rv, layout)

uint32_t rx_subblocks(uint32_t K, bool tdec_layout)
{
  return tdec_layout ? srsran_tdec_autoimp_get_subblocks(K) : 0;
}

// nsb: sub-blocks of the decoder layout (0 natural; 8 / 16 / 32 as rm_turbo.c's deinterleaver_sb)
bool inv_table_nsb(uint32_t cb_idx, uint32_t rv, uint32_t nsb, InvTable* out)
{
  const uint32_t              K   = (uint32_t)srsran_cbsegm_cbsize(cb_idx);
  const uint64_t              key = ((uint64_t)cur_dev() << 32) | ((cb_idx * 4 + rv) * 64 + nsb);
  std::lock_guard<std::mutex> lk(g_mu);
  auto                        it = g_inv.find(key);
  if (it != g_inv.end()) {
    *out = it->second;
    return true;
  }
  if (!have_gpu_locked()) {
    return false;
  }
  const uint32_t D = K + 4, R = (D + 31) / 32, Kp = 32 * R, ND = Kp - D, Kw = 3 * Kp;
  const uint32_t k0 = R * (2 * ((Kw + 8 * R - 1) / (8 * R)) * rv + 2);  // 36.212 5.1.4.1.2
  InvTable       t;
  t.N   = 3 * K + 12;
  t.len = nsb ? 3 * (K + 32) + 12 : t.N;
  std::vector<uint16_t> inv(t.len, 0xFFFF);
  const uint32_t        L = nsb ? K / nsb : K;
  for (uint32_t k = 0, j = 0; k < t.N; j++) {
    const uint32_t w = (k0 + j) % Kw;
    uint32_t       stream, col;
    if (w < Kp) {
      stream = 0;
      col    = w;
    } else {
      stream = 1 + ((w - Kp) & 1);
      col    = (w - Kp) >> 1;
    }
    uint32_t y = kColPerm[col / R] + 32 * (col % R);  // position in the padded stream
    if (stream == 2) {
      y = (y + 1) % Kp;  // pi(k) for the second parity stream
    }
    if (y < ND) {
      continue;  // dummy bit, not transmitted
    }
    const uint32_t i = y - ND;        // bit index in d^(stream)
    uint32_t       n = 3 * i + stream;  // encoder output order (natural 3K+12 layout)
    if (nsb) {  // turbo decoder sub-block layout (rm_turbo.c:260-273)
      n = n < 3 * K ? (n % 3) * (K + 32) + ((n / 3) % L) * nsb + (n / 3) / L : n - 3 * K + 3 * (K + 32);
    }
    inv[n] = (uint16_t)k++;
  }
  if (hipMalloc(&t.d, t.len * sizeof(uint16_t)) != hipSuccess ||
      hipMemcpy(t.d, inv.data(), t.len * sizeof(uint16_t), hipMemcpyHostToDevice) != hipSuccess) {
    return false;
  }
  g_inv[key] = t;
  *out       = t;
  return true;
}

bool inv_table(uint32_t cb_idx, uint32_t rv, bool tdec_layout, InvTable* out)
{
  return inv_table_nsb(cb_idx, rv, rx_subblocks((uint32_t)srsran_cbsegm_cbsize(cb_idx), tdec_layout), out);
}

// ---------------- soft buffer device arena ----------------
struct SbGpu {
  short*   d_buf   = nullptr;  // max_cb x stride int16
  uint8_t* d_data  = nullptr;  // max_cb x data_stride bytes
  uint8_t* d_flags = nullptr;  // [0, max_cb): cb_crc, [max_cb]: tb_crc
  uint32_t stride = 0, data_stride = 0;
  size_t   buf_bytes = 0;      // d_buf size (rounded as the arena hands it out)
  int      buf_dev   = -1;     // >= 0: d_buf lives in that device's soft-buffer arena
  int      dev       = 0;      // the device every buffer of this soft buffer lives on
};

// Makes `dev` current for a scope and restores the caller's device: soft buffers are synchronised
// and released on the device they live on, whatever device the caller has selected.
struct DevScope {
  int prev = -1;
  explicit DevScope(int dev)
  {
    if (hipGetDevice(&prev) == hipSuccess && prev != dev) {
      hipSetDevice(dev);
    } else {
      prev = -1;
    }
  }
  ~DevScope()
  {
    if (prev >= 0) {
      hipSetDevice(prev);
    }
  }
};

// Soft-buffer arena: the int16 soft buffers of every srsran_softbuffer_rx_t of a device come from one
// allocation (1 GiB by default, srsran_softbuffer_rx_gpu_arena), which keeps the per-object
// hipMalloc off the HARQ setup path and the blocks of a batch close together in L2 / TLB terms.
// Decoder selection does not depend on it: the turbo descriptor list is padded wherever two
// blocks of a lane-pair workgroup lie far apart (tdec_pair_cbs).  Freed buffers are kept per size
// for reuse; when the arena is full, buffers fall back to hipMalloc (reported once).
struct SbArena {
  uint8_t*                       base = nullptr;
  size_t                         cap = 0, top = 0;
  bool                           tried = false;
  std::multimap<size_t, size_t>  free_by_size;  // size -> offset
};
std::mutex                       g_arena_mu;
std::unordered_map<int, SbArena> g_arenas;
size_t                           g_arena_bytes = (size_t)1 << 30;  // capacity of arenas created from now on
bool                             g_arena_on    = true;             // false: every buffer its own hipMalloc
bool                             g_arena_warned = false;

void* sb_arena_alloc(size_t bytes, int* dev_out)
{
  bytes   = (bytes + 255) & ~(size_t)255;
  int dev = 0;
  hipGetDevice(&dev);
  if (g_arena_on) {
    std::lock_guard<std::mutex> lk(g_arena_mu);
    SbArena&                    a = g_arenas[dev];
    if (!a.tried) {
      a.tried = true;
      if (hipMalloc((void**)&a.base, g_arena_bytes) == hipSuccess) {
        a.cap = g_arena_bytes;
      } else {
        a.base = nullptr;
      }
    }
    auto it = a.free_by_size.find(bytes);
    if (it != a.free_by_size.end()) {
      const size_t off = it->second;
      a.free_by_size.erase(it);
      *dev_out = dev;
      return a.base + off;
    }
    if (a.base && a.top + bytes <= a.cap) {
      const size_t off = a.top;
      a.top += bytes;
      *dev_out = dev;
      return a.base + off;
    }
    if (!g_arena_warned) {
      g_arena_warned = true;
      fprintf(stderr, "[srsran_softbuffer] soft-buffer arena of device %d full (%zu MiB): further buffers use hipMalloc\n",
              dev, a.cap >> 20);
    }
  }
  void* p  = nullptr;
  *dev_out = -1;
  return hipMalloc(&p, bytes) == hipSuccess ? p : nullptr;
}

void sb_arena_free(void* p, size_t bytes, int dev)
{
  if (!p) {
    return;
  }
  if (dev < 0) {
    hipFree(p);
    return;
  }
  bytes = (bytes + 255) & ~(size_t)255;
  std::lock_guard<std::mutex> lk(g_arena_mu);
  SbArena&                    a = g_arenas[dev];
  a.free_by_size.emplace(bytes, (size_t)((uint8_t*)p - a.base));
}

}  // namespace

namespace srsran_amd {
// device views of a soft buffer for other modules of the library (NR SCH)
uint8_t* softbuffer_dflags(srsran_softbuffer_rx_t* q) { return q && q->gpu ? ((SbGpu*)q->gpu)->d_flags : nullptr; }
uint8_t* softbuffer_ddata(srsran_softbuffer_rx_t* q) { return q && q->gpu ? ((SbGpu*)q->gpu)->d_data : nullptr; }
uint32_t softbuffer_data_stride(srsran_softbuffer_rx_t* q) { return q && q->gpu ? ((SbGpu*)q->gpu)->data_stride : 0; }
}  // namespace srsran_amd

namespace {

// ---------------- sch object device context ----------------
// Descriptor staging of one batch.  A ring of kStageRing slots: the host builds the next batches while the GPU
// still reads earlier ones' descriptors, and waits only for the slot's previous user (kStageRing batches back).
constexpr int kStageRing = 3;
struct StageSlot {
  hipEvent_t staged = nullptr;  // SRSRAN_AMD_STAGE=side: this slot's last upload done (pinned staging reusable)
  hipEvent_t done   = nullptr;  // SRSRAN_AMD_STAGE=side: the batch that last used this slot finished with it
  uint32_t   seq    = 0;        // default staging: fence sequence number of the batch that last filled the slot
  bool       used   = false;
  char*      h      = nullptr;  // pinned coherent host memory (stage_host_alloc)
  char*      hd     = nullptr;  // its device alias
  char*      d      = nullptr;
  size_t     cap    = 0;
};

struct SchCtx {
  hipStream_t stream = nullptr;
  hipStream_t copy   = nullptr;  // descriptor uploads of the batch path, ahead of the launches that read them
  hipEvent_t  done   = nullptr;  // last batch finished with the shared scratch (cbout, flags, chunk CRCs, wide rows)
  StageSlot   ring[kStageRing];
  uint32_t    ring_next = 0;
  srsran_amd::StageFence    fence;  // the copy kernel's "slot read" words (stage_copy.h)
  srsran_amd::StreamHandoff ho;     // stream of the previous batch (device-side reuse of slots and scratch)
  uint8_t*    d_cbout = nullptr;
  uint8_t*    d_noi = nullptr;
  uint8_t*    d_crc_ok = nullptr;
  size_t      slot_cap = 0;
  // synchronous decode scratch
  int16_t*    d_e = nullptr;
  size_t      e_cap = 0;
  uint8_t*    d_data = nullptr;
  int32_t*    d_res = nullptr;
  float*      d_avg = nullptr;
  uint8_t*    h_io = nullptr;  // pinned: flags in/out, result, avg
  uint8_t*    d_zero = nullptr;  // a cleared cb_crc flag for new transmissions
  bool        used = false;
  int16_t*    d_ul = nullptr;    // srsran_ulsch_decode: q then g bits
  size_t      ul_cap = 0;
  UlDeint*    d_uldesc = nullptr;  // srsran_ulsch_gpu_decode_batch descriptors (device)
  UlDeint*    h_uldesc = nullptr;  // their pinned staging
  hipEvent_t  uldesc_used = nullptr;  // recorded after the de-interleaver launch that reads them
  bool        uldesc_live = false;
  size_t      uldesc_cap = 0;
  uint8_t*    d_uci = nullptr;     // srsran_ulsch_decode with UCI: descriptors, results, sequence
  size_t      uci_cap = 0;
  uint8_t*    d_ubs = nullptr;     // the batched UL-SCH receive: descriptors and results (device)
  size_t      dubs_cap = 0;
  uint8_t*    h_ubs = nullptr;     // its pinned staging
  size_t      hubs_cap = 0;
  uint8_t*    d_enc = nullptr;     // DL-SCH encode: descriptors, TB CRCs, unpacked e bits, staging
  size_t      enc_cap = 0;
  short*      d_wide = nullptr;    // llr_is_8bit, K <= 800: the widened soft buffers the 16-bit decoders read
  size_t      wide_cap = 0;        // rows of kWideStride
};

constexpr uint32_t kWideStride = 4096;  // int16 values a widened row (>= 3 (800 + 32) + 12 and the decoders' reads)

constexpr size_t kDataCap = (size_t)SCH_MAX_CB * SCH_SLOT_BYTES;

size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

bool init_ring(SchCtx* x)
{
  for (StageSlot& st : x->ring) {
    if (srsran_amd::ring_event_create(&st.staged) != hipSuccess ||
        srsran_amd::ring_event_create(&st.done) != hipSuccess) {
      return false;
    }
  }
  return srsran_amd::stage_fence_init(x->fence, kStageRing);
}

// the object's previous batches are done with its shared device state (grow paths)
void drain_batches(SchCtx* x)
{
  if (srsran_amd::stage_side_copy()) {
    if (x->used) {
      hipEventSynchronize(x->done);
    }
  } else {
    srsran_amd::handoff_drain(x->ho);
  }
}

bool grow_dev(void** p, size_t* cap, size_t need)
{
  if (*cap >= need) {
    return true;
  }
  hipFree(*p);
  *p = nullptr;
  if (hipMalloc(p, need) != hipSuccess) {
    *cap = 0;
    return false;
  }
  *cap = need;
  return true;
}

struct Plan {
  srsran_cbsegm_t s{};
  int32_t         status = 1;
  uint32_t        slot0  = 0;
};

// decode_tb's checks (sch.c:509-546, decode_tb_cb 383-386), in the reference's order.
int32_t check_tb(const srsran_dlsch_gpu_tb_t& tb, srsran_cbsegm_t* s)
{
  if (srsran_cbsegm(s, tb.tbs)) {
    return SRSRAN_ERROR;  // srsran_dlsch_decode2: segmentation error (sch.c:592-595)
  }
  if (!tb.d_data || !tb.softbuffer || !tb.softbuffer->gpu || !tb.d_e_bits || tb.Qm == 0) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (s->tbs == 0 || s->C == 0) {
    return SRSRAN_SUCCESS;
  }
  if (s->F || s->C > tb.softbuffer->max_cb || tb.rv > 3) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (s->C > SRSRAN_MAX_CODEBLOCKS) {
    return SRSRAN_ERROR;
  }
  return 1;
}

// Enqueue the three-kernel DL-SCH decode of ntb transport blocks on `stream`.
// out_idx (optional): TB i's result / average-iterations slot is d_result[out_idx[i]] (default i).
int enqueue_batch(srsran_sch_t* q, uint32_t ntb, const srsran_dlsch_gpu_tb_t* tbs, int32_t* d_result, float* d_avg,
                  hipStream_t stream, bool early_copy = false, const uint32_t* out_idx = nullptr)
{
  srsran_amd::HostScope desc(srsran_amd::HP_SCH_DESC);
  SchCtx*           x  = (SchCtx*)q->gpu;
  const bool        b8 = q->llr_is_8bit;  // int8 e bits / soft buffers (sch.c:409-428)
  std::vector<Plan> plan(ntb);
  uint32_t          nslots = 0;
  for (uint32_t i = 0; i < ntb; i++) {
    plan[i].status = check_tb(tbs[i], &plan[i].s);
    if (plan[i].status == 1) {
      plan[i].slot0 = nslots;
      nslots += plan[i].s.C;
    }
  }
  // per-slot de-matching descriptors, and turbo descriptors grouped by K
  std::vector<RmSlot>                         rm(nslots);
  std::map<uint32_t, std::vector<uint32_t>>   by_k;
  std::vector<uint8_t>                        slot_crc_a(nslots);
  uint32_t                                    max_len = 0, max_e = 0;
  for (uint32_t i = 0; i < ntb; i++) {
    if (plan[i].status != 1) {
      continue;
    }
    const srsran_cbsegm_t& s  = plan[i].s;
    const SbGpu*           sb = (const SbGpu*)tbs[i].softbuffer->gpu;
    const uint32_t         Qm = tbs[i].Qm;
    InvTable               tk[2];  // the de-matching tables of K1 and K2 (looked up once per TB)
    // the soft buffer layout of the decoder that takes K: the 16-bit AUTO one, or with llr_is_8bit the 8-bit one
    // (rm_turbo_rx_lut_8bit: srsran_tdec_autoimp_get_subblocks_8bit)
    auto table = [&](uint32_t idx, InvTable* t) {
      return b8 ? inv_table_nsb(idx, tbs[i].rv, srsran_tdec_autoimp_get_subblocks_8bit(srsran_cbsegm_cbsize(idx)), t)
                : inv_table(idx, tbs[i].rv, true, t);
    };
    if (!table(s.K1_idx, &tk[0]) || (s.C2 && !table(s.K2_idx, &tk[1]))) {
      return SRSRAN_ERROR;
    }
    for (uint32_t cb = 0; cb < s.C; cb++) {
      const uint32_t K     = cb < s.C1 ? s.K1 : s.K2;
      // E split over the CBs, including the reference's '>' (sch.c:398-407)
      const uint32_t Gp    = tbs[i].nof_e_bits / Qm;
      const uint32_t gamma = Gp % s.C;
      const uint32_t n_e   = Qm * (Gp / s.C);
      uint32_t       rp = cb * n_e, n_e2 = n_e;
      if (cb > s.C - gamma) {
        n_e2 = n_e + Qm;
        rp   = (s.C - gamma) * n_e + (cb - (s.C - gamma)) * n_e2;
      }
      const InvTable& t    = tk[cb < s.C1 ? 0 : 1];
      const uint32_t slot = plan[i].slot0 + cb;
      RmSlot&        r    = rm[slot];
      r.e                 = b8 ? (const short*)((const int8_t*)tbs[i].d_e_bits + rp) : tbs[i].d_e_bits + rp;
      r.sb                = sb->d_buf + (size_t)cb * sb->stride;
      r.skip              = sb->d_flags + cb;
      r.inv               = t.d;
      r.E                 = n_e2;
      r.len               = t.len;
      r.N                 = t.N;
      r.overwrite         = tbs[i].new_data ? 1 : 0;
      max_len             = std::max(max_len, t.len);
      max_e               = std::max(max_e, n_e2);
      by_k[K].push_back(slot);
      slot_crc_a[slot] = s.C == 1;  // single-CB TB: CRC24A over tbs + 24 (sch.c:440-446)
    }
  }
  // turbo descriptors by K; every two consecutive blocks of a group (one lane-pair workgroup) lie
  // within TDEC_PAIR_SPAN of each other, padded where the soft buffers are far apart
  // llr_is_8bit with K <= 800: the reference widens the block for a 16-bit decoder (tdec_iteration_8,
  // turbodecoder.c:470-481); those rows are widened into d_wide first
  std::vector<Widen8> wide;
  uint32_t            max_wide = 0;
  if (b8) {
    for (auto& kv : by_k) {
      if (srsran_tdec_autoimp_get_subblocks_8bit(kv.first) < 16) {
        for (uint32_t slot : kv.second) {
          wide.push_back(Widen8{(const int8_t*)rm[slot].sb, nullptr, rm[slot].len});
          max_wide = std::max(max_wide, rm[slot].len);
        }
      }
    }
    if (wide.size() > x->wide_cap) {
      drain_batches(x);
      hipFree(x->d_wide);
      x->d_wide         = nullptr;
      const size_t rows = std::max(wide.size() * 2, (size_t)16);
      if (hipMalloc((void**)&x->d_wide, rows * kWideStride * sizeof(short)) != hipSuccess) {
        x->wide_cap = 0;
        return SRSRAN_ERROR;
      }
      x->wide_cap = rows;
    }
    for (size_t j = 0; j < wide.size(); j++) {
      wide[j].dst = x->d_wide + j * kWideStride;
    }
  }
  std::vector<TdecCb> cbs;
  cbs.reserve(nslots + 16);
  std::vector<std::pair<uint32_t, uint32_t>> groups;  // (K, first index into cbs)
  std::vector<TdecCb>                        kcbs;
  uint32_t                                   nw = 0;
  for (auto& kv : by_k) {
    groups.emplace_back(kv.first, (uint32_t)cbs.size());
    kcbs.clear();
    const bool widened = b8 && srsran_tdec_autoimp_get_subblocks_8bit(kv.first) < 16;
    for (uint32_t slot : kv.second) {
      TdecCb c;
      c.in    = widened ? wide[nw++].dst : rm[slot].sb;
      c.skip  = rm[slot].overwrite ? x->d_zero : rm[slot].skip;  // a new transmission decodes every CB
      c.slot  = slot;
      c.crc_a = slot_crc_a[slot];
      kcbs.push_back(c);
    }
    tdec_pair_cbs(kcbs.data(), (uint32_t)kcbs.size(), cbs.size(), &cbs);
  }
  const uint32_t ncbs = (uint32_t)cbs.size();
  std::vector<SchTb> tbd(ntb);
  for (uint32_t i = 0; i < ntb; i++) {
    SchTb& t = tbd[i];
    memset(&t, 0, sizeof(t));
    t.result = d_result + (out_idx ? out_idx[i] : i);
    t.avg    = d_avg + (out_idx ? out_idx[i] : i);
    t.status = plan[i].status;
    const srsran_softbuffer_rx_t* sbh = tbs[i].softbuffer;
    if (sbh && sbh->gpu) {
      const SbGpu* sb = (const SbGpu*)sbh->gpu;
      t.cb_crc        = sb->d_flags;
      t.tb_crc        = sb->d_flags + sbh->max_cb;
      t.saved         = sb->d_data;
      t.saved_stride  = sb->data_stride;
      t.sbuf          = sb->d_buf;
      t.sb_stride     = sb->stride;
      t.max_cb        = sbh->max_cb;
      t.nof_cb_reset  = std::min((tbs[i].tbs + 24) / (SRSRAN_TCOD_MAX_LEN_CB - 24) + 1, sbh->max_cb);
      t.new_data      = tbs[i].new_data ? 1 : 0;
    }
    if (plan[i].status != 1) {
      continue;
    }
    t.data          = tbs[i].d_data;
    t.cbout         = nullptr;  // filled below once the scratch is sized
    t.slot0         = plan[i].slot0;
    t.C             = plan[i].s.C;
    t.C1            = plan[i].s.C1;
    t.K1            = plan[i].s.K1;
    t.K2            = plan[i].s.K2;
    t.tbs           = plan[i].s.tbs;
  }

  // the previous batch of this object must be done with the shared scratch: ordered by the stream, or by the
  // hand-over when this batch comes on another stream (side staging: the round-3 event)
  const bool side = srsran_amd::stage_side_copy();
  if (side) {
    if (x->used) {
      hipStreamWaitEvent(stream, x->done, 0);
    }
  } else if (srsran_amd::handoff(x->ho, stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  const size_t off_cbs  = align16(nslots * sizeof(RmSlot));
  const size_t off_tb   = off_cbs + align16(ncbs * sizeof(TdecCb));
  const size_t off_wide = off_tb + align16(ntb * sizeof(SchTb));
  const size_t bytes    = off_wide + align16(wide.size() * sizeof(Widen8));
  desc.stop();
  srsran_amd::HostScope wait(srsran_amd::HP_SCH_WAIT);
  const int  slot   = (int)x->ring_next;
  StageSlot& st     = x->ring[slot];
  x->ring_next = (x->ring_next + 1) % kStageRing;
  if (st.used) {
    if (side) {
      hipEventSynchronize(st.staged);
    } else if (!srsran_amd::stage_fence_wait(x->fence, slot, st.seq)) {
      return SRSRAN_ERROR;
    }
  }
  wait.stop();
  srsran_amd::HostScope launch(srsran_amd::HP_SCH_LAUNCH);
  if (bytes > st.cap) {  // every slot of the ring grows now: no allocation when the others come round
    const size_t cap = std::max(bytes * 2, (size_t)4096);
    for (StageSlot& r : x->ring) {
      if (r.cap >= cap) {
        continue;
      }
      if (r.used) {
        if (side) {
          hipEventSynchronize(r.done);
        } else {
          srsran_amd::handoff_drain(x->ho);
        }
      }
      hipHostFree(r.h);
      hipFree(r.d);
      r.h = nullptr;
      r.d = nullptr;
      r.h = (char*)srsran_amd::stage_host_alloc(cap, (void**)&r.hd);
      if (!r.h || hipMalloc((void**)&r.d, cap) != hipSuccess) {
        r.cap = 0;
        return SRSRAN_ERROR;
      }
      r.cap = cap;
    }
  }
  if (nslots > x->slot_cap) {
    drain_batches(x);
    {
      const size_t cap = std::max((size_t)nslots * 2, (size_t)64);
      hipFree(x->d_cbout);
      hipFree(x->d_noi);
      hipFree(x->d_crc_ok);
      x->d_cbout = x->d_noi = x->d_crc_ok = nullptr;
      if (hipMalloc((void**)&x->d_cbout, cap * SCH_SLOT_BYTES) != hipSuccess ||
          hipMalloc((void**)&x->d_noi, cap) != hipSuccess || hipMalloc((void**)&x->d_crc_ok, cap) != hipSuccess) {
        x->slot_cap = 0;
        return SRSRAN_ERROR;
      }
      x->slot_cap = cap;
    }
  }
  uint32_t max_tbs = 0;
  for (uint32_t i = 0; i < ntb; i++) {
    SchTb& t = tbd[i];
    if (t.status == 1) {
      t.cbout  = x->d_cbout;
      t.noi    = x->d_noi;
      t.crc_ok = x->d_crc_ok;
      max_tbs  = std::max(max_tbs, t.tbs);
    }
  }
  memcpy(st.h, rm.data(), nslots * sizeof(RmSlot));
  memcpy(st.h + off_cbs, cbs.data(), ncbs * sizeof(TdecCb));
  memcpy(st.h + off_tb, tbd.data(), ntb * sizeof(SchTb));
  if (!wide.empty()) {
    memcpy(st.h + off_wide, wide.data(), wide.size() * sizeof(Widen8));
  }
  // SRSRAN_AMD_STAGE=side, early_copy (the PDSCH chain, whose stream runs OFDM ... LLR before the de-matching): the upload runs on
  // the copy stream as soon as the slot's previous batch is done with it, beside those stages, and the
  // launches below wait for it instead of having the copy's latency in line in front of them (chain
  // 243-246 k -> 250-255 k subframes/s, gpurun_out r03ah).  A batch with nothing in front of it keeps the
  // in-stream upload (the cross-stream wait costs a standalone DL-SCH batch ~10 us).
  // Default: a copy kernel in the launch stream reads the pinned slot (stage_copy.h) -- no copy-engine launch
  // and no cross-stream waits, each of which left the GPU idle ~10-15 us (r04j trace).
  if (!side) {
    st.seq = ++x->fence.seq;
    if (srsran_amd::stage_copy_or_record(st.d, st.hd, bytes, stream, nullptr, 0, &x->fence, slot, st.seq) !=
        hipSuccess) {
      return SRSRAN_ERROR;
    }
  } else {
    hipStream_t up = stream;
    if (early_copy) {
      up = x->copy;
      if (st.used) {
        hipStreamWaitEvent(up, st.done, 0);
      }
    }
    if (hipMemcpyAsync(st.d, st.h, bytes, hipMemcpyHostToDevice, up) != hipSuccess) {
      return SRSRAN_ERROR;
    }
    hipEventRecord(st.staged, up);
    if (early_copy) {
      hipStreamWaitEvent(stream, st.staged, 0);
    }
  }
  x->used  = true;
  st.used  = true;
  char* ds = st.d;

  // the launches (recorded instead when a UE DL batch defers them, stage_copy.h)
  int ret = SRSRAN_SUCCESS;
  if (nslots) {
    const RmSlot*  slots = (const RmSlot*)ds;
    const Widen8*  wd    = (const Widen8*)(ds + off_wide);
    const uint32_t nwide = (uint32_t)wide.size();
    if (srsran_amd::launch_or_record([=] {
          const hipError_t e = b8 ? rm8_rx_slots_launch(slots, nslots, max_len, stream)
                                  : rm_rx_launch(slots, nslots, max_len, max_e, stream);
          return e != hipSuccess ? e : widen8_launch(wd, nwide, max_wide, stream);
        }) != hipSuccess) {
      ret = SRSRAN_ERROR;
    }
    const int n_end = q->max_iterations > 0 ? (int)q->max_iterations : 1;
    for (size_t g = 0; g < groups.size() && ret == SRSRAN_SUCCESS; g++) {
      const uint32_t first  = groups[g].second;
      const uint32_t count  = (g + 1 < groups.size() ? groups[g + 1].second : (uint32_t)cbs.size()) - first;
      const uint32_t K      = groups[g].first;
      const TdecCb*  dcb    = (const TdecCb*)(ds + off_cbs) + first;
      const bool     dec8   = b8 && srsran_tdec_autoimp_get_subblocks_8bit(K) >= 16;
      uint8_t*       cbout  = x->d_cbout;
      uint8_t*       noi    = x->d_noi;
      uint8_t*       crc_ok = x->d_crc_ok;
      if (srsran_amd::launch_or_record([=] {
            const int r = dec8 ? tdec8_sch_enqueue(K, dcb, count, cbout, SCH_SLOT_BYTES, noi, crc_ok, n_end, stream)
                               : tdec_sch_enqueue(K, dcb, count, cbout, SCH_SLOT_BYTES, noi, crc_ok, n_end, stream);
            return r == SRSRAN_SUCCESS ? hipSuccess : hipErrorLaunchFailure;
          }) != hipSuccess) {
        ret = SRSRAN_ERROR;
      }
    }
  }
  const SchTb* d_tbs = (const SchTb*)(ds + off_tb);
  if (ret == SRSRAN_SUCCESS &&
      srsran_amd::launch_or_record([=] { return tb_launch(d_tbs, ntb, max_tbs, stream); }) != hipSuccess) {
    ret = SRSRAN_ERROR;
  }
  if (side) {
    hipEventRecord(x->done, stream);
    hipEventRecord(st.done, stream);
  }
  return ret;
}

}  // namespace

extern "C" {

// ---------------- cbsegm.c:62-151 ----------------
int srsran_cbsegm_cbsize(uint32_t index)
{
  if (index >= SRSRAN_NOF_TC_CB_SIZES) {
    return SRSRAN_ERROR;
  }
  // 36.212 Table 5.1.3-3: K = 40..512 step 8, ..1024 step 16, ..2048 step 32, ..6144 step 64
  if (index < 60) {
    return 40 + 8 * (int)index;
  }
  if (index < 92) {
    return 512 + 16 * (int)(index - 59);
  }
  if (index < 124) {
    return 1024 + 32 * (int)(index - 91);
  }
  return 2048 + 64 * (int)(index - 123);
}

int srsran_cbsegm_cbindex(uint32_t long_cb)
{
  for (uint32_t j = 0; j < SRSRAN_NOF_TC_CB_SIZES; j++) {
    if ((uint32_t)srsran_cbsegm_cbsize(j) >= long_cb) {
      return (int)j;
    }
  }
  return SRSRAN_ERROR;
}

bool srsran_cbsegm_cbsize_isvalid(uint32_t size)
{
  const int j = srsran_cbsegm_cbindex(size);
  return j >= 0 && (uint32_t)srsran_cbsegm_cbsize((uint32_t)j) == size;
}

int srsran_cbsegm(srsran_cbsegm_t* s, uint32_t tbs)
{
  if (!s) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (tbs == 0) {
    memset(s, 0, sizeof(*s));
    return SRSRAN_SUCCESS;
  }
  // 36.212 5.1.2: B = TBS + 24; C blocks of at most Z = 6144 bits, each with its own CRC24B
  const uint32_t B = tbs + 24, Z = SRSRAN_TCOD_MAX_LEN_CB;
  const uint32_t C  = B <= Z ? 1 : (B + (Z - 24) - 1) / (Z - 24);
  const uint32_t Bp = B <= Z ? B : B + 24 * C;
  s->tbs            = tbs;
  s->C              = C;
  const int idx1    = srsran_cbsegm_cbindex((Bp - 1) / C + 1);  // K+ = smallest K with C*K >= B'
  if (idx1 < 0) {
    return SRSRAN_ERROR;
  }
  s->K1     = (uint32_t)srsran_cbsegm_cbsize((uint32_t)idx1);
  s->K1_idx = (uint32_t)idx1;
  if (C == 1) {
    s->K2 = s->K2_idx = s->C2 = 0;
    s->C1                     = 1;
  } else {
    // K- = the next smaller size (cbsegm.c:86-100; idx1 >= 1 whenever C > 1)
    s->K2_idx = (uint32_t)idx1 - 1;
    s->K2     = (uint32_t)srsran_cbsegm_cbsize(s->K2_idx);
    s->C2     = (C * s->K1 - Bp) / (s->K1 - s->K2);
    s->C1     = C - s->C2;
  }
  s->L_tb = 24;
  s->L_cb = 24;
  s->F    = s->C1 * s->K1 + s->C2 * s->K2 - Bp;
  return SRSRAN_SUCCESS;
}

// ---------------- crc.c:69-195 (host utility, table driven) ----------------
int srsran_crc_set_init(srsran_crc_t* h, uint64_t init_value)
{
  h->crcinit = init_value;
  return init_value == (init_value & h->crcmask) ? 0 : -1;
}

int srsran_crc_init(srsran_crc_t* h, uint32_t poly, int order)
{
  if (!h || order < 1 || order > 32) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  h->polynom    = (int)poly;
  h->order      = order;
  h->crcmask    = ((((uint64_t)1 << (order - 1)) - 1) << 1) | 1;
  h->crchighbit = (uint64_t)1 << (order - 1);
  h->crcinit    = 0;
  for (uint32_t i = 0; i < 256; i++) {  // CRC register after shifting byte i in (MSB first)
    uint64_t reg = order >= 8 ? (uint64_t)i << (order - 8) : (uint64_t)i >> (8 - order);
    for (int k = 0; k < 8; k++) {
      reg = (reg & h->crchighbit) ? ((reg << 1) ^ poly) : (reg << 1);
    }
    h->table[i] = reg & h->crcmask;
  }
  return 0;
}

uint32_t srsran_crc_checksum_byte(srsran_crc_t* h, const uint8_t* data, int len)
{
  uint64_t crc = 0;
  for (int i = 0; i < len / 8; i++) {
    const uint32_t idx = h->order >= 8 ? (uint32_t)((crc >> (h->order - 8)) & 0xff) ^ data[i]
                                       : (uint32_t)((crc << (8 - h->order)) & 0xff) ^ data[i];
    crc = (crc << 8) ^ h->table[idx];
  }
  h->crcinit = crc;
  return (uint32_t)(crc & h->crcmask);
}

bool srsran_crc_match_byte(srsran_crc_t* h, uint8_t* data, int len)
{
  return srsran_crc_checksum_byte(h, data, len + h->order) == 0;
}

uint32_t srsran_crc_attach_byte(srsran_crc_t* h, uint8_t* data, int len)
{
  const uint32_t c = srsran_crc_checksum_byte(h, data, len);
  for (int i = 0; i < h->order / 8; i++) {
    data[len / 8 + (h->order / 8 - i - 1)] = (uint8_t)(c >> (8 * i));
  }
  return c;
}

uint32_t srsran_mod_bits_x_symbol(srsran_mod_t mod)
{
  switch (mod) {
    case SRSRAN_MOD_BPSK:
      return 1;
    case SRSRAN_MOD_QPSK:
      return 2;
    case SRSRAN_MOD_16QAM:
      return 4;
    case SRSRAN_MOD_64QAM:
      return 6;
    case SRSRAN_MOD_256QAM:
      return 8;
    default:
      return 0;
  }
}

// ---------------- rm_turbo.c:276-483 ----------------
void srsran_rm_turbo_gentables(void)
{
  // device tables are built lazily per (K, rv, layout) on first use and kept for the process
}

void srsran_rm_turbo_free_tables(void) {}

namespace {
std::mutex g_rm_mu;
struct RmCtx {  // one per device: the host-synchronous srsran_rm_turbo_rx_lut_ scratch
  hipStream_t stream = nullptr;
  int16_t*    d_in   = nullptr;
  size_t      in_cap = 0;
  int16_t*    d_out  = nullptr;
  RmSlot*     d_slot = nullptr;
  uint8_t*    d_zero = nullptr;
};
std::map<int, RmCtx> g_rm;
}  // namespace

int srsran_rm_turbo_rx_lut_(int16_t* input,
                            int16_t* output,
                            uint32_t in_len,
                            uint32_t cb_idx,
                            uint32_t rv_idx,
                            bool     enable_input_tdec)
{
  if (rv_idx >= 4 || cb_idx >= SRSRAN_NOF_TC_CB_SIZES) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (!input || !output) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  InvTable t;
  if (!inv_table(cb_idx, rv_idx, enable_input_tdec, &t)) {
    fprintf(stderr, "[srsran_rm_turbo] no HIP device available\n");
    return SRSRAN_ERROR;
  }
  std::lock_guard<std::mutex> lk(g_rm_mu);
  RmCtx&                      c = g_rm[cur_dev()];
  if (!c.stream) {
    if (hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc((void**)&c.d_out, (size_t)SOFTBUFFER_SIZE * sizeof(int16_t)) != hipSuccess ||
        hipMalloc((void**)&c.d_slot, sizeof(RmSlot)) != hipSuccess || hipMalloc((void**)&c.d_zero, 8) != hipSuccess ||
        hipMemset(c.d_zero, 0, 8) != hipSuccess) {
      return SRSRAN_ERROR;
    }
  }
  if (!grow_dev((void**)&c.d_in, &c.in_cap, std::max<size_t>(in_len, 1) * sizeof(int16_t))) {
    return SRSRAN_ERROR;
  }
  RmSlot s;
  s.e    = c.d_in;
  s.sb   = c.d_out;
  s.skip = c.d_zero;
  s.inv  = t.d;
  s.E    = in_len;
  s.len  = t.len;
  s.N    = t.N;
  s.overwrite = 0;
  hipMemcpyAsync(c.d_in, input, (size_t)in_len * sizeof(int16_t), hipMemcpyHostToDevice, c.stream);
  hipMemcpyAsync(c.d_out, output, t.len * sizeof(int16_t), hipMemcpyHostToDevice, c.stream);
  hipMemcpyAsync(c.d_slot, &s, sizeof(s), hipMemcpyHostToDevice, c.stream);
  if (rm_rx_launch(c.d_slot, 1, t.len, in_len, c.stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  hipMemcpyAsync(output, c.d_out, t.len * sizeof(int16_t), hipMemcpyDeviceToHost, c.stream);
  return hipStreamSynchronize(c.stream) == hipSuccess ? SRSRAN_SUCCESS : SRSRAN_ERROR;
}

int srsran_rm_turbo_rx_lut(int16_t* input, int16_t* output, uint32_t in_len, uint32_t cb_idx, uint32_t rv_idx)
{
  return srsran_rm_turbo_rx_lut_(input, output, in_len, cb_idx, rv_idx, true);
}

// rm_turbo.c:447-483 (the SSE 8-bit path of an AVX2 build, :586-687): output[deinter[i % (3K + 12)]] += input[i]
// with int8 wrap-around, on the sub-block layout of the 8-bit decoder that takes K
// (srsran_tdec_autoimp_get_subblocks_8bit: 32 / 16 / 8 sub-blocks, natural below K = 408)
int srsran_rm_turbo_rx_lut_8bit(int8_t* input, int8_t* output, uint32_t in_len, uint32_t cb_idx, uint32_t rv_idx)
{
  if (rv_idx >= 4 || cb_idx >= SRSRAN_NOF_TC_CB_SIZES || !input || !output) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  const uint32_t K = (uint32_t)srsran_cbsegm_cbsize(cb_idx);
  InvTable       t;
  if (!inv_table_nsb(cb_idx, rv_idx, srsran_tdec_autoimp_get_subblocks_8bit(K), &t)) {
    fprintf(stderr, "[srsran_rm_turbo] no HIP device available\n");
    return SRSRAN_ERROR;
  }
  std::lock_guard<std::mutex> lk(g_rm_mu);
  RmCtx&                      c = g_rm[cur_dev()];
  if (!c.stream) {
    if (hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc((void**)&c.d_out, (size_t)SOFTBUFFER_SIZE * sizeof(int16_t)) != hipSuccess ||
        hipMalloc((void**)&c.d_slot, sizeof(RmSlot)) != hipSuccess || hipMalloc((void**)&c.d_zero, 8) != hipSuccess ||
        hipMemset(c.d_zero, 0, 8) != hipSuccess) {
      return SRSRAN_ERROR;
    }
  }
  if (!grow_dev((void**)&c.d_in, &c.in_cap, std::max<size_t>(in_len, 1))) {
    return SRSRAN_ERROR;
  }
  int8_t* d_in  = (int8_t*)c.d_in;
  int8_t* d_out = (int8_t*)c.d_out;
  hipMemcpyAsync(d_in, input, in_len, hipMemcpyHostToDevice, c.stream);
  hipMemcpyAsync(d_out, output, t.len, hipMemcpyHostToDevice, c.stream);
  if (srsran_amd::rm8_rx_launch(d_in, d_out, t.d, in_len, t.len, t.N, c.stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  hipMemcpyAsync(output, d_out, t.len, hipMemcpyDeviceToHost, c.stream);
  return hipStreamSynchronize(c.stream) == hipSuccess ? SRSRAN_SUCCESS : SRSRAN_ERROR;
}

// ---------------- softbuffer.c:36-178 ----------------
int srsran_softbuffer_rx_init(srsran_softbuffer_rx_t* q, uint32_t nof_prb)
{
  if (nof_prb == 0 || nof_prb > SRSRAN_MAX_PRB) {
    return SRSRAN_ERROR;
  }
  const uint32_t max_cb = (uint32_t)kTbsMaxIdx[nof_prb - 1] / (SRSRAN_TCOD_MAX_LEN_CB - 24) + 1;
  return srsran_softbuffer_rx_init_guru(q, max_cb, SOFTBUFFER_SIZE);
}

int srsran_softbuffer_rx_init_guru(srsran_softbuffer_rx_t* q, uint32_t max_cb, uint32_t max_cb_size)
{
  if (!q) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  memset(q, 0, sizeof(*q));
  if (!have_gpu()) {
    fprintf(stderr, "[srsran_softbuffer] no HIP device available\n");
    return SRSRAN_ERROR;
  }
  SbGpu* g       = new SbGpu();
  g->stride      = (max_cb_size + 3) & ~3u;  // keeps every buffer 8-byte aligned
  g->data_stride = max_cb_size / 8;
  hipGetDevice(&g->dev);
  q->max_cb      = max_cb;
  q->max_cb_size = max_cb_size;
  q->gpu         = g;
  q->buffer_f    = (int16_t**)calloc(max_cb ? max_cb : 1, sizeof(int16_t*));
  q->data        = (uint8_t**)calloc(max_cb ? max_cb : 1, sizeof(uint8_t*));
  q->cb_crc      = (bool*)calloc(max_cb ? max_cb : 1, sizeof(bool));
  if (!q->buffer_f || !q->data || !q->cb_crc ||
      !(g->buf_bytes = std::max<size_t>((size_t)max_cb * g->stride * sizeof(int16_t), 8),
        g->d_buf     = (short*)sb_arena_alloc(g->buf_bytes, &g->buf_dev)) ||
      hipMalloc((void**)&g->d_data, std::max<size_t>((size_t)max_cb * g->data_stride, 8)) != hipSuccess ||
      hipMalloc((void**)&g->d_flags, max_cb + 1) != hipSuccess) {
    srsran_softbuffer_rx_free(q);
    return SRSRAN_ERROR;
  }
  for (uint32_t i = 0; i < max_cb; i++) {
    q->buffer_f[i] = g->d_buf + (size_t)i * g->stride;
    q->data[i]     = g->d_data + (size_t)i * g->data_stride;
  }
  srsran_softbuffer_rx_reset(q);
  return SRSRAN_SUCCESS;
}

void srsran_softbuffer_rx_reset_cb(srsran_softbuffer_rx_t* q, uint32_t nof_cb)
{
  if (!q || !q->gpu) {
    return;
  }
  SbGpu*   g = (SbGpu*)q->gpu;
  DevScope ds(g->dev);
  nof_cb   = std::min(nof_cb, q->max_cb);
  hipDeviceSynchronize();  // the buffers may still be in use by an asynchronous batch
  if (nof_cb) {
    hipMemset(g->d_buf, 0, (size_t)nof_cb * g->stride * sizeof(int16_t));
    hipMemset(g->d_data, 0, (size_t)nof_cb * g->data_stride);
  }
  hipMemset(g->d_flags, 0, q->max_cb + 1);
  hipDeviceSynchronize();
  memset(q->cb_crc, 0, q->max_cb * sizeof(bool));
  q->tb_crc = false;
}

void srsran_softbuffer_rx_reset(srsran_softbuffer_rx_t* q)
{
  if (q) {
    srsran_softbuffer_rx_reset_cb(q, q->max_cb);
  }
}

void srsran_softbuffer_rx_reset_tbs(srsran_softbuffer_rx_t* q, uint32_t tbs)
{
  if (q) {
    const uint32_t nof_cb = (tbs + 24) / (SRSRAN_TCOD_MAX_LEN_CB - 24) + 1;
    srsran_softbuffer_rx_reset_cb(q, std::min(nof_cb, q->max_cb));
  }
}

void srsran_softbuffer_rx_reset_cb_crc(srsran_softbuffer_rx_t* q, uint32_t nof_cb)
{
  if (!q || nof_cb == 0 || !q->gpu) {
    return;
  }
  nof_cb = std::min(nof_cb, q->max_cb);
  DevScope ds(((SbGpu*)q->gpu)->dev);
  hipDeviceSynchronize();
  hipMemset(((SbGpu*)q->gpu)->d_flags, 0, nof_cb);
  hipDeviceSynchronize();
  memset(q->cb_crc, 0, nof_cb * sizeof(bool));
}

int srsran_softbuffer_rx_sync(srsran_softbuffer_rx_t* q)
{
  if (!q || !q->gpu) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  std::vector<uint8_t> f(q->max_cb + 1);
  DevScope             ds(((SbGpu*)q->gpu)->dev);
  hipDeviceSynchronize();
  if (hipMemcpy(f.data(), ((SbGpu*)q->gpu)->d_flags, f.size(), hipMemcpyDeviceToHost) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  for (uint32_t i = 0; i < q->max_cb; i++) {
    q->cb_crc[i] = f[i] != 0;
  }
  q->tb_crc = f[q->max_cb] != 0;
  return SRSRAN_SUCCESS;
}

void srsran_softbuffer_rx_free(srsran_softbuffer_rx_t* q)
{
  if (!q) {
    return;
  }
  SbGpu* g = (SbGpu*)q->gpu;
  if (g) {
    // the owning device must be idle before the arena slot can be handed out again
    DevScope ds(g->dev);
    hipDeviceSynchronize();
    sb_arena_free(g->d_buf, g->buf_bytes, g->buf_dev);
    hipFree(g->d_data);
    hipFree(g->d_flags);
    delete g;
  }
  free(q->buffer_f);
  free(q->data);
  free(q->cb_crc);
  memset(q, 0, sizeof(*q));
}

int srsran_softbuffer_rx_gpu_arena(int enable, size_t bytes)
{
  std::lock_guard<std::mutex> lk(g_arena_mu);
  g_arena_on = enable != 0;
  if (bytes) {
    g_arena_bytes = bytes;
  }
  return SRSRAN_SUCCESS;
}

const void* srsran_softbuffer_rx_gpu_ptr(const srsran_softbuffer_rx_t* q)
{
  return q && q->gpu ? ((const SbGpu*)q->gpu)->d_buf : nullptr;
}

// ---------------- sch.c:140-230 ----------------
int srsran_sch_init(srsran_sch_t* q)
{
  if (!q) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  memset(q, 0, sizeof(*q));
  if (srsran_tdec_init(&q->decoder, SRSRAN_TCOD_MAX_LEN_CB)) {
    return SRSRAN_ERROR;
  }
  q->max_iterations = 10;  // SRSRAN_PDSCH_MAX_TDEC_ITERS (sch.c:36)
  SchCtx* x         = new SchCtx();
  q->gpu            = x;
  if (hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&x->copy, hipStreamNonBlocking) != hipSuccess ||
      srsran_amd::ring_event_create(&x->done) != hipSuccess || !init_ring(x) ||
      hipMalloc((void**)&x->d_data, kDataCap) != hipSuccess || hipMalloc((void**)&x->d_res, 16) != hipSuccess ||
      hipMalloc((void**)&x->d_avg, 16) != hipSuccess ||
      hipHostMalloc((void**)&x->h_io, 256, hipHostMallocDefault) != hipSuccess ||
      hipMalloc((void**)&x->d_zero, 8) != hipSuccess || hipMemset(x->d_zero, 0, 8) != hipSuccess) {
    srsran_sch_free(q);
    return SRSRAN_ERROR;
  }
  return SRSRAN_SUCCESS;
}

void srsran_sch_free(srsran_sch_t* q)
{
  if (!q) {
    return;
  }
  SchCtx* x = (SchCtx*)q->gpu;
  if (x) {
    srsran_amd::handoff_drain(x->ho);  // batches on the caller's streams
    if (x->stream) {
      hipStreamSynchronize(x->stream);
      hipStreamDestroy(x->stream);
    }
    if (x->copy) {
      hipStreamSynchronize(x->copy);
      hipStreamDestroy(x->copy);
    }
    if (x->done) {
      hipEventDestroy(x->done);
    }
    for (StageSlot& st : x->ring) {
      if (st.staged) {
        hipEventDestroy(st.staged);
      }
      if (st.done) {
        hipEventDestroy(st.done);
      }
      hipHostFree(st.h);
      hipFree(st.d);
    }
    srsran_amd::stage_fence_free(x->fence);
    srsran_amd::handoff_free(x->ho);
    hipFree(x->d_cbout);
    hipFree(x->d_noi);
    hipFree(x->d_crc_ok);
    hipFree(x->d_e);
    hipFree(x->d_data);
    hipFree(x->d_res);
    hipFree(x->d_avg);
    hipHostFree(x->h_io);
    hipFree(x->d_zero);
    hipFree(x->d_ul);
    hipFree(x->d_uldesc);
    hipHostFree(x->h_uldesc);
    if (x->uldesc_used) {
      hipEventDestroy(x->uldesc_used);
    }
    hipFree(x->d_uci);
    hipFree(x->d_ubs);
    hipHostFree(x->h_ubs);
    hipFree(x->d_enc);
    hipFree(x->d_wide);
    delete x;
  }
  srsran_tdec_free(&q->decoder);
  memset(q, 0, sizeof(*q));
}

void srsran_sch_set_max_noi(srsran_sch_t* q, uint32_t max_iterations)
{
  if (q) {
    q->max_iterations = max_iterations ? max_iterations : 10;
  }
}

float srsran_sch_last_noi(srsran_sch_t* q) { return q ? q->avg_iterations : 0.0f; }

// ---------------- sch.c:509-609 (host-synchronous) ----------------
// decode_tb of one TB, host-synchronous; LLRs from the host (e_bits) or already on the device (d_e_bits)
static int dlsch_decode_sync(srsran_sch_t*       q,
                             srsran_pdsch_cfg_t* cfg,
                             const int16_t*      e_bits,
                             const int16_t*      d_e_bits,
                             uint8_t*            data,
                             int                 tb_idx,
                             uint32_t            nof_layers)
{
  if (!q || !q->gpu || !cfg || tb_idx < 0 || tb_idx >= SRSRAN_MAX_CODEWORDS) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  const uint32_t  Nl = nof_layers != cfg->grant.nof_tb ? 2 : 1;
  srsran_cbsegm_t s;
  if (srsran_cbsegm(&s, (uint32_t)cfg->grant.tb[tb_idx].tbs)) {
    fprintf(stderr, "[srsran_sch] Error computing Codeword (%d) segmentation for TBS=%d\n", tb_idx,
            cfg->grant.tb[tb_idx].tbs);
    return SRSRAN_ERROR;
  }
  const uint32_t          Qm = srsran_mod_bits_x_symbol(cfg->grant.tb[tb_idx].mod) * Nl;
  srsran_softbuffer_rx_t* sb = cfg->softbuffers.rx[tb_idx];
  if (!data || !sb || (!e_bits && !d_e_bits) || Qm == 0) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (s.tbs == 0 || s.C == 0) {
    return SRSRAN_SUCCESS;
  }
  if (s.F || s.C > sb->max_cb) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (s.C > SRSRAN_MAX_CODEBLOCKS) {
    return SRSRAN_ERROR;
  }
  SchCtx*        x   = (SchCtx*)q->gpu;
  const uint32_t nbe = cfg->grant.tb[tb_idx].nof_bits;
  const size_t   esz = q->llr_is_8bit ? sizeof(int8_t) : sizeof(int16_t);  // e_bits are int8 with llr_is_8bit
  hipStreamSynchronize(x->stream);
  if (!d_e_bits && !grow_dev((void**)&x->d_e, &x->e_cap, std::max<size_t>(nbe, 1) * esz)) {
    return SRSRAN_ERROR;
  }
  // the host cb_crc mirror is authoritative for the synchronous API
  SbGpu* g = (SbGpu*)sb->gpu;
  for (uint32_t i = 0; i < s.C; i++) {
    x->h_io[i] = sb->cb_crc[i] ? 1 : 0;
  }
  hipMemcpyAsync(g->d_flags, x->h_io, s.C, hipMemcpyHostToDevice, x->stream);
  if (!d_e_bits) {
    hipMemcpyAsync(x->d_e, e_bits, (size_t)nbe * esz, hipMemcpyHostToDevice, x->stream);
  }
  uint32_t end = 0;  // bytes of `data` the reference writes (sch.c:425-431, 476-480)
  for (uint32_t cb = 0; cb < s.C; cb++) {
    const uint32_t K    = cb < s.C1 ? s.K1 : s.K2;
    const uint32_t rlen = s.C == 1 ? K : K - 24;
    end                 = std::max(end, cb * rlen / 8 + (sb->cb_crc[cb] ? rlen / 8 : K / 8));
  }
  srsran_dlsch_gpu_tb_t tb;
  tb.tbs        = (uint32_t)cfg->grant.tb[tb_idx].tbs;
  tb.Qm         = Qm;
  tb.rv         = (uint32_t)cfg->grant.tb[tb_idx].rv;
  tb.nof_e_bits = nbe;
  tb.d_e_bits   = d_e_bits ? d_e_bits : x->d_e;
  tb.d_data     = x->d_data;
  tb.softbuffer = sb;
  tb.new_data   = 0;
  hipStreamSynchronize(x->stream);  // h_io is reused below
  int ret = enqueue_batch(q, 1, &tb, x->d_res, x->d_avg, x->stream);
  if (ret != SRSRAN_SUCCESS) {
    hipStreamSynchronize(x->stream);
    return ret;
  }
  uint8_t* h_flags = x->h_io;
  int32_t* h_res   = (int32_t*)(x->h_io + 128);
  float*   h_avg   = (float*)(x->h_io + 136);
  hipMemcpyAsync(data, x->d_data, end, hipMemcpyDeviceToHost, x->stream);
  hipMemcpyAsync(h_flags, g->d_flags, s.C, hipMemcpyDeviceToHost, x->stream);
  hipMemcpyAsync(h_flags + 64, g->d_flags + sb->max_cb, 1, hipMemcpyDeviceToHost, x->stream);
  hipMemcpyAsync(h_res, x->d_res, sizeof(int32_t), hipMemcpyDeviceToHost, x->stream);
  hipMemcpyAsync(h_avg, x->d_avg, sizeof(float), hipMemcpyDeviceToHost, x->stream);
  if (hipStreamSynchronize(x->stream) != hipSuccess) {
    fprintf(stderr, "[srsran_sch] decode failed: %s\n", hipGetErrorString(hipGetLastError()));
    return SRSRAN_ERROR;
  }
  for (uint32_t i = 0; i < s.C; i++) {
    sb->cb_crc[i] = h_flags[i] != 0;
  }
  sb->tb_crc        = h_flags[64] != 0;
  q->avg_iterations = *h_avg;
  return *h_res;
}

int srsran_dlsch_decode2(srsran_sch_t*       q,
                         srsran_pdsch_cfg_t* cfg,
                         int16_t*            e_bits,
                         uint8_t*            data,
                         int                 tb_idx,
                         uint32_t            nof_layers)
{
  return dlsch_decode_sync(q, cfg, e_bits, nullptr, data, tb_idx, nof_layers);
}

/* added: srsran_dlsch_decode2 with the LLRs already in device memory (complete before the call) */
int srsran_dlsch_decode2_dev(srsran_sch_t*       q,
                             srsran_pdsch_cfg_t* cfg,
                             const int16_t*      d_e_bits,
                             uint8_t*            data,
                             int                 tb_idx,
                             uint32_t            nof_layers)
{
  if (!d_e_bits) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  return dlsch_decode_sync(q, cfg, nullptr, d_e_bits, data, tb_idx, nof_layers);
}

int srsran_dlsch_decode(srsran_sch_t* q, srsran_pdsch_cfg_t* cfg, int16_t* e_bits, uint8_t* data)
{
  return srsran_dlsch_decode2(q, cfg, e_bits, data, 0, 1);
}

int srsran_dlsch_gpu_decode_batch(srsran_sch_t*                q,
                                  uint32_t                     nof_tb,
                                  const srsran_dlsch_gpu_tb_t* tbs,
                                  int32_t*                     d_result,
                                  float*                       d_avg_noi,
                                  void*                        stream)
{
  if (!q || !q->gpu || (nof_tb && (!tbs || !d_result || !d_avg_noi))) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (nof_tb == 0) {
    return SRSRAN_SUCCESS;
  }
  return enqueue_batch(q, nof_tb, tbs, d_result, d_avg_noi, (hipStream_t)stream);
}

}  // extern "C"

namespace srsran_amd {
int dlsch_gpu_decode_batch_early_copy(srsran_sch_t* q, uint32_t nof_tb, const srsran_dlsch_gpu_tb_t* tbs,
                                      int32_t* d_result, float* d_avg_noi, void* stream)
{
  if (!q || !q->gpu || (nof_tb && (!tbs || !d_result || !d_avg_noi))) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (nof_tb == 0) {
    return SRSRAN_SUCCESS;
  }
  return enqueue_batch(q, nof_tb, tbs, d_result, d_avg_noi, (hipStream_t)stream, true);
}

int dlsch_gpu_decode_batch_limits(srsran_sch_t* q, uint32_t nof_tb, const srsran_dlsch_gpu_tb_t* tbs,
                                  const uint32_t* max_noi, int32_t* d_result, float* d_avg_noi, void* stream)
{
  if (!q || !q->gpu || (nof_tb && (!tbs || !max_noi || !d_result || !d_avg_noi))) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (nof_tb == 0) {
    return SRSRAN_SUCCESS;
  }
  // distinct limits in first-appearance order; 0 keeps the limit in force, as pdsch.c:815-817 does
  std::vector<uint32_t> lim(nof_tb);
  std::vector<uint32_t> order;
  for (uint32_t i = 0; i < nof_tb; i++) {
    lim[i] = max_noi[i] ? max_noi[i] : (i ? lim[i - 1] : q->max_iterations);
    if (std::find(order.begin(), order.end(), lim[i]) == order.end()) {
      order.push_back(lim[i]);
    }
  }
  if (order.size() == 1) {
    srsran_sch_set_max_noi(q, order[0]);
    return enqueue_batch(q, nof_tb, tbs, d_result, d_avg_noi, (hipStream_t)stream, true);
  }
  std::vector<srsran_dlsch_gpu_tb_t> sub;
  std::vector<uint32_t>              idx;
  for (uint32_t l : order) {
    sub.clear();
    idx.clear();
    for (uint32_t i = 0; i < nof_tb; i++) {
      if (lim[i] == l) {
        sub.push_back(tbs[i]);
        idx.push_back(i);
      }
    }
    srsran_sch_set_max_noi(q, l);
    const int r = enqueue_batch(q, (uint32_t)sub.size(), sub.data(), d_result, d_avg_noi, (hipStream_t)stream, true,
                                idx.data());
    if (r != SRSRAN_SUCCESS) {
      return r;
    }
  }
  srsran_sch_set_max_noi(q, lim[nof_tb - 1]);  // as after the last TB's sequential decode
  return SRSRAN_SUCCESS;
}
}  // namespace srsran_amd

extern "C" {

// ---------------- UCI on PUSCH, host side ----------------
// Offset tables of 36.213 Tables 8.6.3-1/-2/-3 with the reference's out-of-range behaviour
// (sch.c:43-95: an error message and the first valid entry).
static float beta_harq(uint32_t i)
{
  static const float t[15] = {2.0f, 2.5f, 3.125f, 4.0f, 5.0f, 6.25f, 8.0f, 10.0f, 12.625f, 15.875f, 20.0f, 31.0f,
                              50.0f, 80.0f, 126.0f};
  if (i < 15) {
    return t[i];
  }
  fprintf(stderr, "[srsran_sch] Invalid I_offset_ack %u (min: 0, max: 14)\n", i);
  return t[0];
}

static float beta_ri(uint32_t i)
{
  static const float t[13] = {1.25f, 1.625f, 2.0f, 2.5f, 3.125f, 4.0f, 5.0f, 6.25f, 8.0f, 10.0f, 12.625f, 15.875f,
                              20.0f};
  if (i < 13) {
    return t[i];
  }
  fprintf(stderr, "[srsran_sch] Invalid I_offset_ri %u (min: 0, max: 12)\n", i);
  return t[0];
}

static float beta_cqi(uint32_t i)
{
  static const float t[16] = {-1.0f, -1.0f, 1.125f, 1.25f, 1.375f, 1.625f, 1.75f, 2.0f, 2.25f, 2.5f, 2.875f,
                              3.125f, 3.5f, 4.0f, 5.0f, 6.25f};
  if (i > 1 && i < 16) {
    return t[i];
  }
  fprintf(stderr, "[srsran_sch] Invalid I_offset_cqi %u (min: 2, max: 15)\n", i);
  return t[2];
}

float srsran_sch_beta_cqi(uint32_t I_cqi) { return I_cqi < 16 ? beta_cqi(I_cqi) : 0.0f; }
float srsran_sch_beta_ack(uint32_t I_harq) { return I_harq < 16 ? beta_harq(I_harq) : 0.0f; }

// the first index whose offset reaches beta (sch.c:108-136, 16 indices through the getters)
uint32_t srsran_sch_find_Ioffset_ack(float beta)
{
  for (uint32_t i = 0; i < 16; i++) {
    if (beta_harq(i) >= beta) {
      return i;
    }
  }
  return 0;
}
uint32_t srsran_sch_find_Ioffset_ri(float beta)
{
  for (uint32_t i = 0; i < 16; i++) {
    if (beta_ri(i) >= beta) {
      return i;
    }
  }
  return 0;
}
uint32_t srsran_sch_find_Ioffset_cqi(float beta)
{
  for (uint32_t i = 0; i < 16; i++) {
    if (beta_cqi(i) >= beta) {
      return i;
    }
  }
  return 0;
}

uint32_t srsran_uci_cfg_total_ack(const srsran_uci_cfg_t* uci_cfg)
{
  uint32_t n = 0;  // uci.c:716-723
  for (uint32_t i = 0; i < SRSRAN_MAX_CARRIERS; i++) {
    n += uci_cfg->ack[i].nof_acks;
  }
  return n;
}

// Q'_ACK / Q'_RI, 36.212 5.2.2.6 (uci.c:414-440); float arithmetic in the reference's order
static uint32_t qprime_ri_ack(uint32_t K, uint32_t L_prb, uint32_t nof_symb, uint32_t O, uint32_t O_cqi, float beta)
{
  if (beta < 0) {
    return (uint32_t)-1;
  }
  if (K == 0) {  // no UL-SCH: 5.2.4.1
    K = O_cqi <= 11 ? O_cqi : O_cqi + 8;
  }
  if (K == 0) {
    return 0;
  }
  const uint32_t x = (uint32_t)ceilf((float)O * (float)L_prb * (float)SRSRAN_NRE * (float)nof_symb * beta / (float)K);
  return std::min(x, 4 * L_prb * SRSRAN_NRE);
}

// Q'_CQI (uci.c:170-186)
static uint32_t qprime_cqi(uint32_t K, uint32_t L_prb, uint32_t nof_symb, uint32_t O, float beta, uint32_t Q_prime_ri)
{
  const uint32_t L = O < 11 ? 0 : 8;
  uint32_t       x = 999999;
  if (K > 0) {
    x = (uint32_t)ceilf((float)(O + L) * (float)L_prb * (float)SRSRAN_NRE * (float)nof_symb * beta / (float)K);
  }
  return std::min(x, L_prb * SRSRAN_NRE * nof_symb - Q_prime_ri);
}

uint32_t srsran_qprime_cqi_ext(uint32_t L_prb, uint32_t nof_symbols, uint32_t tbs, float beta)
{
  return qprime_cqi(tbs, L_prb, nof_symbols, 20 + 8, beta, 0);  // O = SRSRAN_UCI_CQI_CODED_PUCCH_B + 8
}

uint32_t srsran_qprime_ack_ext(uint32_t L_prb, uint32_t nof_symbols, uint32_t tbs, uint32_t nof_ack, float beta)
{
  return qprime_ri_ack(tbs, L_prb, nof_symbols, nof_ack, 0, beta);
}

// ---- CQI report sizes and fields, 36.212 Tables 5.2.2.6.2-1/-2, 5.2.3.3.1-1/-2 (cqi.c:41-384) ----
static uint32_t bits_get(const uint8_t** p, uint32_t n)  // srsran_bit_pack: MSB first
{
  uint32_t v = 0;
  for (uint32_t i = 0; i < n; i++) {
    v = (v << 1) | ((*p)[i] & 1u);
  }
  *p += n;
  return v;
}

static void bits_put(uint32_t v, uint8_t** p, uint32_t n)  // srsran_bit_unpack
{
  for (uint32_t i = 0; i < n; i++) {
    (*p)[i] = (uint8_t)((v >> (n - 1 - i)) & 1u);
  }
  *p += n;
}

int srsran_cqi_size(srsran_cqi_cfg_t* cfg)
{
  if (!cfg->data_enable) {
    return (int)cfg->ri_len;
  }
  int size = 0;
  switch (cfg->type) {
    case SRSRAN_CQI_TYPE_WIDEBAND:
      size = 4;
      if (cfg->pmi_present) {
        if (cfg->four_antenna_ports) {
          size += (cfg->rank_is_not_one ? 3 : 0) + 4;
        } else {
          size += cfg->rank_is_not_one ? 3 + 1 : 2;
        }
      }
      break;
    case SRSRAN_CQI_TYPE_SUBBAND_UE:
      size = 4 + (cfg->subband_label_2_bits ? 2 : 1);
      break;
    case SRSRAN_CQI_TYPE_SUBBAND_UE_DIFF:
      size = 4 + 2 + (int)cfg->L;
      break;
    case SRSRAN_CQI_TYPE_SUBBAND_HL:
      size = 4 + 2 * (int)cfg->N;
      if (cfg->rank_is_not_one && cfg->pmi_present) {
        size += 4 + 2 * (int)cfg->N;
      }
      if (cfg->pmi_present) {
        size += cfg->four_antenna_ports ? 4 : cfg->rank_is_not_one ? 1 : 2;
      }
      break;
    default:
      size = SRSRAN_ERROR;
  }
  return size;
}

int srsran_cqi_value_pack(srsran_cqi_cfg_t* cfg, srsran_cqi_value_t* v, uint8_t buff[SRSRAN_CQI_MAX_BITS])
{
  uint8_t* p = buff;
  switch (cfg->type) {
    case SRSRAN_CQI_TYPE_WIDEBAND:
      bits_put(v->wideband.wideband_cqi, &p, 4);
      if (cfg->pmi_present) {
        if (cfg->rank_is_not_one) {
          bits_put(v->wideband.spatial_diff_cqi, &p, 3);
        }
        bits_put(v->wideband.pmi, &p, cfg->four_antenna_ports ? 4 : cfg->rank_is_not_one ? 1 : 2);
      }
      return (int)(p - buff);
    case SRSRAN_CQI_TYPE_SUBBAND_UE:
      bits_put(v->subband_ue.subband_cqi, &p, 4);
      bits_put(v->subband_ue.subband_label, &p, cfg->subband_label_2_bits ? 2 : 1);
      return 4 + (cfg->subband_label_2_bits ? 2 : 1);
    case SRSRAN_CQI_TYPE_SUBBAND_UE_DIFF:  // the reference writes subband_diff_cqi twice (cqi.c:77-85)
      bits_put(v->subband_ue_diff.wideband_cqi, &p, 4);
      bits_put(v->subband_ue_diff.subband_diff_cqi, &p, 2);
      bits_put(v->subband_ue_diff.subband_diff_cqi, &p, cfg->L);
      return 4 + 2 + (int)cfg->L;
    case SRSRAN_CQI_TYPE_SUBBAND_HL: {
      int n = 4 + 2 * (int)cfg->N;
      bits_put(v->subband_hl.wideband_cqi_cw0, &p, 4);
      bits_put(v->subband_hl.subband_diff_cqi_cw0, &p, 2 * cfg->N);
      if (cfg->rank_is_not_one) {
        bits_put(v->subband_hl.wideband_cqi_cw1, &p, 4);
        bits_put(v->subband_hl.subband_diff_cqi_cw1, &p, 2 * cfg->N);
        n += 4 + 2 * (int)cfg->N;
      }
      if (cfg->pmi_present) {
        const uint32_t w = cfg->four_antenna_ports ? 4 : cfg->rank_is_not_one ? 1 : 2;
        bits_put(v->subband_hl.pmi, &p, w);
        n += (int)w;
      }
      return n;
    }
  }
  return -1;
}

int srsran_cqi_value_unpack(srsran_cqi_cfg_t* cfg, uint8_t buff[SRSRAN_CQI_MAX_BITS], srsran_cqi_value_t* v)
{
  const uint8_t* p = buff;
  switch (cfg->type) {
    case SRSRAN_CQI_TYPE_WIDEBAND:
      v->wideband.wideband_cqi = (uint8_t)bits_get(&p, 4);
      if (cfg->pmi_present) {
        if (cfg->rank_is_not_one) {
          v->wideband.spatial_diff_cqi = (uint8_t)bits_get(&p, 3);
        }
        v->wideband.pmi = (uint8_t)bits_get(&p, cfg->four_antenna_ports ? 4 : cfg->rank_is_not_one ? 1 : 2);
      }
      return 4;
    case SRSRAN_CQI_TYPE_SUBBAND_UE:
      v->subband_ue.subband_cqi   = (uint8_t)bits_get(&p, 4);
      v->subband_ue.subband_label = (uint8_t)bits_get(&p, cfg->subband_label_2_bits ? 2 : 1);
      return 4 + (cfg->subband_label_2_bits ? 2 : 1);
    case SRSRAN_CQI_TYPE_SUBBAND_UE_DIFF:  // the L-bit field overwrites the 2-bit one (cqi.c:175-184)
      v->subband_ue_diff.wideband_cqi     = (uint8_t)bits_get(&p, 4);
      v->subband_ue_diff.subband_diff_cqi = (uint8_t)bits_get(&p, 2);
      v->subband_ue_diff.subband_diff_cqi = (uint8_t)bits_get(&p, cfg->L);
      return 4 + 2 + (int)cfg->L;
    case SRSRAN_CQI_TYPE_SUBBAND_HL: {
      int n = 4 + 2 * (int)cfg->N;
      v->subband_hl.wideband_cqi_cw0     = (uint8_t)bits_get(&p, 4);
      v->subband_hl.subband_diff_cqi_cw0 = bits_get(&p, 2 * cfg->N);
      if (cfg->rank_is_not_one) {
        v->subband_hl.wideband_cqi_cw1     = (uint8_t)bits_get(&p, 4);
        v->subband_hl.subband_diff_cqi_cw1 = bits_get(&p, 2 * cfg->N);
        n += 4 + 2 * (int)cfg->N;
      }
      if (cfg->pmi_present) {
        const uint32_t w = cfg->four_antenna_ports ? 4 : cfg->rank_is_not_one ? 1 : 2;
        v->subband_hl.pmi = (uint8_t)bits_get(&p, w);
        n += (int)w;
      }
      return n;
    }
  }
  return -1;
}

// ---------------- UL-SCH receive with UCI (sch.c:994-1193) ----------------
// The host part shared by srsran_ulsch_decode and the batched path: segmentation, sizes, Q'_ACK / Q'_RI.
struct UlsPlan {
  srsran_cbsegm_t s;
  uint32_t        nb, Qm, nsymb, H, rows, nack, ack_Qp, ri_Qp;
  bool            uci, hl_ri, need_c;
};

static int ulsch_plan(srsran_pusch_cfg_t* cfg, UlsPlan* p)
{
  srsran_cbsegm_t& s = p->s;
  if (srsran_cbsegm(&s, (uint32_t)cfg->grant.tb.tbs)) {
    fprintf(stderr, "[srsran_sch] Error computing segmentation for TBS=%d\n", cfg->grant.tb.tbs);
    return SRSRAN_ERROR;
  }
  p->nb       = cfg->grant.tb.nof_bits;
  p->Qm       = srsran_mod_bits_x_symbol(cfg->grant.tb.mod);
  cfg->K_segm = s.C1 * s.K1 + s.C2 * s.K2;
  if (p->Qm == 0) {
    fprintf(stderr, "[srsran_sch] Invalid modulation\n");
    return SRSRAN_ERROR;
  }
  p->nsymb = cfg->grant.nof_symb;
  if (p->nsymb == 0 || p->nsymb > 14 || p->nb % p->Qm || p->Qm > 8) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  p->H                  = p->nb / p->Qm;
  p->rows               = p->H / p->nsymb;
  srsran_cqi_cfg_t& cq  = cfg->uci_cfg.cqi;
  p->nack               = srsran_uci_cfg_total_ack(&cfg->uci_cfg);
  p->uci                = p->nack > 0 || cq.ri_len > 0 || cq.data_enable;
  // ---- uci_decode_ri_ack, host part (sch.c:1023-1120): Q'_ACK, Q'_RI ----
  p->hl_ri = cq.data_enable && cq.type == SRSRAN_CQI_TYPE_SUBBAND_HL && cq.ri_len;
  if (p->hl_ri) {
    cq.rank_is_not_one = false;  // RI = 1 assumed for the RI / ACK sizes (36.212 5.2.4.1)
  }
  const uint32_t cqi_len0 = (uint32_t)srsran_cqi_size(&cq);
  p->ack_Qp = p->ri_Qp = 0;
  if (p->nack > 0) {
    if (p->nack > SRSRAN_UCI_MAX_ACK_BITS) {
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
    float beta = beta_harq(cfg->uci_offset.I_offset_ack);
    if (cfg->grant.tb.tbs == 0) {
      beta /= beta_cqi(cfg->uci_offset.I_offset_cqi);
    }
    p->ack_Qp = qprime_ri_ack(cfg->K_segm, cfg->grant.L_prb, p->nsymb, p->nack, cqi_len0, beta);
  }
  if (cq.ri_len > 0) {
    if (cq.ri_len > 4) {
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
    float beta = beta_ri(cfg->uci_offset.I_offset_ri);
    if (cfg->grant.tb.tbs == 0) {
      beta /= beta_cqi(cfg->uci_offset.I_offset_cqi);
    }
    p->ri_Qp = qprime_ri_ack(cfg->K_segm, cfg->grant.L_prb, p->nsymb, cq.ri_len, cqi_len0, beta);
  }
  // the ACK / RI rows are counted up from the bottom of the interleaver: positions past its top
  // (uci.c:378-386 "Error interleaving") are refused
  if (p->ack_Qp > 4 * p->rows || p->ri_Qp > 4 * p->rows || p->ri_Qp > p->H) {
    fprintf(stderr, "[srsran_sch] UCI does not fit the PUSCH interleaver (Q'_ACK=%u Q'_RI=%u rows=%u)\n", p->ack_Qp,
            p->ri_Qp, p->rows);
    return SRSRAN_ERROR;
  }
  p->need_c = (p->nack == 1 && p->ack_Qp > 0) || (cq.ri_len == 1 && p->ri_Qp > 0);
  return SRSRAN_SUCCESS;
}

// The de-interleaver descriptor: it skips the RI cells, column set[c] holding the RI indices
// q = 3c mod 4 (mod 4)
static UlDeint ulsch_deint_desc(int16_t* d_q, int16_t* d_g, const UlsPlan& p)
{
  UlDeint d = {d_q, d_g, p.rows, p.nsymb, p.Qm, {}, -1};
  if (p.ri_Qp > 0) {
    static const uint8_t kRiNorm[4] = {1, 4, 7, 10}, kRiExt[4] = {0, 3, 5, 8};
    const uint8_t*       set        = p.nsymb > 10 ? kRiNorm : kRiExt;
    int64_t              last       = -1;  // the largest RI position in q order
    for (uint32_t c = 0; c < 4; c++) {
      const uint32_t m = (3 * c) % 4, n = p.ri_Qp > m ? (p.ri_Qp - m + 3) / 4 : 0;
      d.ri_rows[set[c]] = (uint16_t)n;
      if (n > 0) {
        last = std::max<int64_t>(last, (int64_t)(p.rows - 1) * p.Qm + (int64_t)set[c] * p.rows * p.Qm + p.Qm - 1);
      }
    }
    uint32_t first = 0;  // the first non-RI column of row 0 holds g[0] in its own right
    while (first < p.nsymb && d.ri_rows[first] >= p.rows) {
      first++;
    }
    d.g0_src = (int32_t)std::max<int64_t>(last, (int64_t)first * p.rows * p.Qm);
  }
  return d;
}

// CQI (sch.c:1160-1183): its size may depend on the RI just decoded (ri: the decoded RI, or -1 when
// not needed)
static int ulsch_cqi_plan(srsran_pusch_cfg_t* cfg, const UlsPlan& p, int ri, uint32_t* cqi_len, uint32_t* cqi_Qp)
{
  srsran_cqi_cfg_t& cq = cfg->uci_cfg.cqi;
  *cqi_len = *cqi_Qp = 0;
  if (!cq.data_enable) {
    if (p.hl_ri) {
      cq.rank_is_not_one = false;
    }
    return SRSRAN_SUCCESS;
  }
  if (p.hl_ri) {
    cq.rank_is_not_one = ri > 0;
  }
  const int len = srsran_cqi_size(&cq);
  if (len <= 0 || len > (int)UCI_MAX_CQI_BITS) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  *cqi_len = (uint32_t)len;
  *cqi_Qp  = qprime_cqi(cfg->K_segm, cfg->grant.L_prb, p.nsymb, (uint32_t)len, beta_cqi(cfg->uci_offset.I_offset_cqi),
                        p.ri_Qp);
  return (uint64_t)*cqi_Qp + p.ri_Qp > p.H ? SRSRAN_ERROR : SRSRAN_SUCCESS;
}

// The decoded UCI into the caller's srsran_uci_value_t (sch.c:1084-1117, uci.c)
static void ulsch_uci_out(srsran_pusch_cfg_t* cfg, const UlsPlan& p, const UciOut& o, srsran_uci_value_t* uci)
{
  srsran_cqi_cfg_t& cq = cfg->uci_cfg.cqi;
  if (p.nack > 0) {
    memcpy(uci->ack.ack_value, o.ack, std::min<uint32_t>(p.nack, SRSRAN_UCI_MAX_ACK_BITS));
    uci->ack.valid = o.ack_valid != 0;
  }
  if (cq.ri_len > 0) {
    uci->ri = o.ri[0];
  }
  if (cq.data_enable) {
    uci->cqi.data_crc = o.cqi_crc != 0;
    srsran_cqi_value_unpack(&cq, const_cast<uint8_t*>(o.cqi), &uci->cqi);
  }
  if (p.hl_ri) {
    cq.rank_is_not_one = uci->ri > 0;  // sch.c:1112-1117
  }
}

// One device scratch block per call: the UCI / de-interleaver descriptors, the UCI results and
// the unpacked scrambling sequence.
struct UlsUciScratch {
  UciDesc uci;
  UlDeint deint;
  UciOut  out;
};

// srsran_ulsch_decode's body.  The LLRs come from the host (h_q) or are already on the device
// (d_q_ext, zeroed in place at the ACK positions); the scrambling sequence likewise (h_c / d_c_ext).
// q_out / g_bits (host, optional) receive q after the ACK zeroing and the de-interleaved LLRs.
static int ulsch_decode_impl(srsran_sch_t*       q,
                             srsran_pusch_cfg_t* cfg,
                             const int16_t*      h_q,
                             int16_t*            d_q_ext,
                             int16_t*            q_out,
                             int16_t*            g_bits,
                             const uint8_t*      h_c,
                             const uint8_t*      d_c_ext,
                             uint8_t*            data,
                             srsran_uci_value_t* uci_data)
{
  if (!q || !q->gpu || !cfg || (!h_q && !d_q_ext)) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (q->llr_is_8bit) {
    // srsENB's experimental pusch_8bit_decoder (cc_worker.cc:155-157): pusch.c:419-440 writes int8 LLRs into its
    // int16 q buffer and hands it to srsran_ulsch_decode, whose uci_decode_ri_ack / ulsch_deinterleave read it as
    // int16 (sch.c:1145-1161: pairs of int8 LLRs taken as one, nof_bits of them, past the int8 data) -- the
    // reference's own 8-bit UL-SCH cannot decode, so there is no behaviour to reproduce; refused
    fprintf(stderr, "[srsran_sch] 8-bit UL-SCH LLRs are not provided (the reference's 8-bit PUSCH path passes int8 "
                    "LLRs through int16 interfaces)\n");
    return SRSRAN_ERROR;
  }
  UlsPlan   p;
  const int prc = ulsch_plan(cfg, &p);
  if (prc != SRSRAN_SUCCESS) {
    return prc;
  }
  const uint32_t nb = p.nb, Qm = p.Qm, H = p.H;
  if ((p.uci && !uci_data) || (p.need_c && !h_c && !d_c_ext)) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }

  SchCtx* x = (SchCtx*)q->gpu;
  if (2 * (size_t)nb > x->ul_cap) {
    hipFree(x->d_ul);
    x->d_ul   = nullptr;
    x->ul_cap = 0;
    if (hipMalloc((void**)&x->d_ul, 2 * (size_t)nb * sizeof(int16_t)) != hipSuccess) {
      return SRSRAN_ERROR;
    }
    x->ul_cap = 2 * (size_t)nb;
  }
  int16_t* d_q = d_q_ext ? d_q_ext : x->d_ul;
  int16_t* d_g = x->d_ul + nb;
  // the reference leaves the de-interleaved LLRs in g_bits (positions it does not write untouched)
  if ((g_bits && hipMemcpyAsync(d_g, g_bits, (size_t)nb * 2, hipMemcpyHostToDevice, x->stream) != hipSuccess) ||
      (h_q && hipMemcpyAsync(d_q, h_q, (size_t)nb * 2, hipMemcpyHostToDevice, x->stream) != hipSuccess)) {
    return SRSRAN_ERROR;
  }
  if (!p.uci) {
    if (ul_deint_launch(d_q, d_g, Qm, H, p.nsymb, x->stream) != hipSuccess ||
        (g_bits && hipMemcpyAsync(g_bits, d_g, (size_t)nb * 2, hipMemcpyDeviceToHost, x->stream) != hipSuccess) ||
        (q_out && hipMemcpyAsync(q_out, d_q, (size_t)nb * 2, hipMemcpyDeviceToHost, x->stream) != hipSuccess) ||
        hipStreamSynchronize(x->stream) != hipSuccess) {
      return SRSRAN_ERROR;
    }
    if (p.s.tbs == 0) {
      return SRSRAN_SUCCESS;
    }
    srsran_pdsch_cfg_t pc;
    memset(&pc, 0, sizeof(pc));
    pc.grant.nof_tb       = 1;
    pc.grant.tb[0]        = cfg->grant.tb;
    pc.softbuffers.rx[0]  = cfg->softbuffers.rx;
    pc.max_nof_iterations = cfg->max_nof_iterations;
    return dlsch_decode_sync(q, &pc, nullptr, d_g, data, 0, 1);
  }

  // ---- device scratch: descriptors, results, sequence ----
  const bool   up_c = p.need_c && !d_c_ext;
  const size_t scr  = align16(sizeof(UlsUciScratch)) + (up_c ? (size_t)nb : 0);
  if (!grow_dev((void**)&x->d_uci, &x->uci_cap, scr)) {
    return SRSRAN_ERROR;
  }
  UlsUciScratch* d_s = (UlsUciScratch*)x->d_uci;
  const uint8_t* d_c = up_c ? x->d_uci + align16(sizeof(UlsUciScratch)) : d_c_ext;
  srsran_cqi_cfg_t& cq = cfg->uci_cfg.cqi;
  UlsUciScratch  h;
  memset(&h, 0, sizeof(h));
  h.uci   = {d_q, p.need_c ? d_c : nullptr, d_g, &d_s->out, Qm, p.rows, p.nsymb, p.nack, p.ack_Qp, cq.ri_len, p.ri_Qp, 0, 0};
  h.deint = ulsch_deint_desc(d_q, d_g, p);
  if (hipMemcpyAsync(d_s, &h, sizeof(h), hipMemcpyHostToDevice, x->stream) != hipSuccess ||
      (up_c && hipMemcpyAsync((void*)d_c, h_c, nb, hipMemcpyHostToDevice, x->stream) != hipSuccess) ||
      uci_ack_ri_launch(&d_s->uci, 1, x->stream) != hipSuccess ||
      ul_deint_batch_launch(&d_s->deint, 1, p.rows, x->stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }

  // ---- CQI (sch.c:1160-1183): its size may depend on the RI just decoded ----
  uint32_t cqi_len = 0, cqi_Qp = 0;
  if (cq.data_enable && p.hl_ri &&
      (hipMemcpyAsync(&h.out, &d_s->out, sizeof(UciOut), hipMemcpyDeviceToHost, x->stream) != hipSuccess ||
       hipStreamSynchronize(x->stream) != hipSuccess)) {
    return SRSRAN_ERROR;
  }
  const int crc = ulsch_cqi_plan(cfg, p, h.out.ri[0], &cqi_len, &cqi_Qp);
  if (crc != SRSRAN_SUCCESS) {
    return crc;
  }
  UciDesc u  = h.uci;  // a second copy: the first upload may still be reading h
  u.cqi_bits = cqi_len;
  u.cqi_Qp   = cqi_Qp;
  if (cqi_len && (hipMemcpyAsync(&d_s->uci, &u, sizeof(UciDesc), hipMemcpyHostToDevice, x->stream) != hipSuccess ||
                  uci_cqi_launch(&d_s->uci, 1, x->stream) != hipSuccess)) {
    return SRSRAN_ERROR;
  }

  // ---- decode_tb over the UL-SCH part (after the CQI) ----
  int ret = cq.data_enable ? (int)cqi_Qp : (int)p.ri_Qp;  // the value left in ret when there is no TB
  if (p.s.tbs > 0) {
    srsran_pdsch_cfg_t pc;
    memset(&pc, 0, sizeof(pc));
    pc.grant.nof_tb          = 1;
    pc.grant.tb[0]           = cfg->grant.tb;
    pc.grant.tb[0].nof_bits  = (H - p.ri_Qp - cqi_Qp) * Qm;
    pc.softbuffers.rx[0]     = cfg->softbuffers.rx;
    pc.max_nof_iterations    = cfg->max_nof_iterations;
    ret                      = dlsch_decode_sync(q, &pc, nullptr, d_g + (size_t)cqi_Qp * Qm, data, 0, 1);
  }
  if (hipMemcpyAsync(&h.out, &d_s->out, sizeof(UciOut), hipMemcpyDeviceToHost, x->stream) != hipSuccess ||
      (q_out && hipMemcpyAsync(q_out, d_q, (size_t)nb * 2, hipMemcpyDeviceToHost, x->stream) != hipSuccess) ||
      (g_bits && hipMemcpyAsync(g_bits, d_g, (size_t)nb * 2, hipMemcpyDeviceToHost, x->stream) != hipSuccess) ||
      hipStreamSynchronize(x->stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  ulsch_uci_out(cfg, p, h.out, uci_data);
  return ret;
}

int srsran_ulsch_decode(srsran_sch_t*       q,
                        srsran_pusch_cfg_t* cfg,
                        int16_t*            q_bits,
                        int16_t*            g_bits,
                        uint8_t*            c_seq,
                        uint8_t*            data,
                        srsran_uci_value_t* uci_data)
{
  if (!q_bits || !g_bits) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  return ulsch_decode_impl(q, cfg, q_bits, nullptr, q_bits, g_bits, c_seq, nullptr, data, uci_data);
}

}  // extern "C"

namespace srsran_amd {
// Rate-matching read-out for the transmitter (rm_turbo.c:345-388): fwd[k] = the natural-layout
// encoder output index (3 i + stream, tail 3K..3K+11) of the k-th transmitted bit of the rv's
// circular buffer, period 3K + 12 along the E bits.  The inverse of the receive table.
bool rm_fwd_table(uint32_t cb_idx, uint32_t rv, const uint16_t** d_fwd, uint32_t* N)
{
  static std::map<uint64_t, uint16_t*> cache;
  const uint32_t                       K   = (uint32_t)srsran_cbsegm_cbsize(cb_idx);
  const uint64_t                       key = ((uint64_t)cur_dev() << 32) | (cb_idx * 4 + rv);
  *N                                       = 3 * K + 12;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto                        it = cache.find(key);
    if (it != cache.end()) {
      *d_fwd = it->second;
      return true;
    }
  }
  InvTable t;
  if (!inv_table(cb_idx, rv, false, &t)) {
    return false;
  }
  std::vector<uint16_t> inv(t.len), fwd(t.N);
  if (hipMemcpy(inv.data(), t.d, t.len * sizeof(uint16_t), hipMemcpyDeviceToHost) != hipSuccess) {
    return false;
  }
  for (uint32_t n = 0; n < t.len; n++) {
    fwd[inv[n]] = (uint16_t)n;
  }
  uint16_t* d = nullptr;
  if (hipMalloc((void**)&d, t.N * sizeof(uint16_t)) != hipSuccess ||
      hipMemcpy(d, fwd.data(), t.N * sizeof(uint16_t), hipMemcpyHostToDevice) != hipSuccess) {
    return false;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  cache[key] = d;
  *d_fwd     = d;
  return true;
}

hipStream_t sch_stream(srsran_sch_t* q) { return q && q->gpu ? ((SchCtx*)q->gpu)->stream : nullptr; }

// The object's decode stream moved to a hardware queue of its own (own_queue_stream, stage_copy.h).  srsENB runs one PUSCH object
// per PHY worker, several batches at once: two workers' streams that the runtime maps to one queue run their
// batches one after the other (least-used queue assignment, which depends on the streams created and freed before:
// 424 k UE-subframes/s with two workers standalone, 284 k after a PDSCH run in the same process, 422 k with this;
// tools/r06as_pusch_order.py).  SRSRAN_AMD_PUSCH_OWN_QUEUE=0 (read once) keeps the shared queue.
int sch_own_queue(srsran_sch_t* q)
{
  static const bool on = [] {
    const char* e = getenv("SRSRAN_AMD_PUSCH_OWN_QUEUE");
    return !e || atoi(e) != 0;
  }();
  SchCtx* x = q && q->gpu ? (SchCtx*)q->gpu : nullptr;
  if (!x) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (!on) {
    return SRSRAN_SUCCESS;
  }
  hipStream_t s = nullptr;
  if (own_queue_stream(&s) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  hipStreamSynchronize(x->stream);
  hipStreamDestroy(x->stream);
  x->stream = s;
  return SRSRAN_SUCCESS;
}

int ulsch_decode_dev(srsran_sch_t* q, srsran_pusch_cfg_t* cfg, int16_t* d_q, const uint8_t* d_c, uint8_t* data,
                     srsran_uci_value_t* uci_data)
{
  return ulsch_decode_impl(q, cfg, nullptr, d_q, nullptr, nullptr, nullptr, d_c, data, uci_data);
}

// Batched srsran_ulsch_decode (ulsch_batch.h): the same stages as ulsch_decode_impl, each one launch
// over every UE of the batch, and one decode_tb batch for all their transport blocks.
int ulsch_decode_batch_dev(srsran_sch_t* q, uint32_t n, UlschBatchUe* ues, const uint8_t* d_data_base,
                           size_t data_bytes, hipStream_t st)
{
  if (!q || !q->gpu || (n && !ues)) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (q->llr_is_8bit) {
    return SRSRAN_ERROR;
  }
  SchCtx*              x = (SchCtx*)q->gpu;
  std::vector<UlsPlan> plan(n);
  std::vector<int32_t> uix(n, -1);  // index in the UCI arrays
  std::vector<uint32_t> live;
  uint32_t              m = 0, max_rows = 0;
  bool                  need_ri = false;
  for (uint32_t i = 0; i < n; i++) {
    UlschBatchUe& u = ues[i];
    u.avg           = NAN;
    u.ret           = u.cfg ? ulsch_plan(u.cfg, &plan[i]) : SRSRAN_ERROR_INVALID_INPUTS;
    if (u.ret == SRSRAN_SUCCESS &&
        (!u.d_q || !u.d_g || (plan[i].uci && !u.uci) || (plan[i].need_c && !u.d_c) ||
         (plan[i].s.tbs > 0 && (!u.cfg->softbuffers.rx || !u.d_data || u.d_data < d_data_base ||
                                u.d_data + plan[i].s.tbs / 8 > d_data_base + data_bytes)))) {
      u.ret = SRSRAN_ERROR_INVALID_INPUTS;
    }
    if (u.ret != SRSRAN_SUCCESS) {
      continue;
    }
    live.push_back(i);
    max_rows = std::max(max_rows, plan[i].rows);
    if (plan[i].uci) {
      uix[i] = (int32_t)m++;
      need_ri |= plan[i].hl_ri;
    }
  }
  const uint32_t nl = (uint32_t)live.size();
  // device scratch: UciDesc[m] | UlDeint[nl] | UciOut[m] | result[nl] | avg[nl]; pinned staging:
  // the two uploads (the CQI pass rewrites the UCI descriptors) and the read-back
  const size_t o_dd = align16(m * sizeof(UciDesc)), o_out = o_dd + align16(nl * sizeof(UlDeint));
  const size_t o_res = o_out + align16(m * sizeof(UciOut)), o_avg = o_res + align16(nl * sizeof(int32_t));
  const size_t dev_need = o_avg + align16(nl * sizeof(float));
  const size_t h_cqi = dev_need, h_back = h_cqi + align16(m * sizeof(UciDesc));
  const size_t back_len = dev_need - o_out, h_need = h_back + back_len + data_bytes;
  if (!grow_dev((void**)&x->d_ubs, &x->dubs_cap, dev_need)) {
    return SRSRAN_ERROR;
  }
  if (h_need > x->hubs_cap) {
    hipHostFree(x->h_ubs);
    x->h_ubs    = nullptr;
    x->hubs_cap = 0;
    if (hipHostMalloc((void**)&x->h_ubs, h_need, hipHostMallocDefault) != hipSuccess) {
      return SRSRAN_ERROR;
    }
    x->hubs_cap = h_need;
  }
  uint8_t* d = x->d_ubs;
  uint8_t* h = x->h_ubs;
  UciDesc* h_ud  = (UciDesc*)h;
  UlDeint* h_dd  = (UlDeint*)(h + o_dd);
  UciOut*  d_out = (UciOut*)(d + o_out);
  for (uint32_t j = 0; j < nl; j++) {
    const uint32_t i = live[j];
    const UlsPlan& p = plan[i];
    h_dd[j]          = ulsch_deint_desc(ues[i].d_q, ues[i].d_g, p);
    if (uix[i] >= 0) {
      h_ud[uix[i]] = {ues[i].d_q, p.need_c ? ues[i].d_c : nullptr, ues[i].d_g, d_out + uix[i], p.Qm, p.rows, p.nsymb,
                      p.nack, p.ack_Qp, ues[i].cfg->uci_cfg.cqi.ri_len, p.ri_Qp, 0, 0};
    }
  }
  // ACK decode + zeroing and RI decode (sch.c:1023-1120), then the de-interleaver reading the zeroed q
  if (nl && (hipMemcpyAsync(d, h, o_out, hipMemcpyHostToDevice, st) != hipSuccess ||
             (m && uci_ack_ri_launch((const UciDesc*)d, m, st) != hipSuccess) ||
             ul_deint_batch_launch((const UlDeint*)(d + o_dd), nl, max_rows, st) != hipSuccess)) {
    return SRSRAN_ERROR;
  }
  UciOut* h_out = (UciOut*)(h + h_back);
  if (need_ri && (hipMemcpyAsync(h_out, d_out, m * sizeof(UciOut), hipMemcpyDeviceToHost, st) != hipSuccess ||
                  hipStreamSynchronize(st) != hipSuccess)) {
    return SRSRAN_ERROR;
  }
  // CQI sizes (after the RI where the report needs it) and the UL-SCH parts
  std::vector<uint32_t>              cqi_Qp(n, 0);
  std::vector<srsran_dlsch_gpu_tb_t> tbs;
  std::vector<int32_t>               tbix(n, -1);
  UciDesc*                           h_ud2 = (UciDesc*)(h + h_cqi);
  bool                               any_cqi = false;
  std::vector<uint32_t>              tb_maxit;  // each TB's max_nof_iterations (pusch.c:450 sets it per UE)
  memcpy(h_ud2, h_ud, m * sizeof(UciDesc));
  for (uint32_t i : live) {
    UlschBatchUe&  u = ues[i];
    const UlsPlan& p = plan[i];
    if (uix[i] >= 0) {
      uint32_t len = 0;
      u.ret        = ulsch_cqi_plan(u.cfg, p, need_ri ? h_out[uix[i]].ri[0] : 0, &len, &cqi_Qp[i]);
      if (u.ret != SRSRAN_SUCCESS) {
        continue;
      }
      h_ud2[uix[i]].cqi_bits = len;
      h_ud2[uix[i]].cqi_Qp   = cqi_Qp[i];
      any_cqi |= len > 0;
    }
    if (p.s.tbs > 0) {
      srsran_dlsch_gpu_tb_t t;
      memset(&t, 0, sizeof(t));
      t.tbs        = p.s.tbs;
      t.Qm         = p.Qm;
      t.rv         = (uint32_t)u.cfg->grant.tb.rv;
      t.nof_e_bits = (p.H - p.ri_Qp - cqi_Qp[i]) * p.Qm;
      t.d_e_bits   = u.d_g + (size_t)cqi_Qp[i] * p.Qm;
      t.d_data     = u.d_data;
      t.softbuffer = u.cfg->softbuffers.rx;
      t.new_data   = u.new_data ? 1 : 0;
      tbix[i]      = (int32_t)tbs.size();
      tbs.push_back(t);
      tb_maxit.push_back(u.cfg->max_nof_iterations ? u.cfg->max_nof_iterations : 10);  // set unconditionally
    }
  }
  if (any_cqi && (hipMemcpyAsync(d, h_ud2, m * sizeof(UciDesc), hipMemcpyHostToDevice, st) != hipSuccess ||
                  uci_cqi_launch((const UciDesc*)d, m, st) != hipSuccess)) {
    return SRSRAN_ERROR;
  }
  if (!tbs.empty() &&
      srsran_amd::dlsch_gpu_decode_batch_limits(q, (uint32_t)tbs.size(), tbs.data(), tb_maxit.data(),
                                                (int32_t*)(d + o_res), (float*)(d + o_avg), st) != SRSRAN_SUCCESS) {
    return SRSRAN_ERROR;  // one decode batch per UE iteration limit (pusch.c:450 sets it per decode)
  }
  // results, UCI and payloads back in one sync
  if ((nl && hipMemcpyAsync(h + h_back, d + o_out, back_len, hipMemcpyDeviceToHost, st) != hipSuccess) ||
      (!tbs.empty() && data_bytes &&
       hipMemcpyAsync(h + h_back + back_len, d_data_base, data_bytes, hipMemcpyDeviceToHost, st) != hipSuccess) ||
      hipStreamSynchronize(st) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  const int32_t* h_res = (const int32_t*)(h + h_back + (o_res - o_out));
  const float*   h_avg = (const float*)(h + h_back + (o_avg - o_out));
  float          last  = q->avg_iterations;  // avg_iterations as sequential decodes would leave it
  for (uint32_t i = 0; i < n; i++) {
    UlschBatchUe&  u = ues[i];
    const UlsPlan& p = plan[i];
    if (uix[i] < 0 && tbix[i] < 0) {
      u.avg = last;
      continue;  // a failed check, or neither UCI nor a TB: srsran_ulsch_decode returns SUCCESS
    }
    if (u.ret != SRSRAN_SUCCESS) {
      u.avg = last;
      continue;
    }
    if (uix[i] >= 0) {
      ulsch_uci_out(u.cfg, p, h_out[uix[i]], u.uci);
      u.ret = u.cfg->uci_cfg.cqi.data_enable ? (int)cqi_Qp[i] : (int)p.ri_Qp;
    }
    if (tbix[i] >= 0) {
      u.ret = h_res[tbix[i]];
      last  = h_avg[tbix[i]];
      if (u.data) {
        memcpy(u.data, h + h_back + back_len + (u.d_data - d_data_base), p.s.tbs / 8);
      }
    }
    u.avg = last;
  }
  q->avg_iterations = last;
  return SRSRAN_SUCCESS;
}
}  // namespace srsran_amd

extern "C" {

int srsran_ulsch_gpu_decode_batch(srsran_sch_t*                q,
                                  uint32_t                     nof_tb,
                                  const srsran_ulsch_gpu_tb_t* tbs,
                                  int32_t*                     d_result,
                                  float*                       d_avg_noi,
                                  void*                        stream)
{
  if (!q || !q->gpu || (nof_tb && (!tbs || !d_result || !d_avg_noi))) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (q->llr_is_8bit) {
    return SRSRAN_ERROR;
  }
  std::vector<srsran_dlsch_gpu_tb_t> dl(nof_tb);
  std::vector<UlDeint>               desc(nof_tb);
  uint32_t                           max_n = 0;
  for (uint32_t i = 0; i < nof_tb; i++) {
    const srsran_ulsch_gpu_tb_t& t = tbs[i];
    if (!t.d_q_bits || !t.d_g_bits || t.Qm == 0 || t.Qm > 8 || t.nof_symb == 0 || t.nof_symb > 14 ||
        t.nof_e_bits % t.Qm) {
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
    const uint32_t rows = t.nof_e_bits / t.Qm / t.nof_symb;
    desc[i]             = {t.d_q_bits, t.d_g_bits, rows, t.nof_symb, t.Qm, {}, -1};
    max_n               = std::max(max_n, rows);
    dl[i]               = {t.tbs, t.Qm, t.rv, t.nof_e_bits, t.d_g_bits, t.d_data, t.softbuffer, t.new_data};
  }
  SchCtx* x = (SchCtx*)q->gpu;
  // the previous call's de-interleaver must have read its descriptors before staging is rewritten
  if (x->uldesc_live) {
    hipEventSynchronize(x->uldesc_used);
  }
  if (!x->uldesc_used && hipEventCreateWithFlags(&x->uldesc_used, hipEventDisableTiming) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  if (nof_tb > x->uldesc_cap) {
    hipFree(x->d_uldesc);
    hipHostFree(x->h_uldesc);
    x->d_uldesc   = nullptr;
    x->h_uldesc   = nullptr;
    x->uldesc_cap = 0;
    const size_t cap = std::max<size_t>(2 * nof_tb, 64);
    if (hipMalloc((void**)&x->d_uldesc, cap * sizeof(UlDeint)) != hipSuccess ||
        hipHostMalloc((void**)&x->h_uldesc, cap * sizeof(UlDeint), hipHostMallocDefault) != hipSuccess) {
      return SRSRAN_ERROR;
    }
    x->uldesc_cap = cap;
  }
  if (nof_tb) {
    memcpy(x->h_uldesc, desc.data(), nof_tb * sizeof(UlDeint));
    if (hipMemcpyAsync(x->d_uldesc, x->h_uldesc, nof_tb * sizeof(UlDeint), hipMemcpyHostToDevice,
                       (hipStream_t)stream) != hipSuccess ||
        ul_deint_batch_launch(x->d_uldesc, nof_tb, max_n, (hipStream_t)stream) != hipSuccess) {
      return SRSRAN_ERROR;
    }
    hipEventRecord(x->uldesc_used, (hipStream_t)stream);
    x->uldesc_live = true;
  }
  return srsran_dlsch_gpu_decode_batch(q, nof_tb, dl.data(), d_result, d_avg_noi, stream);
}


// ---------------- DL-SCH transmit (sch.c:240-359, 621-652) ----------------
}  // extern "C"
namespace srsran_amd {
bool rm_fwd_table(uint32_t cb_idx, uint32_t rv, const uint16_t** d_fwd, uint32_t* N);
void qpp_coeffs(uint32_t idx, uint32_t* f1, uint32_t* f2);
}  // namespace srsran_amd
extern "C" {

int srsran_dlsch_gpu_encode_batch(srsran_sch_t* q, uint32_t nof_tb, const srsran_dlsch_gpu_enc_t* tbs, void* stream)
{
  if (!q || !q->gpu || (nof_tb && !tbs)) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (nof_tb == 0) {
    return SRSRAN_SUCCESS;
  }
  SchCtx*              x  = (SchCtx*)q->gpu;
  hipStream_t          st = (hipStream_t)stream;
  std::vector<EncTb>   tb(nof_tb);
  std::vector<EncCb>   cb;
  std::vector<size_t>  e_off(nof_tb);
  size_t               e_tot = 0;
  uint32_t             max_bytes = 0;
  std::map<uint32_t, std::pair<const uint16_t*, uint32_t>> fwd;  // (cb_idx, rv) -> table, looked up once
  for (uint32_t t = 0; t < nof_tb; t++) {
    const srsran_dlsch_gpu_enc_t& in = tbs[t];
    srsran_cbsegm_t               s;
    if (!in.d_data || !in.d_e_bits || in.Qm == 0 || in.rv > 3 || srsran_cbsegm(&s, in.tbs) || s.tbs == 0) {
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
    if (s.F) {
      fprintf(stderr, "[srsran_sch] Error filler bits are not supported. Use standard TBS\n");
      return SRSRAN_ERROR;
    }
    e_off[t] = e_tot;
    e_tot += (in.nof_e_bits + 15) & ~15u;
    max_bytes = std::max(max_bytes, (in.nof_e_bits + 7) / 8);
    // encode_tb_off's split of the E bits over the blocks (sch.c:271-305); the K2 blocks come first
    const uint32_t Gp = in.nof_e_bits / in.Qm, gamma = Gp % s.C;
    uint32_t       rp = 0, wp = 0;
    for (uint32_t i = 0; i < s.C; i++) {
      const uint32_t K   = i < s.C2 ? s.K2 : s.K1;
      const uint32_t idx = i < s.C2 ? s.K2_idx : s.K1_idx;
      EncCb          c;
      memset(&c, 0, sizeof(c));
      c.rlen = s.C > 1 ? K - 24 : K;
      c.E    = i <= s.C - gamma - 1 ? in.Qm * (Gp / s.C) : in.Qm * ((Gp + s.C - 1) / s.C);
      c.K    = K;
      c.rp   = rp;
      c.cb_crc   = s.C > 1;
      c.tb_bytes = in.tbs / 8;
      c.data     = in.d_data;
      qpp_coeffs(idx, &c.f1, &c.f2);
      auto it = fwd.find(idx * 4 + in.rv);
      if (it == fwd.end()) {
        std::pair<const uint16_t*, uint32_t> v;
        if (!rm_fwd_table(idx, in.rv, &v.first, &v.second)) {
          return SRSRAN_ERROR;
        }
        it = fwd.emplace(idx * 4 + in.rv, v).first;
      }
      c.fwd = it->second.first;
      c.N   = it->second.second;
      c.e    = (uint8_t*)(uintptr_t)(e_off[t] + wp);  // offsets: fixed up after the allocation
      c.tb_crc = (const uint32_t*)(uintptr_t)t;
      cb.push_back(c);
      rp += c.rlen;
      wp += c.E;
    }
    if (wp > in.nof_e_bits) {
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
    tb[t] = {in.d_data, nullptr, nullptr, in.d_e_bits, in.tbs / 8, in.nof_e_bits};
  }
  // device scratch: [EncTb x ntb][EncCb x ncb][crc x ntb][unpacked e bits]
  const size_t o_cb = align16(nof_tb * sizeof(EncTb)), o_crc = o_cb + align16(cb.size() * sizeof(EncCb));
  const size_t o_e = o_crc + align16(nof_tb * sizeof(uint32_t)), need = o_e + e_tot;
  if (!grow_dev((void**)&x->d_enc, &x->enc_cap, need)) {
    return SRSRAN_ERROR;
  }
  uint32_t* d_crc = (uint32_t*)(x->d_enc + o_crc);
  uint8_t*  d_e   = x->d_enc + o_e;
  for (uint32_t t = 0; t < nof_tb; t++) {
    tb[t].crc    = d_crc + t;
    tb[t].e_bits = d_e + e_off[t];
  }
  for (EncCb& c : cb) {
    c.e      = d_e + (size_t)(uintptr_t)c.e;
    c.tb_crc = d_crc + (size_t)(uintptr_t)c.tb_crc;
  }
  const EncTb* d_tb = (const EncTb*)x->d_enc;
  const EncCb* d_cb = (const EncCb*)(x->d_enc + o_cb);
  if (hipMemcpyAsync(x->d_enc, tb.data(), nof_tb * sizeof(EncTb), hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemcpyAsync(x->d_enc + o_cb, cb.data(), cb.size() * sizeof(EncCb), hipMemcpyHostToDevice, st) != hipSuccess ||
      enc_tb_crc_launch(d_tb, nof_tb, st) != hipSuccess || enc_cb_launch(d_cb, (uint32_t)cb.size(), st) != hipSuccess ||
      enc_pack_launch(d_tb, nof_tb, max_bytes, st) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  // x->d_enc is reused by the next call in stream order (one stream per object)
  return SRSRAN_SUCCESS;
}

int srsran_dlsch_encode2(srsran_sch_t*       q,
                         srsran_pdsch_cfg_t* cfg,
                         uint8_t*            data,
                         uint8_t*            e_bits,
                         int                 tb_idx,
                         uint32_t            nof_layers)
{
  if (!q || !q->gpu || !cfg || !e_bits || tb_idx < 0 || tb_idx >= SRSRAN_MAX_CODEWORDS) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (!data) {
    fprintf(stderr, "[srsran_sch] encoding from the soft buffer (data == NULL) is not provided\n");
    return SRSRAN_ERROR;
  }
  const srsran_ra_tb_t& t  = cfg->grant.tb[tb_idx];
  const uint32_t        Nl = nof_layers != cfg->grant.nof_tb ? 2 : 1;  // sch.c:633-636
  const uint32_t        Qm = srsran_mod_bits_x_symbol(t.mod) * Nl;
  if (t.tbs <= 0) {
    return t.tbs == 0 ? SRSRAN_SUCCESS : SRSRAN_ERROR_INVALID_INPUTS;
  }
  SchCtx*        x      = (SchCtx*)q->gpu;
  const uint32_t nbytes = (uint32_t)t.tbs / 8, ebytes = (t.nof_bits + 7) / 8;
  uint8_t*       d_io   = nullptr;
  if (hipMallocAsync((void**)&d_io, nbytes + ebytes + 16, x->stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  srsran_dlsch_gpu_enc_t e = {(uint32_t)t.tbs, Qm, (uint32_t)t.rv, t.nof_bits, d_io, d_io + nbytes};
  int                    r = SRSRAN_ERROR;
  if (hipMemcpyAsync(d_io, data, nbytes, hipMemcpyHostToDevice, x->stream) == hipSuccess) {
    r = srsran_dlsch_gpu_encode_batch(q, 1, &e, x->stream);
    if (r == SRSRAN_SUCCESS &&
        (hipMemcpyAsync(e_bits, d_io + nbytes, ebytes, hipMemcpyDeviceToHost, x->stream) != hipSuccess ||
         hipStreamSynchronize(x->stream) != hipSuccess)) {
      r = SRSRAN_ERROR;
    }
  }
  hipFreeAsync(d_io, x->stream);
  hipStreamSynchronize(x->stream);
  return r;
}

int srsran_dlsch_encode(srsran_sch_t* q, srsran_pdsch_cfg_t* cfg, uint8_t* data, uint8_t* e_bits)
{
  return srsran_dlsch_encode2(q, cfg, data, e_bits, 0, 1);
}

}  // extern "C"
