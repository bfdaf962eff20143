// srsran_4g_amd/csrc/tdec_api.cpp -- C-ABI host side of the HIP turbo decoder.
//
// Implements include/srsran_tdec.h (the srsran_tdec_* surface of
// lib/include/srsran/phy/fec/turbo/turbodecoder.h) over the kernel in
// tdec_kernel.hip.  Host semantics follow turbodecoder.c:
//   init / init_manual / free            turbodecoder.c:129-363
//   new_cb / iteration / run_all          turbodecoder.c:510-549
//   AUTO dispatch (sub-blocks per K)      turbodecoder.c:381-408
// Calls are host-synchronous like the reference; the batch entry points are
// extensions.  There is no CPU fallback: without a HIP device every decode call
// fails with SRSRAN_ERROR.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <map>
#include <tuple>
#include <mutex>
#include <vector>

#include "../../include/srsran_tdec.h"
#include "stage_copy.h"
#include "devkey.h"
#include "tdec_kernel.h"
#include "tdec8bit_kernel.h"

using namespace srsran_amd;

namespace {

const uint16_t kCbSizes[SRSRAN_NOF_TC_CB_SIZES] = {
    40,   48,   56,   64,   72,   80,   88,   96,   104,  112,  120,  128,  136,  144,  152,  160,  168,  176,  184,
    192,  200,  208,  216,  224,  232,  240,  248,  256,  264,  272,  280,  288,  296,  304,  312,  320,  328,  336,
    344,  352,  360,  368,  376,  384,  392,  400,  408,  416,  424,  432,  440,  448,  456,  464,  472,  480,  488,
    496,  504,  512,  528,  544,  560,  576,  592,  608,  624,  640,  656,  672,  688,  704,  720,  736,  752,  768,
    784,  800,  816,  832,  848,  864,  880,  896,  912,  928,  944,  960,  976,  992,  1008, 1024, 1056, 1088, 1120,
    1152, 1184, 1216, 1248, 1280, 1312, 1344, 1376, 1408, 1440, 1472, 1504, 1536, 1568, 1600, 1632, 1664, 1696, 1728,
    1760, 1792, 1824, 1856, 1888, 1920, 1952, 1984, 2016, 2048, 2112, 2176, 2240, 2304, 2368, 2432, 2496, 2560, 2624,
    2688, 2752, 2816, 2880, 2944, 3008, 3072, 3136, 3200, 3264, 3328, 3392, 3456, 3520, 3584, 3648, 3712, 3776, 3840,
    3904, 3968, 4032, 4096, 4160, 4224, 4288, 4352, 4416, 4480, 4544, 4608, 4672, 4736, 4800, 4864, 4928, 4992, 5056,
    5120, 5184, 5248, 5312, 5376, 5440, 5504, 5568, 5632, 5696, 5760, 5824, 5888, 5952, 6016, 6080, 6144};

// QPP coefficients, 36.212 Table 5.1.3-3 (tc_interl_lte.c:39-61).
const uint16_t kF1[SRSRAN_NOF_TC_CB_SIZES] = {
    3,   7,   19,  7,   7,   11,  5,   11,  7,   41,  103, 15,  9,   17,  9,   21,  101, 21,  57, 23,  13,
    27,  11,  27,  85,  29,  33,  15,  17,  33,  103, 19,  19,  37,  19,  21,  21,  115, 193, 21, 133, 81,
    45,  23,  243, 151, 155, 25,  51,  47,  91,  29,  29,  247, 29,  89,  91,  157, 55,  31,  17, 35,  227,
    65,  19,  37,  41,  39,  185, 43,  21,  155, 79,  139, 23,  217, 25,  17,  127, 25,  239, 17, 137, 215,
    29,  15,  147, 29,  59,  65,  55,  31,  17,  171, 67,  35,  19,  39,  19,  199, 21,  211, 21, 43,  149,
    45,  49,  71,  13,  17,  25,  183, 55,  127, 27,  29,  29,  57,  45,  31,  59,  185, 113, 31, 17,  171,
    209, 253, 367, 265, 181, 39,  27,  127, 143, 43,  29,  45,  157, 47,  13,  111, 443, 51,  51, 451, 257,
    57,  313, 271, 179, 331, 363, 375, 127, 31,  33,  43,  33,  477, 35,  233, 357, 337, 37,  71, 71,  37,
    39,  127, 39,  39,  31,  113, 41,  251, 43,  21,  43,  45,  45,  161, 89,  323, 47,  23,  47, 263};
const uint16_t kF2[SRSRAN_NOF_TC_CB_SIZES] = {
    10,  12,  42,  16,  18,  20,  22,  24,  26,  84,  90,  32,  34,  108, 38,  120, 84,  44,  46,  48,  50,
    52,  36,  56,  58,  60,  62,  32,  198, 68,  210, 36,  74,  76,  78,  120, 82,  84,  86,  44,  90,  46,
    94,  48,  98,  40,  102, 52,  106, 72,  110, 168, 114, 58,  118, 180, 122, 62,  84,  64,  66,  68,  420,
    96,  74,  76,  234, 80,  82,  252, 86,  44,  120, 92,  94,  48,  98,  80,  102, 52,  106, 48,  110, 112,
    114, 58,  118, 60,  122, 124, 84,  64,  66,  204, 140, 72,  74,  76,  78,  240, 82,  252, 86,  88,  60,
    92,  846, 48,  28,  80,  102, 104, 954, 96,  110, 112, 114, 116, 354, 120, 610, 124, 420, 64,  66,  136,
    420, 216, 444, 456, 468, 80,  164, 504, 172, 88,  300, 92,  188, 96,  28,  240, 204, 104, 212, 192, 220,
    336, 228, 232, 236, 120, 244, 248, 168, 64,  130, 264, 134, 408, 138, 280, 142, 480, 146, 444, 120, 152,
    462, 234, 158, 80,  96,  902, 166, 336, 170, 86,  174, 176, 178, 120, 182, 184, 186, 94,  190, 480};

int cb_index(uint32_t K)
{
  for (int i = 0; i < SRSRAN_NOF_TC_CB_SIZES; i++) {
    if (kCbSizes[i] == K) {
      return i;
    }
  }
  return -1;
}

constexpr size_t kMaxLds = 160 * 1024;

// Geometry + device tables of one (K, sub-block count) decoder configuration.
struct Config {
  int       nsb;  // 16, 8 or 1 (generic)
  TdecArgs  proto;
  uint16_t* d_tfwd = nullptr;  // visit (SB) order
  uint16_t* d_trev = nullptr;
  uint16_t* d_tfwd_nat = nullptr;  // natural order
  uint16_t* d_trev_nat = nullptr;
};

std::mutex                             g_mu;
std::map<std::tuple<int, uint32_t, int>, Config*> g_cfg;  // (device, K, nsb)
int                                    g_have_gpu = -1;

bool have_gpu()
{
  if (g_have_gpu < 0) {
    int n = 0;
    g_have_gpu = (hipGetDeviceCount(&n) == hipSuccess && n > 0) ? 1 : 0;
  }
  return g_have_gpu == 1;
}

// Build (once) the configuration for K decoded with nsb sub-blocks (1 = generic).
Config* get_config(uint32_t K, int nsb)
{
  std::lock_guard<std::mutex> lk(g_mu);
  auto key = std::make_tuple(cur_dev(), K, nsb);
  auto it  = g_cfg.find(key);
  if (it != g_cfg.end()) {
    return it->second;
  }
  const int idx = cb_index(K);
  if (idx < 0 || !have_gpu()) {
    return nullptr;
  }
  TdecArgs a{};
  a.K = K;
  if (nsb > 1) {
    if (K % nsb || K / nsb < (uint32_t)TDEC_OVERLAP) {
      return nullptr;
    }
    a.L   = K / nsb;
    a.Ls  = a.L | 1u;  // odd slot stride: quads of different sub-blocks hit different LDS banks
    a.xyw = nsb * a.Ls;
    a.M   = (a.L + TDEC_W - 1) / TDEC_W;
  } else {
    a.L   = K;
    a.Ls  = (K + 3) | 1u;
    a.xyw = a.Ls;
    a.M   = (K + 3 + TDEC_W - 1) / TDEC_W;
  }
  a.magicL  = (uint32_t)(((1ull << 32) + a.L - 1) / a.L);
  a.magicLs = (uint32_t)(((1ull << 32) + a.Ls - 1) / a.Ls);
  if (tdec_lds_bytes(nsb, a.xyw, a.M) > kMaxLds) {
    return nullptr;
  }
  // QPP tables (tc_interl_lte.c:69-107) expressed directly as LDS slots.
  std::vector<uint16_t> fwd(K), rev(K), tf(K), tr(K), tfn(K), trn(K);
  const uint64_t f1 = kF1[idx], f2 = kF2[idx];
  for (uint64_t i = 0; i < K; i++) {
    const uint32_t j = (uint32_t)((f1 * i + f2 * i * i) % K);
    fwd[i]           = (uint16_t)j;
    rev[j]           = (uint16_t)i;
  }
  auto slot = [&](uint32_t n) -> uint16_t {
    return nsb > 1 ? (uint16_t)((n / a.L) * a.Ls + n % a.L) : (uint16_t)n;
  };
  // indexed in the kernel's visiting order q (rm_turbo SB order for window decoders)
  for (uint32_t q = 0; q < K; q++) {
    const uint32_t n = nsb > 1 ? (q % nsb) * a.L + q / nsb : q;
    tf[q]            = slot(fwd[n]);
    tr[q]            = slot(rev[n]);
    tfn[q]           = slot(fwd[q]);
    trn[q]           = slot(rev[q]);
  }
  Config* c = new Config();
  c->nsb    = nsb;
  c->proto  = a;
  auto up = [&](uint16_t** d, const std::vector<uint16_t>& h) {
    return hipMalloc(d, K * sizeof(uint16_t)) == hipSuccess &&
           hipMemcpy(*d, h.data(), K * sizeof(uint16_t), hipMemcpyHostToDevice) == hipSuccess;
  };
  if (!up(&c->d_tfwd, tf) || !up(&c->d_trev, tr) || !up(&c->d_tfwd_nat, tfn) || !up(&c->d_trev_nat, trn)) {
    fprintf(stderr, "[srsran_tdec] device table allocation failed for K=%u\n", K);
    delete c;
    return nullptr;
  }
  g_cfg[key] = c;
  return c;
}

int auto_nsb(uint32_t K)
{
  const uint32_t n = srsran_tdec_autoimp_get_subblocks(K);
  return n ? (int)n : 1;
}

int nsb_for(const srsran_tdec_t* h, uint32_t K)
{
  switch (h->dec_type) {
    case SRSRAN_TDEC_AUTO:
      return auto_nsb(K);
    case SRSRAN_TDEC_GENERIC:
      return 1;
    case SRSRAN_TDEC_SSE_WINDOW:
      return 8;
    case SRSRAN_TDEC_AVX_WINDOW:
      return 16;
    default:
      return -1;
  }
}

// Per-object device context (the reference's app/ext/syst/parity buffers).
struct Ctx {
  hipStream_t stream = nullptr;
  short*      d_in   = nullptr;  // one code block input (max SB layout)
  uint8_t*    d_out  = nullptr;
  short*      d_state = nullptr; // saved LDS state between srsran_tdec_iteration calls
  size_t      state_elems = 0;
  // batch scratch
  short*      d_bin  = nullptr;
  uint8_t*    d_bout = nullptr;
  size_t      bin_elems = 0, bout_bytes = 0;
};

const size_t kMaxIn = 3 * (SRSRAN_TCOD_MAX_LEN_CB + 32) + SRSRAN_TCOD_TOTALTAIL;

int enqueue(const Config* c, const short* d_in, uint32_t in_stride, int layout_sb, uint8_t* d_out, uint32_t ncb,
            int n_start, int n_end, short* d_state, hipStream_t stream)
{
  TdecArgs a  = c->proto;
  a.in        = d_in;
  a.in_stride = in_stride;
  a.layout_sb = (c->nsb > 1) ? layout_sb : 0;  // K<=400 is always natural (rm_turbo.c:403-425)
  a.ncb       = ncb;
  a.n_start   = n_start;
  a.n_end     = n_end;
  a.out       = d_out;
  a.tfwd      = c->d_tfwd;
  a.trev      = c->d_trev;
  a.tfwd_nat  = c->d_tfwd_nat;
  a.trev_nat  = c->d_trev_nat;
  a.state     = d_state;
  hipError_t e = tdec_launch(c->nsb, a, stream);
  if (e != hipSuccess) {
    fprintf(stderr, "[srsran_tdec] launch failed: %s\n", hipGetErrorString(e));
    return SRSRAN_ERROR;
  }
  return SRSRAN_SUCCESS;
}

bool grow(void** p, size_t* have, size_t need)
{
  if (*have >= need) {
    return true;
  }
  if (*p) {
    (void)hipFree(*p);
    *p = nullptr;
  }
  if (hipMalloc(p, need) != hipSuccess) {
    *have = 0;
    return false;
  }
  *have = need;
  return true;
}

// x^(8m) mod CRC24A / CRC24B, m = 0..768, for the in-kernel CB CRC (device, built once)
struct XpowTables {
  const uint32_t* d[2] = {nullptr, nullptr};
};
std::map<int, XpowTables> g_xpow;  // per device

// the current device's tables (nullptr if they cannot be built)
const XpowTables* xpow_tables()
{
  std::lock_guard<std::mutex> lk(g_mu);
  const int dev = cur_dev();
  auto      it  = g_xpow.find(dev);
  if (it != g_xpow.end()) {
    return &it->second;
  }
  const int             nm = SRSRAN_TCOD_MAX_LEN_CB / 8 + 1;
  std::vector<uint32_t> h(nm);
  uint32_t*             d[2] = {nullptr, nullptr};
  const uint32_t        poly[2] = {LTE_CRC24A, LTE_CRC24B};
  for (int i = 0; i < 2; i++) {
    crc24_xpow_table(poly[i], h.data(), nm);
    if (hipMalloc(&d[i], nm * sizeof(uint32_t)) != hipSuccess ||
        hipMemcpy(d[i], h.data(), nm * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
      return nullptr;
    }
  }
  XpowTables& t = g_xpow[dev];
  t.d[0]        = d[0];
  t.d[1]        = d[1];
  return &t;
}

// The 8-bit decoders' interleaver in their sub-block layout (NSB = 16 or 32 sub-blocks of Ls = K / NSB): entry j
// (SB index j = row * NSB + sub-block) is the SB index of the QPP image of j's natural position (tc_interl_lte.c:88-106,
// turbodecoder_win.h's inter / deinter).  Per (device, K), built once.
std::map<std::pair<int, uint32_t>, const uint16_t*> g_qpp8;

const uint16_t* qpp8_table(uint32_t K, uint32_t nsb, int idx)
{
  std::lock_guard<std::mutex> lk(g_mu);
  const auto                  key = std::make_pair(cur_dev(), K);
  auto                        it  = g_qpp8.find(key);
  if (it != g_qpp8.end()) {
    return it->second;
  }
  const uint64_t        f1 = kF1[idx], f2 = kF2[idx], Ls = K / nsb;
  std::vector<uint16_t> h(K);
  for (uint64_t j = 0; j < K; j++) {
    const uint64_t n  = (j % nsb) * Ls + j / nsb;            // natural position of SB index j
    const uint64_t fn = ((f2 * n % K) * n + f1 * n) % K;     // its QPP image
    h[j]              = (uint16_t)((fn % Ls) * nsb + fn / Ls);  // back to the SB index
  }
  uint16_t* d = nullptr;
  if (hipMalloc((void**)&d, K * sizeof(uint16_t)) != hipSuccess ||
      hipMemcpy(d, h.data(), K * sizeof(uint16_t), hipMemcpyHostToDevice) != hipSuccess) {
    hipFree(d);
    return nullptr;
  }
  g_qpp8[key] = d;
  return d;
}

}  // namespace

namespace srsran_amd {
// QPP coefficients of code block size index idx (36.212 Table 5.1.3-3), for the encoder
void qpp_coeffs(uint32_t idx, uint32_t* f1, uint32_t* f2)
{
  *f1 = kF1[idx];
  *f2 = kF2[idx];
}
}  // namespace srsran_amd

namespace srsran_amd {

int tdec_cb_index(uint32_t K) { return cb_index(K); }

int tdec_sch_enqueue(uint32_t      K,
                     const TdecCb* d_cbs,
                     uint32_t      ncb,
                     uint8_t*      d_out,
                     uint32_t      out_stride,
                     uint8_t*      d_noi,
                     uint8_t*      d_crc_ok,
                     int           n_end,
                     hipStream_t   stream)
{
  if (ncb == 0) {
    return SRSRAN_SUCCESS;
  }
  Config* c = get_config(K, auto_nsb(K));
  const XpowTables* xp = xpow_tables();
  if (!c || !xp) {
    return SRSRAN_ERROR;
  }
  TdecArgs a   = c->proto;
  a.in         = nullptr;
  a.in_stride  = 0;
  a.layout_sb  = c->nsb > 1 ? 1 : 0;  // soft buffer layout (rm_turbo.c:403-418)
  a.ncb        = ncb;
  a.n_start    = 0;
  a.n_end      = n_end > 0 ? n_end : 1;
  a.out        = d_out;
  a.tfwd       = c->d_tfwd;
  a.trev       = c->d_trev;
  a.tfwd_nat   = c->d_tfwd_nat;
  a.trev_nat   = c->d_trev_nat;
  a.state      = nullptr;
  a.cbs        = d_cbs;
  a.out_stride = out_stride;
  a.noi_out    = d_noi;
  a.crc_ok     = d_crc_ok;
  a.xpow_a     = xp->d[0];
  a.xpow_b     = xp->d[1];
  a.min_iters  = 2;  // SRSRAN_PDSCH_MIN_TDEC_ITERS (sch.c:35)
  hipError_t e = tdec_launch(c->nsb, a, stream);
  if (e != hipSuccess) {
    fprintf(stderr, "[srsran_sch] turbo launch failed: %s\n", hipGetErrorString(e));
    return SRSRAN_ERROR;
  }
  return SRSRAN_SUCCESS;
}

}  // namespace srsran_amd

namespace {
// Scratch of one 8-bit launch (the beta of a MAP pass / the widened int16 input), stream-ordered: allocated on
// the launch's stream and released on it behind the launch, so nothing outlives the call, no process-wide cache
// keyed by stream, no synchronisation (the device memory pool recycles the bytes).
struct Scratch8 {
  void*       p = nullptr;
  hipStream_t s = nullptr;
  Scratch8(hipStream_t stream, size_t bytes) : s(stream)
  {
    if (hipMallocAsync(&p, bytes, stream) != hipSuccess) {
      p = nullptr;
    }
  }
  ~Scratch8()
  {
    if (p) {
      hipFreeAsync(p, s);
    }
  }
  Scratch8(const Scratch8&)            = delete;
  Scratch8& operator=(const Scratch8&) = delete;
};
}  // namespace

namespace srsran_amd {
// DL-SCH decode with llr_is_8bit of ncb blocks of K > 800 (the 8-bit window decoders, 16 / 32 sub-blocks): int8 soft
// buffers in the 8-bit layout, CRC early stop after >= 2 half-iterations, at most n_end half-iterations
int tdec8_sch_enqueue(uint32_t      K,
                      const TdecCb* d_cbs,
                      uint32_t      ncb,
                      uint8_t*      d_out,
                      uint32_t      out_stride,
                      uint8_t*      d_noi,
                      uint8_t*      d_crc_ok,
                      int           n_end,
                      hipStream_t   stream)
{
  if (ncb == 0) {
    return SRSRAN_SUCCESS;
  }
  const int      idx = cb_index(K);
  const uint32_t nsb = srsran_tdec_autoimp_get_subblocks_8bit(K);
  const XpowTables* xp = xpow_tables();
  if (idx < 0 || (nsb != 16 && nsb != 32) || !xp) {
    return SRSRAN_ERROR;
  }
  Tdec8Args a{};
  a.in         = nullptr;
  a.layout_sb  = 1;
  a.K          = K;
  a.ncb        = ncb;
  a.n_end      = n_end > 0 ? n_end : 1;
  a.out        = d_out;
  a.cbs        = d_cbs;
  a.out_stride = out_stride;
  a.noi_out    = d_noi;
  a.crc_ok     = d_crc_ok;
  a.xpow_a     = xp->d[0];
  a.xpow_b     = xp->d[1];
  a.min_iters  = 2;  // SRSRAN_PDSCH_MIN_TDEC_ITERS (sch.c:35)
  a.qpp        = qpp8_table(K, nsb, idx);
  if (!a.qpp) {
    return SRSRAN_ERROR;
  }
  Scratch8 beta(stream, tdec8bit_beta_bytes((int)nsb, K, ncb));
  a.beta = (uint2*)beta.p;
  if (!a.beta) {
    return SRSRAN_ERROR;
  }
  const hipError_t e = tdec8bit_launch((int)nsb, a, stream);
  tdec_set_last_kernel(nsb == 32 ? "tdec8bit_kernel<32>" : "tdec8bit_kernel<16>");
  if (e != hipSuccess) {
    fprintf(stderr, "[srsran_sch] 8-bit turbo launch failed: %s\n", hipGetErrorString(e));
    return SRSRAN_ERROR;
  }
  return SRSRAN_SUCCESS;
}
}  // namespace srsran_amd

extern "C" {

uint32_t srsran_tdec_autoimp_get_subblocks(uint32_t long_cb)
{
  if (!(long_cb % 16) && long_cb > 800) {
    return 16;
  }
  if (!(long_cb % 8) && long_cb > 400) {
    return 8;
  }
  return 0;
}

uint32_t srsran_tdec_autoimp_get_subblocks_8bit(uint32_t long_cb)
{
  if (!(long_cb % 32) && long_cb > 2048) {
    return 32;
  }
  if (!(long_cb % 16) && long_cb > 800) {
    return 16;
  }
  if (!(long_cb % 8) && long_cb > 400) {
    return 8;
  }
  return 0;
}

int srsran_tdec_gpu_available(void)
{
  std::lock_guard<std::mutex> lk(g_mu);
  return have_gpu() ? 1 : 0;
}

const char* srsran_tdec_gpu_kernel_name(uint32_t long_cb)
{
  switch (auto_nsb(long_cb)) {
    case 16:
      return "tdec_kernel<16>";
    case 8:
      return "tdec_kernel<8>";
    default:
      return "tdec_kernel<1>";
  }
}

const char* srsran_tdec_gpu_last_kernel(void) { return tdec_last_kernel(); }

void srsran_tdec_gpu_set_pair_threshold(uint32_t nof_cb) { tdec16_set_min_cb(nof_cb); }

uint32_t srsran_tdec_gpu_get_pair_threshold(void) { return tdec16_min_cb(); }

void srsran_tdec_gpu_set_w8_max_k(uint32_t k) { tdecs_set_w8_max_k(k); }

uint32_t srsran_tdec_gpu_get_w8_max_k(void) { return tdecs_w8_max_k(); }

void srsran_tdec_gpu_set_w8_fused_max_k(uint32_t k) { tdecs_set_w8_fused_max_k(k); }

uint32_t srsran_tdec_gpu_get_w8_fused_max_k(void) { return tdecs_w8_fused_max_k(); }



void srsran_tdec_gpu_set_class_single_threshold(uint32_t nof_subblocks, uint32_t nof_cb)
{
  if (nof_subblocks == 16) {
    tdec16s_set_min_cb(nof_cb);
  } else if (nof_subblocks == 8) {
    tdec8s_set_min_cb(nof_cb);
  } else if (nof_subblocks <= 1) {
    tdec1s_set_min_cb(nof_cb);
  }
}

uint32_t srsran_tdec_gpu_get_class_single_threshold(uint32_t nof_subblocks)
{
  return nof_subblocks == 16 ? tdec16s_min_cb() : nof_subblocks == 8 ? tdec8s_min_cb() : tdec1s_min_cb();
}

void srsran_tdec_gpu_set_single_threshold(uint32_t nof_cb)
{
  tdec16s_set_min_cb(nof_cb);
  tdec8s_set_min_cb(nof_cb);
}

uint32_t srsran_tdec_gpu_get_single_threshold(void) { return tdec16s_min_cb(); }

void srsran_tdec_gpu_set_generic_single_threshold(uint32_t nof_cb) { tdec1s_set_min_cb(nof_cb); }

uint32_t srsran_tdec_gpu_get_generic_single_threshold(void) { return tdec1s_min_cb(); }

const char* srsran_tdec_gpu_kernel_name_batch(uint32_t long_cb, uint32_t nof_cb)
{
  const int nsb = auto_nsb(long_cb);
  if (nsb == 16) {
    const int k = tdec16_choice(nof_cb);
    if (k) {
      return k == 2 ? "tdec16s_kernel" : "tdec16_kernel";
    }
  }
  if (nsb == 8 && nof_cb >= tdec8s_min_cb()) {
    return "tdec8s_kernel";
  }
  if (nsb == 1 && nof_cb >= tdec1s_min_cb()) {
    return "tdec1s_kernel";
  }
  return srsran_tdec_gpu_kernel_name(long_cb);
}

int srsran_tdec_init(srsran_tdec_t* h, uint32_t max_long_cb)
{
  return srsran_tdec_init_manual(h, max_long_cb, SRSRAN_TDEC_AUTO);
}

int srsran_tdec_init_manual(srsran_tdec_t* h, uint32_t max_long_cb, srsran_tdec_impl_type_t dec_type)
{
  if (!h) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  memset(h, 0, sizeof(*h));
  if (dec_type != SRSRAN_TDEC_AUTO && dec_type != SRSRAN_TDEC_GENERIC && dec_type != SRSRAN_TDEC_SSE_WINDOW &&
      dec_type != SRSRAN_TDEC_AVX_WINDOW) {
    fprintf(stderr, "[srsran_tdec] decoder %d not supported\n", (int)dec_type);
    return SRSRAN_ERROR;
  }
  if (max_long_cb > SRSRAN_TCOD_MAX_LEN_CB) {
    return SRSRAN_ERROR;
  }
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!have_gpu()) {
      fprintf(stderr, "[srsran_tdec] no HIP device available\n");
      return SRSRAN_ERROR;
    }
  }
  Ctx* c = new Ctx();
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->d_in, kMaxIn * sizeof(short)) != hipSuccess ||
      hipMalloc(&c->d_out, SRSRAN_TCOD_MAX_LEN_CB / 8) != hipSuccess) {
    delete c;
    return SRSRAN_ERROR;
  }
  hipMemset(c->d_in, 0, kMaxIn * sizeof(short));
  h->gpu           = c;
  h->max_long_cb   = max_long_cb;
  h->dec_type      = dec_type;
  h->current_cbidx = -1;
  return SRSRAN_SUCCESS;
}

void srsran_tdec_free(srsran_tdec_t* h)
{
  if (!h) {
    return;
  }
  Ctx* c = (Ctx*)h->gpu;
  if (c) {
    if (c->stream) {
      hipStreamSynchronize(c->stream);
      hipStreamDestroy(c->stream);
    }
    hipFree(c->d_in);
    hipFree(c->d_out);
    hipFree(c->d_state);
    hipFree(c->d_bin);
    hipFree(c->d_bout);
    delete c;
  }
  memset(h, 0, sizeof(*h));
}

void srsran_tdec_force_not_sb(srsran_tdec_t* h)
{
  if (h) {
    h->force_not_sb = true;
  }
}

int srsran_tdec_new_cb(srsran_tdec_t* h, uint32_t long_cb)
{
  if (!h || long_cb > h->max_long_cb) {
    fprintf(stderr, "[srsran_tdec] TDEC was initialized for max_long_cb=%d\n", h ? h->max_long_cb : 0);
    return SRSRAN_ERROR;
  }
  h->n_iter          = 0;
  h->current_long_cb = long_cb;
  h->current_cbidx   = cb_index(long_cb);
  if (h->current_cbidx < 0) {
    fprintf(stderr, "[srsran_tdec] Invalid CB length %d\n", long_cb);
    return SRSRAN_ERROR;
  }
  return SRSRAN_SUCCESS;
}

int srsran_tdec_get_nof_iterations(srsran_tdec_t* h) { return h ? h->n_iter : 0; }

static size_t input_len(const srsran_tdec_t* h, const Config* c, uint32_t K)
{
  const bool sb = !h->force_not_sb && c->nsb > 1;
  return sb ? 3 * (K + 32) + 12 : 3 * K + 12;
}

void srsran_tdec_iteration(srsran_tdec_t* h, int16_t* input, uint8_t* output)
{
  if (!h || !h->gpu || h->current_cbidx < 0) {
    fprintf(stderr, "[srsran_tdec] Error CB index not set (call srsran_tdec_new_cb() first\n");
    return;
  }
  Ctx*           ctx = (Ctx*)h->gpu;
  const uint32_t K   = h->current_long_cb;
  Config*        c   = get_config(K, nsb_for(h, K));
  if (!c) {
    fprintf(stderr, "[srsran_tdec] unsupported K=%u\n", K);
    return;
  }
  const size_t st = 2 * (size_t)c->proto.xyw;
  if (!grow((void**)&ctx->d_state, &ctx->state_elems, st * sizeof(short))) {
    return;
  }
  if (h->n_iter == 0) {
    hipMemcpyAsync(ctx->d_in, input, input_len(h, c, K) * sizeof(short), hipMemcpyHostToDevice, ctx->stream);
  }
  if (enqueue(c, ctx->d_in, (uint32_t)kMaxIn, !h->force_not_sb, ctx->d_out, 1, h->n_iter, h->n_iter + 1,
              ctx->d_state, ctx->stream)) {
    return;
  }
  hipMemcpyAsync(output, ctx->d_out, K / 8, hipMemcpyDeviceToHost, ctx->stream);
  hipStreamSynchronize(ctx->stream);
  h->n_iter++;
}

int srsran_tdec_run_all(srsran_tdec_t* h, int16_t* input, uint8_t* output, uint32_t nof_iterations, uint32_t long_cb)
{
  if (srsran_tdec_new_cb(h, long_cb)) {
    return SRSRAN_ERROR;
  }
  int ret = srsran_tdec_run_all_batch(h, input, 0, output, 1, nof_iterations, long_cb);
  if (ret == SRSRAN_SUCCESS) {
    h->n_iter = nof_iterations > 0 ? (int)nof_iterations : 1;
  }
  return ret;
}

int srsran_tdec_run_all_batch(srsran_tdec_t* h,
                              const int16_t* input,
                              uint32_t       in_stride,
                              uint8_t*       output,
                              uint32_t       nof_cb,
                              uint32_t       nof_iterations,
                              uint32_t       long_cb)
{
  if (!h || !h->gpu || !input || !output) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (long_cb > h->max_long_cb || cb_index(long_cb) < 0) {
    return SRSRAN_ERROR;
  }
  if (nof_cb == 0) {
    return SRSRAN_SUCCESS;
  }
  Ctx*    ctx = (Ctx*)h->gpu;
  Config* c   = get_config(long_cb, nsb_for(h, long_cb));
  if (!c) {
    return SRSRAN_ERROR;
  }
  const size_t len = input_len(h, c, long_cb);
  if (in_stride == 0) {
    in_stride = (uint32_t)len;
  }
  if (in_stride < len) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  const size_t in_elems  = (size_t)in_stride * (nof_cb - 1) + len;
  const size_t out_bytes = (size_t)nof_cb * (long_cb / 8);
  if (!grow((void**)&ctx->d_bin, &ctx->bin_elems, in_elems * sizeof(short)) ||
      !grow((void**)&ctx->d_bout, &ctx->bout_bytes, out_bytes)) {
    return SRSRAN_ERROR;
  }
  hipMemcpyAsync(ctx->d_bin, input, in_elems * sizeof(short), hipMemcpyHostToDevice, ctx->stream);
  const int n_end = nof_iterations > 0 ? (int)nof_iterations : 1;  // do { } while (n_iter < nof_iterations)
  if (enqueue(c, ctx->d_bin, in_stride, !h->force_not_sb, ctx->d_bout, nof_cb, 0, n_end, nullptr, ctx->stream)) {
    return SRSRAN_ERROR;
  }
  hipMemcpyAsync(output, ctx->d_bout, out_bytes, hipMemcpyDeviceToHost, ctx->stream);
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) {
    fprintf(stderr, "[srsran_tdec] decode failed: %s\n", hipGetErrorString(hipGetLastError()));
    return SRSRAN_ERROR;
  }
  return SRSRAN_SUCCESS;
}

int srsran_tdec_gpu_run_batch(uint32_t       long_cb,
                              const int16_t* d_input,
                              uint32_t       in_stride,
                              int            layout_sb,
                              uint8_t*       d_output,
                              uint32_t       nof_cb,
                              uint32_t       nof_iterations,
                              void*          stream)
{
  if (!d_input || !d_output || cb_index(long_cb) < 0) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  Config* c = get_config(long_cb, auto_nsb(long_cb));
  if (!c) {
    return SRSRAN_ERROR;
  }
  const uint32_t len = (layout_sb && c->nsb > 1) ? 3 * (long_cb + 32) + 12 : 3 * long_cb + 12;
  if (in_stride < len) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  const int n_end = nof_iterations > 0 ? (int)nof_iterations : 1;
  return enqueue(c, d_input, in_stride, layout_sb, d_output, nof_cb, 0, n_end, nullptr, (hipStream_t)stream);
}

namespace {
// Internal fork/join stream pool for srsran_tdec_gpu_run_multi (per device).
constexpr int kPoolStreams = 4;
// Device descriptors of one fused multi-size launch (per decoder class).
struct MultiDesc {
  char*      h_stage = nullptr;  // pinned: TdecArgs[n] | first[n]
  char*      d_stage = nullptr;
  size_t     cap     = 0;
  hipEvent_t copied  = nullptr;  // the last upload from h_stage finished
  bool       used    = false;
};

struct StreamPool {
  int         device = -1;
  hipStream_t s[kPoolStreams];
  hipEvent_t  done[kPoolStreams];
  hipEvent_t  fork;
  hipEvent_t  large_done;  // the 16-step part's largest sizes finished (gates the other classes, tdec_gate())
  MultiDesc   md[6];  // launch entries: 16 (16-step, large K), 16 (16-step, mid K), 16 (8-step part), 8, generic x 2
};
std::mutex               g_pool_mu;
std::vector<StreamPool*> g_pools;

// How the classes of a fused multi-size call share the device (SRSRAN_AMD_TDEC_MULTI, read once):
// 0 "streams": one pool stream a class, equal priority; 1 "priority": the first (longest) class's stream at the
// device's highest priority, the others at the lowest; 2 "serial": every class on one stream, longest first.
int multi_mode()
{
  static const int m = [] {
    const char* e = getenv("SRSRAN_AMD_TDEC_MULTI");
    return !e ? 0 : !strcmp(e, "priority") ? 1 : !strcmp(e, "serial") ? 2 : 0;
  }();
  return m;
}

StreamPool* get_pool()
{
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    return nullptr;
  }
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (auto* p : g_pools) {
    if (p->device == dev) {
      return p;
    }
  }
  StreamPool* p = new StreamPool();
  p->device     = dev;
  int lo = 0, hi = 0;
  if (multi_mode() == 1 && hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) {
    lo = hi = 0;
  }
  for (int i = 0; i < kPoolStreams; i++) {
    if (hipStreamCreateWithPriority(&p->s[i], hipStreamNonBlocking, i == 0 ? hi : lo) != hipSuccess ||
        srsran_amd::ring_event_create(&p->done[i]) != hipSuccess) {
      return nullptr;
    }
  }
  if (srsran_amd::ring_event_create(&p->fork) != hipSuccess || srsran_amd::ring_event_create(&p->large_done) != hipSuccess) {
    return nullptr;
  }
  for (auto& m : p->md) {
    if (srsran_amd::ring_event_create(&m.copied) != hipSuccess) {
      return nullptr;
    }
  }
  g_pools.push_back(p);
  return p;
}

// The generic class's quad launch sizes its LDS for its largest K (about 45 KB a workgroup at K = 400: three a
// CU); its sizes up to this K run as a second launch with LDS for them, more workgroups a CU
// (SRSRAN_AMD_TDEC_GEN_CUT, read once; 0 = one launch).
uint32_t gen_cut()
{
  static const uint32_t c = [] {
    const char* e = getenv("SRSRAN_AMD_TDEC_GEN_CUT");
    return e ? (uint32_t)atoi(e) : 0u;
  }();
  return c;
}

// The 16-step part of a fused 16-sub-block class is cut once more at this K (SRSRAN_AMD_TDEC_MIDCUT, read once;
// 0 = one launch): its sizes above run first with K = 6144's LDS a workgroup (two a CU, nothing else fits beside
// them), its sizes up to the cut follow on the same stream with their own, smaller LDS figure -- room beside them
// for the 8-step part's, the 8-sub-block class's and the generic class's workgroups.
uint32_t tdec_midcut()
{
  static const uint32_t c = [] {
    const char* e = getenv("SRSRAN_AMD_TDEC_MIDCUT");
    return e ? (uint32_t)atoi(e) : 3072u;
  }();
  return c;
}
// With a mid cut, the other classes' launches wait for the large sizes to finish (SRSRAN_AMD_TDEC_GATE, read once;
// default on): started at once they only take CUs the large workgroups would have used, since no large workgroup
// leaves room beside it.
bool tdec_gate()
{
  static const bool g = [] {
    const char* e = getenv("SRSRAN_AMD_TDEC_GATE");
    return e ? atoi(e) != 0 : true;
  }();
  return g;
}

// Rough serial-latency model used only to order launches (longest first).
double launch_cost(uint32_t K, uint32_t ncb)
{
  const int    nsb   = auto_nsb(K);
  const double chain = nsb > 1 ? 3.0 * (K / nsb) + 160.0 : 3.0 * (K + 3);
  const double waves = (double)ncb * 4 * nsb / 64.0;
  return chain * (1.0 + waves / 1024.0);
}
}  // namespace

int srsran_tdec_gpu_run_multi(uint32_t              nof_groups,
                              const uint32_t*       long_cb,
                              const int16_t* const* d_input,
                              const uint32_t*       in_stride,
                              int                   layout_sb,
                              uint8_t* const*       d_output,
                              const uint32_t*       nof_cb,
                              uint32_t              nof_iterations,
                              void*                 stream)
{
  if (nof_groups == 0) {
    return SRSRAN_SUCCESS;
  }
  if (!long_cb || !d_input || !in_stride || !d_output || !nof_cb) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  std::vector<Config*>  cfg(nof_groups);
  std::vector<uint32_t> order(nof_groups);
  for (uint32_t g = 0; g < nof_groups; g++) {
    if (cb_index(long_cb[g]) < 0 || !d_input[g] || !d_output[g]) {
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
    cfg[g] = get_config(long_cb[g], auto_nsb(long_cb[g]));
    if (!cfg[g]) {
      return SRSRAN_ERROR;
    }
    const uint32_t len = (layout_sb && cfg[g]->nsb > 1) ? 3 * (long_cb[g] + 32) + 12 : 3 * long_cb[g] + 12;
    if (in_stride[g] < len) {
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
    order[g] = g;
  }
  std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
    return launch_cost(long_cb[a], nof_cb[a]) > launch_cost(long_cb[b], nof_cb[b]);
  });
  StreamPool* p = get_pool();
  if (!p) {
    return SRSRAN_ERROR;
  }
  hipStream_t user = (hipStream_t)stream;
  if (hipEventRecord(p->fork, user) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  for (int i = 0; i < kPoolStreams; i++) {
    hipStreamWaitEvent(p->s[i], p->fork, 0);
  }
  const int n_end = nof_iterations > 0 ? (int)nof_iterations : 1;
  int       ret   = SRSRAN_SUCCESS;
  // One fused launch per decoder class (16 / 8 / generic): the sizes of a class share one grid
  // (more workgroups in flight than per-size launches, no per-launch tail); classes run on
  // separate pool streams, longest first.  A single-lane 16-sub-block class is cut in two at
  // tdecs_w8_fused_max_k(): its sizes up to there run the 8-step-window build (fewer registers and
  // little LDS a workgroup: their workgroups can share SIMDs with the large sizes' ones) as their own
  // launch.
  // launch entries: 16 (16-step, K > mid cut), 16 (16-step, cut < K <= mid cut), 16 (8-step part), 8, generic x 2
  const int      cls_nsb[6] = {16, 16, 16, 8, 1, 1};
  const int      cls_st[6]  = {0, 0, 1, 2, 3, 3};  // pool stream of each entry (both 16-step parts: one stream)
  const uint32_t midcut     = tdec_midcut();
  bool           gated      = false;
  bool           mid_run    = false;  // entry 1 launched: the 16-step part was cut at midcut
  for (int ci = 0; ci < 6 && ret == SRSRAN_SUCCESS; ci++) {
    if (ci == 1 && hipEventRecord(p->large_done, p->s[0]) != hipSuccess) {  // behind the large sizes (entry 0)
      ret = SRSRAN_ERROR;
      break;
    }
    // with the 16-step part cut at midcut, the other classes start when its large sizes are done, beside the mid part
    gated = ci >= 2 && mid_run && tdec_gate() && multi_mode() != 2;
    std::vector<uint32_t> gs;
    uint32_t              cls_cb = 0;  // blocks of the whole class (decides the kernel)
    for (uint32_t i = 0; i < nof_groups; i++) {
      if (cfg[order[i]]->nsb == cls_nsb[ci] && nof_cb[order[i]] > 0) {
        gs.push_back(order[i]);
        cls_cb += nof_cb[order[i]];
      }
    }
    if (gs.empty()) {
      continue;
    }
    // 2 single lane (tdecs_kernel.hip), 1 lane pair (16 sub-blocks only), 0 quad
    const int kind = cls_nsb[ci] == 1               ? (cls_cb >= tdec1s_min_cb() ? 2 : 0)   // natural layout
                     : !layout_sb                   ? 0
                     : cls_nsb[ci] == 16            ? tdec16_choice(cls_cb)
                                                    : (cls_cb >= tdec8s_min_cb() ? 2 : 0);
    const uint32_t cut = std::max(tdecs_w8_max_k(), tdecs_w8_fused_max_k());
    if (cls_nsb[ci] == 16 && kind == 2) {  // entry 0: K above the mid cut; entry 1: up to it; entry 2: up to the cut
      const uint32_t lo = ci == 0 ? std::max(cut, midcut) : ci == 1 ? cut : 0;
      const uint32_t hi = ci == 0 ? UINT32_MAX : ci == 1 ? std::max(cut, midcut) : cut;
      gs.erase(std::remove_if(gs.begin(), gs.end(),
                              [&](uint32_t g) { return !(cfg[g]->proto.K > lo && cfg[g]->proto.K <= hi); }),
               gs.end());
    } else if (ci == 1 || ci == 2) {
      gs.clear();  // no 16-step mid part / 8-step part outside the single-lane class
    } else if (ci >= 4 && kind == 0 && gen_cut() > 0) {  // generic quad: K above the cut, then the rest
      const bool small = ci == 5;
      gs.erase(std::remove_if(gs.begin(), gs.end(), [&](uint32_t g) { return (cfg[g]->proto.K <= gen_cut()) != small; }),
               gs.end());
    } else if (ci == 5) {
      gs.clear();  // one generic launch
    }
    if (gs.empty()) {
      continue;
    }
    mid_run        = mid_run || ci == 1;
    hipStream_t st = p->s[multi_mode() == 2 ? 0 : cls_st[ci]];
    if (gated && st != p->s[0] && hipStreamWaitEvent(st, p->large_done, 0) != hipSuccess) {
      ret = SRSRAN_ERROR;
      break;
    }
    if (gs.size() == 1) {
      const uint32_t g = gs[0];
      ret = enqueue(cfg[g], d_input[g], in_stride[g], layout_sb, d_output[g], nof_cb[g], 0, n_end, nullptr, st);
      continue;
    }
    const int  nsbc = cls_nsb[ci];
    uint32_t   kmax = 0;
    for (uint32_t g : gs) {
      kmax = std::max(kmax, cfg[g]->proto.K);
    }
    const bool w8  = kind == 2 && nsbc > 1 && kmax <= (nsbc == 16 ? cut : tdecs_w8_max_k());  // 8-step windows
    const int  cpw  = kind == 2   ? (nsbc == 16 ? tdecs16::cpw() : nsbc == 8 ? tdecs8::cpw() : tdecs1::cpw())
                      : kind == 1 ? tdec16_cpw()
                                  : tdec_cpw(nsbc);
    const size_t   n     = gs.size();
    const size_t   abyte = n * sizeof(TdecArgs);
    const size_t   need  = abyte + n * sizeof(uint32_t);
    MultiDesc&     m     = p->md[ci];
    if (m.used) {
      hipEventSynchronize(m.copied);
    }
    if (need > m.cap) {
      hipStreamSynchronize(st);
      hipHostFree(m.h_stage);
      hipFree(m.d_stage);
      m.h_stage = m.d_stage = nullptr;
      m.cap                 = 0;
      if (hipHostMalloc((void**)&m.h_stage, 2 * need) != hipSuccess || hipMalloc((void**)&m.d_stage, 2 * need) != hipSuccess) {
        return SRSRAN_ERROR;
      }
      m.cap = 2 * need;
    }
    TdecArgs* ha    = reinterpret_cast<TdecArgs*>(m.h_stage);
    uint32_t* hf    = reinterpret_cast<uint32_t*>(m.h_stage + abyte);
    uint32_t  nblk  = 0;
    size_t    lds   = 0;
    for (size_t k = 0; k < n; k++) {
      const uint32_t g = gs[k];
      const Config*  c = cfg[g];
      TdecArgs       a = c->proto;
      a.in             = d_input[g];
      a.in_stride      = in_stride[g];
      a.layout_sb      = c->nsb > 1 ? layout_sb : 0;
      a.ncb            = nof_cb[g];
      a.n_start        = 0;
      a.n_end          = n_end;
      a.out            = d_output[g];
      a.tfwd           = c->d_tfwd;
      a.trev           = c->d_trev;
      a.tfwd_nat       = c->d_tfwd_nat;
      a.trev_nat       = c->d_trev_nat;
      a.state          = nullptr;
      ha[k]            = a;
      hf[k]            = nblk;
      nblk += (nof_cb[g] + cpw - 1) / cpw;
      lds = std::max(lds, kind == 2   ? (nsbc == 16  ? (w8 ? tdecs16w8::lds_bytes(a) : tdecs16::lds_bytes(a))
                                         : nsbc == 8 ? (w8 ? tdecs8w8::lds_bytes(a) : tdecs8::lds_bytes(a))
                                                     : tdecs1::lds_bytes(a))
                          : kind == 1 ? tdec16_lds_bytes(a)
                                      : tdec_lds_bytes(c->nsb, a.xyw, a.M));
    }
    if (hipMemcpyAsync(m.d_stage, m.h_stage, need, hipMemcpyHostToDevice, st) != hipSuccess) {
      return SRSRAN_ERROR;
    }
    hipEventRecord(m.copied, st);
    m.used = true;
    const TdecArgs* dg = reinterpret_cast<const TdecArgs*>(m.d_stage);
    const uint32_t* df = reinterpret_cast<const uint32_t*>(m.d_stage + abyte);
    if ((kind == 2   ? (nsbc == 16  ? (w8 ? tdecs16w8::multi_launch(dg, df, (int)n, nblk, lds, st)
                                          : tdecs16::multi_launch(dg, df, (int)n, nblk, lds, st))
                        : nsbc == 8 ? (w8 ? tdecs8w8::multi_launch(dg, df, (int)n, nblk, lds, st)
                                          : tdecs8::multi_launch(dg, df, (int)n, nblk, lds, st))
                                    : tdecs1::multi_launch(dg, df, (int)n, nblk, lds, st))
         : kind == 1 ? tdec16_multi_launch(dg, df, (int)n, nblk, lds, st)
                     : tdec_multi_launch(cls_nsb[ci], dg, df, (int)n, nblk, lds, st)) != hipSuccess) {
      ret = SRSRAN_ERROR;
    }
  }
  for (int i = 0; i < kPoolStreams; i++) {
    hipEventRecord(p->done[i], p->s[i]);
    hipStreamWaitEvent(user, p->done[i], 0);
  }
  return ret;
}

#ifdef TDECS_STAMPS
// Diagnostic build only (lib/stamps/libsrsran_4g_amd.so, tools/tdec_stamps.py): every single-lane
// launch from now on writes its phase-boundary clock stamps to d_buf ([workgroup][wave][64] u64), or
// stops when d_buf is NULL.
int srsran_tdec_gpu_debug_set_stamps(void* d_buf)
{
  using namespace srsran_amd;
  return tdecs16::set_stamps(d_buf) == hipSuccess && tdecs8::set_stamps(d_buf) == hipSuccess &&
                 tdecs16w8::set_stamps(d_buf) == hipSuccess && tdecs8w8::set_stamps(d_buf) == hipSuccess
             ? SRSRAN_SUCCESS
             : SRSRAN_ERROR;
}
#endif

// ---- 8-bit LLR decoders (turbodecoder.c:455-483, 551-577) ----

// AUTO: K > 2048 on the AVX2 8-bit window decoder (32 sub-blocks), 800 < K <= 2048 on the SSE 8-bit
// window decoder (16), smaller K on the 16-bit decoders after widening the input (convert_8_to_16);
// a manually selected 16-bit decoder widens as well (tdec_iteration_8 with dec_type != AUTO).
int srsran_tdec_gpu_run_batch_8bit(uint32_t      long_cb,
                                   const int8_t* d_input,
                                   uint32_t      in_stride,
                                   int           layout_sb,
                                   uint8_t*      d_output,
                                   uint32_t      nof_cb,
                                   uint32_t      nof_iterations,
                                   void*         stream)
{
  using namespace srsran_amd;
  const int idx = cb_index(long_cb);
  if (!d_input || !d_output || idx < 0) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (nof_cb == 0) {
    return SRSRAN_SUCCESS;
  }
  hipStream_t    s     = (hipStream_t)stream;
  const uint32_t nsb8  = srsran_tdec_autoimp_get_subblocks_8bit(long_cb);
  const bool     sb    = layout_sb && nsb8 > 0;
  const uint32_t len   = sb ? 3 * (long_cb + 32) + 12 : 3 * long_cb + 12;
  const int      n_end = nof_iterations > 0 ? (int)nof_iterations : 1;
  if (in_stride < len) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (nsb8 == 16 || nsb8 == 32) {
    Tdec8Args a{};
    a.in        = d_input;
    a.in_stride = in_stride;
    a.layout_sb = sb ? 1 : 0;
    a.K         = long_cb;
    a.ncb       = nof_cb;
    a.n_end     = n_end;
    a.out       = d_output;
    a.qpp       = qpp8_table(long_cb, nsb8, idx);
    if (!a.qpp) {
      return SRSRAN_ERROR;
    }
    Scratch8 beta(s, tdec8bit_beta_bytes((int)nsb8, long_cb, nof_cb));
    if (!beta.p) {
      return SRSRAN_ERROR;
    }
    a.beta           = (uint2*)beta.p;
    const hipError_t e = tdec8bit_launch((int)nsb8, a, s);
    tdec_set_last_kernel(nsb8 == 32 ? "tdec8bit_kernel<32>" : "tdec8bit_kernel<16>");
    return e == hipSuccess ? SRSRAN_SUCCESS : SRSRAN_ERROR;
  }
  // 16-bit decoder on the widened input
  Scratch8 wbuf(s, (size_t)nof_cb * len * sizeof(short));
  short*   wide = (short*)wbuf.p;
  if (!wide) {
    return SRSRAN_ERROR;
  }
  return tdec8bit_widen(d_input, in_stride, wide, len, nof_cb, s) == hipSuccess
             ? srsran_tdec_gpu_run_batch(long_cb, wide, len, sb ? 1 : 0, d_output, nof_cb, nof_iterations, stream)
             : SRSRAN_ERROR;
}

int srsran_tdec_run_all_8bit(srsran_tdec_t* h, int8_t* input, uint8_t* output, uint32_t nof_iterations, uint32_t long_cb)
{
  if (!h || !h->gpu || !input || !output) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (srsran_tdec_new_cb(h, long_cb)) {
    return SRSRAN_ERROR;
  }
  const uint32_t nsb8 = srsran_tdec_autoimp_get_subblocks_8bit(long_cb);
  if (h->dec_type != SRSRAN_TDEC_AUTO || nsb8 < 16) {
    // convert_8_to_16 + the 16-bit decoder of this K (or the manually selected one)
    Config* c = get_config(long_cb, nsb_for(h, long_cb));
    if (!c) {
      return SRSRAN_ERROR;
    }
    const size_t         n = input_len(h, c, long_cb);
    std::vector<int16_t> wide(n);
    for (size_t i = 0; i < n; i++) {
      wide[i] = input[i];
    }
    return srsran_tdec_run_all(h, wide.data(), output, nof_iterations, long_cb);
  }
  Ctx*           ctx = (Ctx*)h->gpu;
  const bool     sb  = !h->force_not_sb;
  const uint32_t len = sb ? 3 * (long_cb + 32) + 12 : 3 * long_cb + 12;
  if (!grow((void**)&ctx->d_bin, &ctx->bin_elems, len) || !grow((void**)&ctx->d_bout, &ctx->bout_bytes, long_cb / 8)) {
    return SRSRAN_ERROR;
  }
  hipMemcpyAsync(ctx->d_bin, input, len, hipMemcpyHostToDevice, ctx->stream);
  int ret = srsran_tdec_gpu_run_batch_8bit(long_cb, (const int8_t*)ctx->d_bin, len, sb ? 1 : 0, ctx->d_bout, 1,
                                           nof_iterations, ctx->stream);
  if (ret != SRSRAN_SUCCESS) {
    return ret;
  }
  hipMemcpyAsync(output, ctx->d_bout, long_cb / 8, hipMemcpyDeviceToHost, ctx->stream);
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) {
    fprintf(stderr, "[srsran_tdec] 8-bit decode failed: %s\n", hipGetErrorString(hipGetLastError()));
    return SRSRAN_ERROR;
  }
  h->n_iter = nof_iterations > 0 ? (int)nof_iterations : 1;
  return SRSRAN_SUCCESS;
}

// One more half-iteration and a decision (turbodecoder.c:551-558): the decoder state after n
// half-iterations is a function of the input alone, so the n + 1 half-iterations run from the input.
void srsran_tdec_iteration_8bit(srsran_tdec_t* h, int8_t* input, uint8_t* output)
{
  if (!h || !h->gpu || h->current_cbidx < 0) {
    fprintf(stderr, "[srsran_tdec] Error CB index not set (call srsran_tdec_new_cb() first\n");
    return;
  }
  const int n = h->n_iter + 1;
  if (srsran_tdec_run_all_8bit(h, input, output, (uint32_t)n, h->current_long_cb) == SRSRAN_SUCCESS) {
    h->n_iter = n;
  }
}

}  // extern "C"
