// srsran_4g_amd/csrc/tx_api.cpp -- the reference's single-code-block transmit entry points over the GPU encoder:
// srsran_tcod_{init,free,encode} (turbocoder.c:44-185) and srsran_rm_turbo_tx_lut (rm_turbo.c:345-388), host
// pointers, host-synchronous (the per-thread default stream), as the reference's callers expect.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "../../include/srsran_sch.h"
#include "devkey.h"
#include "enc_kernel.h"

namespace srsran_amd {
void qpp_coeffs(uint32_t idx, uint32_t* f1, uint32_t* f2);
}

namespace {
using srsran_amd::RmTxLut;

struct TcodGpu {
  uint8_t* d_in  = nullptr;
  uint8_t* d_out = nullptr;
};

// rm_turbo.c:72-73 (36.212 Table 5.1.4-1): the inter-column permutation of the sub-block interleaver
const uint8_t kPerm[32] = {0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30,
                           1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31};

// The interleaver tables of srsran_rm_turbo_gentables for one code block size (rm_turbo.c:95-170, 276-303): w bit
// i <- systematic bit sys[i] (i < K + 4), w bit K + 4 + i <- parity bit par[i] (v1 and the shifted v2 interlaced,
// dummy bits skipped), and k0 of every rv as a position in the dummy-free w
struct RmTxTab {
  uint16_t* d_sys = nullptr;
  uint16_t* d_par = nullptr;
  int       k0[4] = {0, 0, 0, 0};
};

bool build_tab(uint32_t K, RmTxTab& t)
{
  const int in_len = 3 * (int)K + 12;
  const int nrows  = (in_len / 3 - 1) / 32 + 1;
  const int K_p    = nrows * 32;
  const int ndummy = K_p - in_len / 3 > 0 ? K_p - in_len / 3 : 0;
  int       k0v[4][2];
  for (int i = 0; i < 4; i++) {
    k0v[i][0] = nrows * (2 * (uint16_t)ceilf((float)(3 * K_p) / (float)(8 * nrows)) * i + 2);
    k0v[i][1] = -1;
  }
  std::vector<uint16_t> sys(K + 4), par(2 * (K + 4));
  // srsran_rm_turbo_gentable_systematic
  bool last_is_null = true;
  int  k_b = 0, buff_idx = 0;
  for (int j = 0; j < 32; j++) {
    for (int i = 0; i < nrows; i++) {
      if (i * 32 + kPerm[j] >= ndummy) {
        sys[k_b++]   = (uint16_t)(i * 32 + kPerm[j] - ndummy);
        last_is_null = false;
      } else {
        last_is_null = true;
      }
      for (int k = 0; k < 4; k++) {
        if (k0v[k][1] == -1 && k0v[k][0] % (3 * nrows * 32) <= buff_idx && !last_is_null) {
          k0v[k][1] = k_b - 1;
        }
      }
      buff_idx++;
    }
  }
  // srsran_rm_turbo_gentable_parity (offset = in_len / 3)
  const int offset = in_len / 3;
  last_is_null     = true;
  k_b              = 0;
  int buff_idx0 = 0, buff_idx1 = 0;
  for (int j = 0; j < 32; j++) {
    for (int i = 0; i < nrows; i++) {
      if (i * 32 + kPerm[j] >= ndummy) {
        par[k_b++]   = (uint16_t)(i * 32 + kPerm[j] - ndummy);
        last_is_null = false;
      } else {
        last_is_null = true;
      }
      for (int k = 0; k < 4; k++) {
        if (k0v[k][1] == -1 && k0v[k][0] % (3 * K_p) <= 2 * buff_idx0 + K_p && !last_is_null) {
          k0v[k][1] = offset + k_b - 1;
        }
      }
      buff_idx0++;
      const int kidx = (kPerm[buff_idx1 / nrows] + 32 * (buff_idx1 % nrows) + 1) % K_p;
      if (kidx - ndummy >= 0) {
        par[k_b++]   = (uint16_t)(kidx - ndummy + offset);
        last_is_null = false;
      } else {
        last_is_null = true;
      }
      for (int k = 0; k < 4; k++) {
        if (k0v[k][1] == -1 && k0v[k][0] % (3 * K_p) <= 2 * buff_idx1 + 1 + K_p && !last_is_null) {
          k0v[k][1] = offset + k_b - 1;
        }
      }
      buff_idx1++;
    }
  }
  if (k_b != (int)par.size()) {
    return false;
  }
  for (int i = 0; i < 4; i++) {
    t.k0[i] = k0v[i][1];
  }
  return hipMalloc((void**)&t.d_sys, sys.size() * sizeof(uint16_t)) == hipSuccess &&
         hipMalloc((void**)&t.d_par, par.size() * sizeof(uint16_t)) == hipSuccess &&
         hipMemcpy(t.d_sys, sys.data(), sys.size() * sizeof(uint16_t), hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(t.d_par, par.data(), par.size() * sizeof(uint16_t), hipMemcpyHostToDevice) == hipSuccess;
}

std::mutex                                      g_tab_mu;
std::map<std::pair<int, uint32_t>, RmTxTab>     g_tabs;  // (device, cb_idx), built once, read-only

const RmTxTab* rm_tab(uint32_t cb_idx)
{
  std::lock_guard<std::mutex> lk(g_tab_mu);
  const auto                  key = std::make_pair(srsran_amd::cur_dev(), cb_idx);
  auto                        it  = g_tabs.find(key);
  if (it != g_tabs.end()) {
    return &it->second;
  }
  RmTxTab t;
  if (!build_tab((uint32_t)srsran_cbsegm_cbsize(cb_idx), t)) {
    hipFree(t.d_sys);
    hipFree(t.d_par);
    return nullptr;
  }
  return &(g_tabs[key] = t);
}

bool have_device()
{
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess && n > 0;
}
}  // namespace

extern "C" {

int srsran_tcod_init(srsran_tcod_t* h, uint32_t max_long_cb)
{
  if (!h || max_long_cb == 0 || max_long_cb > 6144) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  memset(h, 0, sizeof(*h));
  if (!have_device()) {
    fprintf(stderr, "[srsran_tcod] no HIP device\n");
    return SRSRAN_ERROR;
  }
  TcodGpu* g = new TcodGpu();
  h->gpu     = g;
  if (hipMalloc((void**)&g->d_in, max_long_cb) != hipSuccess ||
      hipMalloc((void**)&g->d_out, 3 * (size_t)max_long_cb + 12) != hipSuccess) {
    srsran_tcod_free(h);
    return SRSRAN_ERROR;
  }
  h->max_long_cb = max_long_cb;
  return SRSRAN_SUCCESS;
}

void srsran_tcod_free(srsran_tcod_t* h)
{
  if (!h) {
    return;
  }
  if (h->gpu) {
    TcodGpu* g = (TcodGpu*)h->gpu;
    hipFree(g->d_in);
    hipFree(g->d_out);
    delete g;
  }
  memset(h, 0, sizeof(*h));
}

int srsran_tcod_encode(srsran_tcod_t* h, uint8_t* input, uint8_t* output, uint32_t long_cb)
{
  if (!h || !h->gpu || !input || !output) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (long_cb > h->max_long_cb) {
    fprintf(stderr, "[srsran_tcod] Turbo coder initiated for max_long_cb=%u\n", h->max_long_cb);
    return -1;
  }
  const int idx = srsran_cbsegm_cbindex(long_cb);
  if (idx < 0) {
    fprintf(stderr, "[srsran_tcod] Invalid CB size %u\n", long_cb);
    return -1;
  }
  TcodGpu*    g  = (TcodGpu*)h->gpu;
  hipStream_t st = hipStreamPerThread;
  uint32_t    f1 = 0, f2 = 0;
  srsran_amd::qpp_coeffs((uint32_t)idx, &f1, &f2);
  if (hipMemcpyAsync(g->d_in, input, long_cb, hipMemcpyHostToDevice, st) != hipSuccess ||
      srsran_amd::tcod_launch(g->d_in, g->d_out, long_cb, f1, f2, st) != hipSuccess ||
      hipMemcpyAsync(output, g->d_out, 3 * (size_t)long_cb + 12, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  return SRSRAN_SUCCESS;
}

int srsran_rm_turbo_tx_lut(uint8_t* w_buff, uint8_t* systematic, uint8_t* parity, uint8_t* output, uint32_t cb_idx,
                           uint32_t out_len, uint32_t w_offset, uint32_t rv_idx)
{
  if (rv_idx >= 4 || cb_idx >= SRSRAN_NOF_TC_CB_SIZES || !w_buff || !output ||
      (rv_idx == 0 && (!systematic || !parity))) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (!have_device()) {
    fprintf(stderr, "[srsran_rm_turbo] no HIP device\n");
    return SRSRAN_ERROR;
  }
  const RmTxTab* t = rm_tab(cb_idx);
  if (!t) {
    return SRSRAN_ERROR;
  }
  const uint32_t K = (uint32_t)srsran_cbsegm_cbsize(cb_idx), in_len = 3 * K + 12, nwb = (in_len + 7) / 8;
  // where the reference's bit-selection loop cuts its copies (rm_turbo.c:369-382) and whether its last
  // srsran_bit_copy took the byte-aligned path, which clears the bits after the copy in the last byte (bit.c:688-694)
  uint32_t w_len = 0, r_ptr = (uint32_t)t->k0[rv_idx], last_dst = w_offset, last_src = r_ptr;
  while (w_len < out_len) {
    uint32_t cp_len = out_len - w_len;
    if (cp_len + r_ptr >= in_len) {
      cp_len = in_len - r_ptr;
    }
    last_dst = w_len + w_offset;
    last_src = r_ptr;
    r_ptr += cp_len;
    if (r_ptr >= in_len) {
      r_ptr -= in_len;
    }
    w_len += cp_len;
  }
  const uint32_t out_bytes = out_len ? (w_offset + out_len - 1) / 8 + 1 : 0;
  hipStream_t    st        = hipStreamPerThread;
  uint8_t*       d         = nullptr;
  const size_t   need      = 3 * (size_t)nwb + out_bytes + 64;
  if (hipMallocAsync((void**)&d, need, st) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  uint8_t* d_w = d;
  uint8_t* d_s = d + nwb;
  uint8_t* d_p = d + 2 * (size_t)nwb;
  uint8_t* d_o = d + 3 * (size_t)nwb;
  RmTxLut  a{};
  a.sys       = d_s;
  a.par       = d_p;
  a.tsys      = t->d_sys;
  a.tpar      = t->d_par;
  a.w_buff    = d_w;
  a.output    = d_o;
  a.K         = K;
  a.rv        = rv_idx;
  a.r_ptr     = (uint32_t)t->k0[rv_idx];
  a.out_len   = out_len;
  a.w_offset  = w_offset;
  a.zero_tail = (last_dst % 8 == 0 && last_src % 8 == 0) ? 1u : 0u;
  const size_t sys_bytes = (K + 4 + 7) / 8, par_bytes = (2 * (K + 4) + 7) / 8;
  bool ok = (rv_idx != 0 || (hipMemcpyAsync(d_s, systematic, sys_bytes, hipMemcpyHostToDevice, st) == hipSuccess &&
                              hipMemcpyAsync(d_p, parity, par_bytes, hipMemcpyHostToDevice, st) == hipSuccess)) &&
            (rv_idx == 0 || hipMemcpyAsync(d_w, w_buff, nwb, hipMemcpyHostToDevice, st) == hipSuccess) &&
            (out_bytes == 0 || hipMemcpyAsync(d_o, output, out_bytes, hipMemcpyHostToDevice, st) == hipSuccess) &&
            srsran_amd::rm_tx_lut_launch(a, st) == hipSuccess &&
            (rv_idx != 0 || hipMemcpyAsync(w_buff, d_w, nwb, hipMemcpyDeviceToHost, st) == hipSuccess) &&
            (out_bytes == 0 || hipMemcpyAsync(output, d_o, out_bytes, hipMemcpyDeviceToHost, st) == hipSuccess);
  hipFreeAsync(d, st);
  ok = hipStreamSynchronize(st) == hipSuccess && ok;
  return ok ? SRSRAN_SUCCESS : SRSRAN_ERROR;
}

}  // extern "C"
