// srsran_4g_amd/csrc/ldpc_api.cpp -- C-ABI host side of the HIP NR LDPC decoder.
//
// Implements include/srsran_ldpc.h (the srsran_ldpc_decoder_* surface of
// lib/include/srsran/phy/fec/ldpc/ldpc_decoder.h and create_compact_pcm of base_graph.h) over
// ldpc_kernel.hip.  Host semantics follow ldpc_decoder.c:
//   init (args check, geometry, compact PCM, default 10 iterations)   ldpc_decoder.c:552-648
//   rate-matched length clamp -> number of layers                     ldpc_decoder.c:48-70
//   return values (max_nof_iter / iterations until CRC / 0)           ldpc_decoder.c:72-95
// There is no CPU fallback: without a HIP device init fails with SRSRAN_ERROR.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

#include "../../include/srsran_ldpc.h"
#include "ldpc_internal.h"

#include "ldpc_bg_tables.inc"

using namespace srsran_amd;

namespace {

struct Graph {
  int                   M, N, K, ne;
  const unsigned short* rs;
  const unsigned char*  col;
  const unsigned short* V;  // this lifting size's set
};

// 38.212 Table 5.3.2-1: Z = a * 2^j, set index by a
int ls_index(int ls)
{
  static const int A[8] = {2, 3, 5, 7, 9, 11, 13, 15};
  if (ls < 2 || ls > MAX_LIFTSIZE) {
    return -1;
  }
  for (int i = 0; i < 8; i++) {
    int z = A[i];
    while (z < ls) {
      z *= 2;
    }
    if (z == ls) {
      return i;
    }
  }
  return -1;
}

bool graph(int bg, int ls, Graph& g)
{
  const int set = ls_index(ls);
  if (set < 0 || (bg != BG1 && bg != BG2)) {
    return false;
  }
  g.M   = bg == BG1 ? BG1M : BG2M;
  g.N   = bg == BG1 ? BG1Nfull : BG2Nfull;
  g.K   = g.N - g.M;
  g.rs  = bg == BG1 ? LDPC_BG1_ROW_START : LDPC_BG2_ROW_START;
  g.col = bg == BG1 ? LDPC_BG1_COL : LDPC_BG2_COL;
  g.V   = bg == BG1 ? LDPC_BG1_V[set] : LDPC_BG2_V[set];
  g.ne  = g.rs[g.M];
  return true;
}

struct Ctx {
  hipStream_t stream    = nullptr;
  uint32_t*   d_sh      = nullptr;
  int8_t*     d_in      = nullptr;  // single-codeword staging of the host-synchronous calls
  uint8_t*    d_out     = nullptr;
  uint8_t*    d_ret     = nullptr;
  uint8_t*    d_lut     = nullptr;  // scale(m), m = 0..127
  int         bits       = 8;  // LLR / message width: 8 (C, C_AVX2, C_AVX512) or 16 (S)
  int         scale_mode = LDPC_SCALE_SIMD;
  int         sf         = 0;
  std::map<uint64_t, uint32_t*> xpow;  // (poly, order) -> x^n mod P, n = 0 .. liftK
};

// x^n mod P for n = 0 .. nmax (P with its x^order bit)
std::vector<uint32_t> xpow_table(uint32_t poly, int order, int nmax)
{
  std::vector<uint32_t> t(nmax + 1);
  uint32_t              v    = 1;
  const uint32_t        mask = (1u << order) - 1u;
  for (int n = 0; n <= nmax; n++) {
    t[n] = v;
    v    = (v & (1u << (order - 1))) ? ((v << 1) ^ poly) : (v << 1);
    v &= mask;
  }
  return t;
}

void free_ctx(Ctx* c)
{
  if (!c) {
    return;
  }
  for (auto& kv : c->xpow) {
    hipFree(kv.second);
  }
  hipFree(c->d_sh);
  hipFree(c->d_in);
  hipFree(c->d_out);
  hipFree(c->d_ret);
  hipFree(c->d_lut);
  if (c->stream) {
    hipStreamDestroy(c->stream);
  }
  delete c;
}

void free_dec(void* o)
{
  srsran_ldpc_decoder_t* q = static_cast<srsran_ldpc_decoder_t*>(o);
  free_ctx(static_cast<Ctx*>(q->ptr));
  free(q->pcm);
  free(q->var_indices);
}

const uint32_t* xpow_for(srsran_ldpc_decoder_t* q, const srsran_crc_t* crc)
{
  Ctx*           c   = static_cast<Ctx*>(q->ptr);
  const uint64_t key = ((uint64_t)(uint32_t)crc->polynom << 8) | (uint32_t)crc->order;
  auto           it  = c->xpow.find(key);
  if (it != c->xpow.end()) {
    return it->second;
  }
  const auto t = xpow_table((uint32_t)crc->polynom, crc->order, q->liftK);
  uint32_t*  d = nullptr;
  if (hipMalloc(&d, t.size() * 4) != hipSuccess ||
      hipMemcpy(d, t.data(), t.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
    hipFree(d);
    return nullptr;
  }
  c->xpow[key] = d;
  return d;
}

// ldpc_decoder.c:48-70: clamp the rate-matched length and derive the processed layers
int layers_for(const srsran_ldpc_decoder_t* q, uint32_t len)
{
  if (len > (uint32_t)q->liftN - 2u * q->ls) {
    len = q->liftN - 2u * q->ls;
  }
  if (len < (uint32_t)(q->bgK + 2) * q->ls) {
    len = (uint32_t)(q->bgK + 2) * q->ls;
  }
  if (len % q->ls) {
    len = (len / q->ls + 1) * q->ls;
  }
  return (int)(len / q->ls) - q->bgK + 2;
}

// llr_stride in bytes; bits = width of the caller's LLRs (must match the decoder type)
int launch(srsran_ldpc_decoder_t* q, const void* d_llrs, int bits, uint32_t llr_stride, uint32_t nof_cw,
           uint32_t len, const srsran_crc_t* crc, uint8_t* d_message, uint32_t message_stride, int packed,
           uint8_t* d_ret, hipStream_t stream)
{
  Ctx* c = static_cast<Ctx*>(q->ptr);
  if (!c || !d_llrs || !d_message) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (bits != c->bits) {
    fprintf(stderr, "[srsran_4g_amd] LDPC: %d-bit LLRs given to a %d-bit decoder\n", bits, c->bits);
    return SRSRAN_ERROR;
  }
  if (crc && (crc->order != 16 && crc->order != 24)) {
    fprintf(stderr, "[srsran_4g_amd] LDPC: CRC order %d not supported\n", crc->order);
    return SRSRAN_ERROR;
  }
  if (packed && (q->liftK % 8)) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  LdpcArgs a;
  memset(&a, 0, sizeof(a));
  a.in         = d_llrs;
  a.llr_bits   = bits;
  a.in_stride  = llr_stride;
  a.out        = d_message;
  a.out_stride = message_stride;
  a.out_packed = packed;
  a.ret        = d_ret;
  a.ncw        = nof_cw;
  a.ls         = q->ls;
  a.cw_per_wg  = ldpc_cw_per_wg(q->ls, bits);
  a.n_layers   = layers_for(q, len);
  a.max_iter   = (int)q->max_nof_iter;
  a.scale_mode = c->scale_mode;
  a.sf         = c->sf;
  a.sh         = c->d_sh;
  a.scale_lut  = c->d_lut;
  a.magic_ls   = (uint32_t)((0x100000000ull + q->ls - 1) / q->ls);
  if (crc) {
    a.xpow = xpow_for(q, crc);
    if (!a.xpow) {
      return SRSRAN_ERROR;
    }
    a.crc_poly  = (uint32_t)crc->polynom;
    a.crc_order = crc->order;
  }
  return ldpc_launch(q->bg == BG1 ? 0 : 1, a, stream) == hipSuccess ? SRSRAN_SUCCESS : SRSRAN_ERROR;
}

int decode_impl(srsran_ldpc_decoder_t* q, const void* llrs, int bits, uint8_t* message, uint32_t len,
                const srsran_crc_t* crc)
{
  Ctx* c = static_cast<Ctx*>(q->ptr);
  if (!c || !llrs || !message) {
    return SRSRAN_ERROR;
  }
  const size_t n = ((size_t)q->liftN - 2u * q->ls) * (size_t)(bits / 8);
  if (bits != c->bits || hipMemcpyAsync(c->d_in, llrs, n, hipMemcpyHostToDevice, c->stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  if (launch(q, c->d_in, bits, (uint32_t)n, 1, len, crc, c->d_out, q->liftK, 0, c->d_ret, c->stream) !=
      SRSRAN_SUCCESS) {
    return SRSRAN_ERROR;
  }
  uint8_t ret = 0;
  if (hipMemcpyAsync(message, c->d_out, q->liftK, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipMemcpyAsync(&ret, c->d_ret, 1, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  return (int)ret;
}

int decode_c_impl(void* o, const int8_t* llrs, uint8_t* message, uint32_t len, srsran_crc_t* crc)
{
  return decode_impl(static_cast<srsran_ldpc_decoder_t*>(o), llrs, 8, message, len, crc);
}

int decode_s_impl(void* o, const int16_t* llrs, uint8_t* message, uint32_t len, srsran_crc_t* crc)
{
  return decode_impl(static_cast<srsran_ldpc_decoder_t*>(o), llrs, 16, message, len, crc);
}

}  // namespace

namespace srsran_amd {

int ldpc_layers_for(const srsran_ldpc_decoder_t* q, uint32_t len) { return layers_for(q, len); }

std::vector<uint32_t> ldpc_xpow_table(uint32_t poly, int order, int nmax) { return xpow_table(poly, order, nmax); }

int ldpc_launch_cws(srsran_ldpc_decoder_t* q, const LdpcCw* d_cws, uint32_t n, const uint32_t* const xpow3[3],
                    uint32_t max_layers, hipStream_t stream)
{
  Ctx* c = static_cast<Ctx*>(q ? q->ptr : nullptr);
  if (!c || c->bits != 8) {
    return SRSRAN_ERROR;
  }
  LdpcArgs a;
  memset(&a, 0, sizeof(a));
  a.llr_bits   = 8;
  a.ncw        = n;
  a.ls         = q->ls;
  a.cw_per_wg  = ldpc_cw_per_wg(q->ls, 8);
  a.n_layers   = (int)std::min<uint32_t>(max_layers ? max_layers : q->bgM, q->bgM);
  a.max_iter   = (int)q->max_nof_iter;
  a.scale_mode = c->scale_mode;
  a.sf         = c->sf;
  a.sh         = c->d_sh;
  a.scale_lut  = c->d_lut;
  a.magic_ls   = (uint32_t)((0x100000000ull + q->ls - 1) / q->ls);
  a.cws        = d_cws;
  for (int i = 0; i < 3; i++) {
    a.xpow3[i] = xpow3[i];
  }
  return ldpc_launch(q->bg == BG1 ? 0 : 1, a, stream) == hipSuccess ? SRSRAN_SUCCESS : SRSRAN_ERROR;
}

}  // namespace srsran_amd

extern "C" {

int create_compact_pcm(uint16_t* pcm, int8_t (*positions)[MAX_CNCT], srsran_basegraph_t bg, uint16_t ls)
{
  Graph g;
  if (!pcm || !graph(bg, ls, g)) {
    fprintf(stderr, "[srsran_4g_amd] Invalid lifting size %d\n", ls);
    return SRSRAN_ERROR;
  }
  for (int i = 0; i < g.M * g.N; i++) {
    pcm[i] = NO_CNCT;
  }
  for (int i = 0; i < g.M; i++) {
    for (int e = g.rs[i]; e < g.rs[i + 1]; e++) {
      pcm[i * g.N + g.col[e]] = (uint16_t)(g.V[e] % ls);
    }
    if (positions) {
      for (int k = 0; k < MAX_CNCT; k++) {
        const int e     = g.rs[i] + k;
        positions[i][k] = e < g.rs[i + 1] ? (int8_t)g.col[e] : (int8_t)-1;
      }
    }
  }
  return SRSRAN_SUCCESS;
}

int srsran_ldpc_decoder_init(srsran_ldpc_decoder_t* q, const srsran_ldpc_decoder_args_t* args)
{
  if (!q || !args) {
    return SRSRAN_ERROR;
  }
  memset(q, 0, sizeof(*q));
  Graph g;
  if (!graph(args->bg, args->ls, g)) {
    fprintf(stderr, "[srsran_4g_amd] LDPC: invalid base graph %d / lifting size %d\n", (int)args->bg + 1, args->ls);
    return SRSRAN_ERROR;
  }
  const float s = args->scaling_fctr;
  if (!(s > 0.0f) || s > 1.0f) {  // ldpc_decoder.c:596-601
    fprintf(stderr, "[srsran_4g_amd] LDPC: scaling factor must be in (0, 1]\n");
    return SRSRAN_ERROR;
  }
  int scale_mode;
  int bits = 8;
  switch (args->type) {
    case SRSRAN_LDPC_DECODER_S:  // ldpc_dec_s.c: 16-bit LLRs, 15-bit messages, scaling m*s100/100
      scale_mode = LDPC_SCALE_C;
      bits       = 16;
      break;
    case SRSRAN_LDPC_DECODER_C:
      scale_mode = LDPC_SCALE_C;
      break;
    case SRSRAN_LDPC_DECODER_C_AVX2:
    case SRSRAN_LDPC_DECODER_C_AVX512:
      scale_mode = LDPC_SCALE_SIMD;
      break;
    default:
      fprintf(stderr, "[srsran_4g_amd] LDPC decoder type %d not provided on the GPU (layered C/AVX2/AVX512/S only)\n",
              (int)args->type);
      return SRSRAN_ERROR;
  }
  q->bg           = args->bg;
  q->ls           = args->ls;
  q->bgN          = (uint8_t)g.N;
  q->bgM          = (uint8_t)g.M;
  q->bgK          = (uint8_t)g.K;
  q->liftK        = (uint16_t)(g.K * args->ls);
  q->liftM        = (uint16_t)(g.M * args->ls);
  q->liftN        = (uint16_t)(g.N * args->ls);
  q->max_nof_iter = args->max_nof_iter == 0 ? 10 : args->max_nof_iter;
  q->scaling_fctr = s;
  q->pcm          = static_cast<uint16_t*>(malloc(sizeof(uint16_t) * g.M * g.N));
  q->var_indices  = static_cast<int8_t(*)[MAX_CNCT]>(malloc((size_t)g.M * MAX_CNCT));
  if (!q->pcm || !q->var_indices || create_compact_pcm(q->pcm, q->var_indices, q->bg, q->ls) != SRSRAN_SUCCESS) {
    free(q->pcm);
    free(q->var_indices);
    memset(q, 0, sizeof(*q));
    return SRSRAN_ERROR;
  }
  Ctx* c        = new Ctx;
  c->scale_mode = scale_mode;
  c->bits       = bits;
  // ldpc_dec_c_avx2.c:148 / ldpc_dec_c.c:149 (float arithmetic as the reference)
  c->sf = scale_mode == LDPC_SCALE_SIMD ? (int)(uint16_t)((s + 0.00001525879) * 65535) : (int)(s * 100);
  std::vector<uint32_t> sh(g.ne);
  for (int e = 0; e < g.ne; e++) {
    sh[e] = (uint32_t)(g.V[e] % args->ls);
  }
  uint8_t lut[128];
  for (int m = 0; m < 128; m++) {  // ldpc_dec_c.c:282 / _mm256_scalei_epi8 (ldpc_dec_c_avx2.c:520-531)
    lut[m] = (uint8_t)(scale_mode == LDPC_SCALE_SIMD ? ((uint32_t)m * (uint32_t)c->sf) >> 16 : m * c->sf / 100);
  }
  const size_t n = ((size_t)q->liftN - 2u * q->ls) * (size_t)(bits / 8);
  if (hipMalloc(&c->d_lut, 128) != hipSuccess || hipMemcpy(c->d_lut, lut, 128, hipMemcpyHostToDevice) != hipSuccess ||
      hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->d_sh, sh.size() * 4) != hipSuccess || hipMalloc(&c->d_in, n) != hipSuccess ||
      hipMalloc(&c->d_out, q->liftK) != hipSuccess || hipMalloc(&c->d_ret, 64) != hipSuccess ||
      hipMemcpy(c->d_sh, sh.data(), sh.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
    fprintf(stderr, "[srsran_4g_amd] LDPC: no HIP device / allocation failed\n");
    (void)hipGetLastError();
    free_ctx(c);
    free(q->pcm);
    free(q->var_indices);
    memset(q, 0, sizeof(*q));
    return SRSRAN_ERROR;
  }
  q->ptr  = c;
  q->free = free_dec;
  if (bits == 16) {
    q->decode_s = decode_s_impl;
  } else {
    q->decode_c = decode_c_impl;
  }
  return SRSRAN_SUCCESS;
}

void srsran_ldpc_decoder_free(srsran_ldpc_decoder_t* q)
{
  if (!q) {
    return;
  }
  if (q->free) {
    q->free(q);
  }
  memset(q, 0, sizeof(*q));
}

int srsran_ldpc_decoder_decode_f(srsran_ldpc_decoder_t* q, const float* llrs, uint8_t* message, uint32_t len)
{
  (void)q, (void)llrs, (void)message, (void)len;
  fprintf(stderr, "[srsran_4g_amd] LDPC: float decoder not provided on the GPU\n");
  return SRSRAN_ERROR;
}

int srsran_ldpc_decoder_decode_s(srsran_ldpc_decoder_t* q, const int16_t* llrs, uint8_t* message, uint32_t len)
{
  if (!q || !q->decode_s) {  // the reference calls a NULL decode_s for 8-bit decoder types
    fprintf(stderr, "[srsran_4g_amd] LDPC: decode_s needs a SRSRAN_LDPC_DECODER_S decoder\n");
    return SRSRAN_ERROR;
  }
  return q->decode_s(q, llrs, message, len, nullptr);
}

int srsran_ldpc_decoder_decode_c(srsran_ldpc_decoder_t* q, const int8_t* llrs, uint8_t* message, uint32_t len)
{
  if (!q || !q->decode_c) {
    return SRSRAN_ERROR;
  }
  return q->decode_c(q, llrs, message, len, nullptr);
}

int srsran_ldpc_decoder_decode_crc_c(srsran_ldpc_decoder_t* q,
                                     const int8_t*          llrs,
                                     uint8_t*               message,
                                     uint32_t               len,
                                     srsran_crc_t*          crc)
{
  if (!q || !q->decode_c) {
    return SRSRAN_ERROR;
  }
  return q->decode_c(q, llrs, message, len, crc);
}

int srsran_ldpc_decoder_gpu_decode_batch(srsran_ldpc_decoder_t* q,
                                         const int8_t*          d_llrs,
                                         uint32_t               llr_stride,
                                         uint32_t               nof_cw,
                                         uint32_t               cdwd_rm_length,
                                         const srsran_crc_t*    crc,
                                         uint8_t*               d_message,
                                         uint32_t               message_stride,
                                         int                    packed,
                                         uint8_t*               d_ret,
                                         void*                  stream)
{
  if (!q || !q->ptr) {
    return SRSRAN_ERROR;
  }
  return launch(q, d_llrs, 8, llr_stride, nof_cw, cdwd_rm_length, crc, d_message, message_stride, packed, d_ret,
                static_cast<hipStream_t>(stream));
}

int srsran_ldpc_decoder_gpu_decode_batch_s(srsran_ldpc_decoder_t* q,
                                           const int16_t*         d_llrs,
                                           uint32_t               llr_stride,
                                           uint32_t               nof_cw,
                                           uint32_t               cdwd_rm_length,
                                           const srsran_crc_t*    crc,
                                           uint8_t*               d_message,
                                           uint32_t               message_stride,
                                           int                    packed,
                                           uint8_t*               d_ret,
                                           void*                  stream)
{
  if (!q || !q->ptr) {
    return SRSRAN_ERROR;
  }
  return launch(q, d_llrs, 16, llr_stride * 2u, nof_cw, cdwd_rm_length, crc, d_message, message_stride, packed,
                d_ret, static_cast<hipStream_t>(stream));
}

}  // extern "C"
