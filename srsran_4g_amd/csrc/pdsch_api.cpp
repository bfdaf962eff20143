// srsran_4g_amd/csrc/pdsch_api.cpp -- srsran_pdsch_t on the GPU (include/srsran_ue_dl.h).
//
// srsran_pdsch_decode (pdsch.c:788-958) as three device passes per batch of subframes:
//   1. predecode_batch  srsran_pdsch_get (pdsch.c:246-254) fused as a gather through the RE
//                       table, apply_power_allocation's rho_b (pdsch.c:485-521) fused as a scale
//                       of CRS-symbol REs, srsran_predecoding_type MMSE + CSI (precoding.c:1866)
//   2. llr_batch        srsran_pdsch_codeword_decode's demod_soft_demodulate_s, sequence_pdsch_
//                       apply_s and csi_correction (pdsch.c:683-737) for every codeword
//   3. DL-SCH batch     srsran_dlsch_decode2 (sch.c:580-609) of every TB (sch_api.cpp)
// The host-synchronous srsran_pdsch_decode uploads the caller's grids / estimates, runs 1-2 and
// decodes each codeword with srsran_dlsch_decode2 semantics on the device LLRs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/srsran_pdcch.h"
#include "llr_kernel.h"
#include "pdsch_internal.h"
#include "stage_copy.h"
#include "stage_timing.h"

using namespace srsran_amd;

namespace {

constexpr uint32_t kMaxQm = 8;

struct Table {
  uint32_t* d      = nullptr;  // len RE entries, then npairs CSI pairs (PredArgs::pairs)
  uint32_t  len    = 0;
  uint32_t  npairs = 0;
};

using TableKey = std::array<uint64_t, 5>;  // RE table cache key (get_table)
static_assert(SRSRAN_MAX_PRB <= 128, "two 64-bit words of PRB bitmap per slot");

// Descriptor staging of one batch (pinned host + device copy).  A ring of kStageRing of them lets the host build
// batch N + 1 .. N + kStageRing - 1 while the GPU still reads batch N's descriptors: the host waits only for the
// batch kStageRing back, so a stall of the calling thread shorter than that many batches leaves the GPU busy.
constexpr int kStageRing = 3;
struct StageSlot {
  hipEvent_t staged = nullptr;  // SRSRAN_AMD_STAGE=side: this slot's last upload finished (pinned staging reusable)
  hipEvent_t read   = nullptr;  // SRSRAN_AMD_STAGE=side: the launches that read this slot's device copy are done
  uint32_t   seq    = 0;        // default staging: fence sequence number of the batch that last filled the slot
  bool       used   = false;
  char*      h      = nullptr;  // pinned coherent host memory (stage_host_alloc)
  char*      hd     = nullptr;  // its device alias
  char*      d      = nullptr;
  size_t     cap    = 0;
};

struct PdschGpu {
  hipStream_t                  stream  = nullptr;  // host-synchronous path
  hipStream_t                  copy    = nullptr;  // descriptor uploads, ahead of the launches that read them
  StageSlot                    ring[kStageRing];
  uint32_t                     ring_next = 0;
  srsran_amd::StageFence       fence;  // the copy kernel's "slot read" words (stage_copy.h)
  srsran_amd::StreamHandoff    ho;     // stream of the previous batch (device-side reuse of slots and d_work)
  char*                        d_work    = nullptr;
  size_t                       work_cap  = 0;
  float2*                      d_in      = nullptr;  // host-synchronous path: grids + estimates
  size_t                       in_cap    = 0;
  std::map<TableKey, Table>    tables;
  struct LlrRef {
    uint32_t       sf, tb, n;
    const int16_t* d;
  };
  std::vector<LlrRef> last_llr;  // the last batch's LLR buffers (srsran_pdsch_gpu_last_llr)
  struct EvmRef {
    uint32_t sf, tb;
    float*   d;
  };
  std::vector<EvmRef> last_evm;       // the last batch's EVM results (srsran_pdsch_gpu_last_evm)
  uint32_t            evm_max_bits = 0;  // srsran_evm_buffer_t.max_bits (pdsch.c:297, 468-471)
};

bool grow_dev(void** p, size_t* cap, size_t need)
{
  if (*cap >= need) {
    return true;
  }
  if (*p) {
    hipDeviceSynchronize();  // buffers may still be in use by enqueued work
    hipFree(*p);
  }
  *p   = nullptr;
  *cap = 0;
  need = std::max(need, (size_t)65536);
  if (hipMalloc(p, need) != hipSuccess) {
    return false;
  }
  *cap = need;
  return true;
}

bool grow_stage(PdschGpu* g, StageSlot& st, size_t need)
{
  if (st.cap >= need) {
    return true;
  }
  if (st.used) {  // the slot's last batch is done with both copies
    if (srsran_amd::stage_side_copy()) {
      hipEventSynchronize(st.read);
    } else {
      srsran_amd::handoff_drain(g->ho);
    }
  }
  hipHostFree(st.h);
  hipFree(st.d);
  st.h   = nullptr;
  st.d   = nullptr;
  st.cap = 0;
  need   = std::max(need, (size_t)65536);
  st.h = (char*)srsran_amd::stage_host_alloc(need, (void**)&st.hd);
  if (!st.h || hipMalloc((void**)&st.d, need) != hipSuccess) {
    return false;
  }
  st.cap = need;
  return true;
}

bool init_ring(PdschGpu* g)
{
  for (StageSlot& st : g->ring) {
    if (srsran_amd::ring_event_create(&st.staged) != hipSuccess ||
        srsran_amd::ring_event_create(&st.read) != hipSuccess || !grow_stage(g, st, 65536)) {
      return false;
    }
  }
  return srsran_amd::stage_fence_init(g->fence, kStageRing);
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

constexpr size_t kTableCache = 512;  // RE tables kept on the device

// Called once before a batch looks up its tables: when the batch could push the cache past its bound
// the cache is emptied here (device idle first), never while a batch holds table pointers.
void table_evict(PdschGpu* g, uint32_t nsf)
{
  if (g->tables.size() + nsf > kTableCache) {
    hipDeviceSynchronize();
    for (auto& kv : g->tables) {
      hipFree(kv.second.d);
    }
    g->tables.clear();
  }
}

// RE table of (grant, CFI, subframe) on the device, built once (pdsch_map.cpp); {nullptr, 0} on failure
Table get_table(srsran_pdsch_t* q, PdschGpu* g, const srsran_pdsch_grant_t& gr, uint32_t lstart,
                       uint32_t sf_idx)
{
  TableKey key{};  // PRB bitmaps of both slots, symbols per slot, first PDSCH symbol, subframe index
  for (uint32_t sl = 0; sl < 2; sl++) {
    for (uint32_t n = 0; n < q->cell.nof_prb; n++) {
      if (gr.prb_idx[sl][n]) {
        key[sl * 2 + n / 64] |= 1ull << (n % 64);
      }
    }
  }
  key[4] = (uint64_t)gr.nof_symb_slot[0] | (uint64_t)gr.nof_symb_slot[1] << 8 | (uint64_t)lstart << 16 |
           (uint64_t)sf_idx << 24;
  auto it = g->tables.find(key);
  if (it != g->tables.end()) {
    return it->second;
  }
  std::vector<uint32_t> t = pdsch_re_table(q->cell, gr, lstart, sf_idx);
  Table                 tb;
  tb.len = (uint32_t)t.size();
  // the distinct (subcarrier, RE parity) pairs: an AVERAGE estimate has one row of subcarriers, so the CSI maximum
  // of the fused path's pre-pass needs these 2 x 12 N_RB at most, not every RE
  const uint32_t       nre = 12 * q->cell.nof_prb;
  std::vector<uint8_t> seen(nre, 0);
  for (uint32_t k = 0; k < tb.len; k++) {
    seen[(t[k] & 0x7fffffffu) % nre] |= (uint8_t)(1u << (k & 1));
  }
  for (uint32_t sc = 0; sc < nre; sc++) {
    for (uint32_t par = 0; par < 2; par++) {
      if (seen[sc] >> par & 1) {
        t.push_back(sc | par << 31);
      }
    }
  }
  tb.npairs = (uint32_t)t.size() - tb.len;
  if (hipMalloc((void**)&tb.d, std::max<size_t>(t.size(), 1) * sizeof(uint32_t)) != hipSuccess ||
      hipMemcpy(tb.d, t.data(), t.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
    hipFree(tb.d);
    return Table{};
  }
  return g->tables[key] = tb;
}

// One decoded codeword of the batch
struct Cw {
  uint32_t sf, tb, cw, Qm, nbits;
  int      mod;
};

// Enqueue predecode + LLR of nsf subframes; fills `cws` and the per-codeword LLR pointers (and, for
// subframes with meas_evm_en, g->last_evm).
// Scratch layout (d_work): x [nsf][2][max_re] float2 | csi [nsf][2][max_re] f32 | csi_max [nsf][2] |
// llr [nsf][2][max_re * 8] int16 | EVM block sums [nsf][2][evm_parts] f32 | EVM results [nsf][2] f32
int enqueue_llr(srsran_pdsch_t* q, uint32_t nsf, const srsran_pdsch_gpu_sf_t* sfs, hipStream_t s,
                std::vector<Cw>& cws, std::vector<int16_t*>& llr)
{
  srsran_amd::HostScope desc(srsran_amd::HP_PDSCH_DESC);
  PdschGpu*      g   = (PdschGpu*)q->gpu;
  const uint32_t nrx = q->nof_rx_antennas, np = q->cell.nof_ports, nre = 12 * q->cell.nof_prb;
  const uint32_t nsf_rows = 2 * SRSRAN_CP_NSYMB(q->cell.cp);  // grid symbols per subframe (14 / 12)
  std::vector<Table>    tabs(nsf);
  std::vector<PredArgs> pa(nsf);
  uint32_t              max_re = 0;
  cws.clear();
  table_evict(g, nsf);
  for (uint32_t b = 0; b < nsf; b++) {
    const srsran_pdsch_gpu_sf_t& f = sfs[b];
    if (!f.cfg || !f.d_grid || !f.d_ce || f.cfi < 1 || f.cfi > 3) {
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
    const srsran_pdsch_grant_t& gr = f.cfg->grant;
    if (gr.nof_layers == 0 || gr.nof_layers > SRSRAN_MAX_LAYERS) {
      return SRSRAN_ERROR_OUT_OF_BOUNDS;
    }
    const bool txd = gr.tx_scheme == SRSRAN_TXSCHEME_DIVERSITY;
    // one codeword on two layers (SM / CDD, 36.211 Table 6.3.3.2-1): predecode both layers, then
    // srsran_layerdemap_type as the reference runs it (pdsch.c:838-863)
    const bool cw1l2 = !txd && gr.nof_tb == 1 && gr.nof_layers == 2 &&
                       (gr.tx_scheme == SRSRAN_TXSCHEME_SPATIALMUX || gr.tx_scheme == SRSRAN_TXSCHEME_CDD);
    if (txd ? (gr.nof_tb != 1 || gr.nof_layers != np)
            : (!cw1l2 && (gr.nof_layers != gr.nof_tb || gr.nof_tb < 1 || gr.nof_tb > 2))) {
      fprintf(stderr, "[srsran_pdsch] unsupported: %u codewords on %u layers\n", gr.nof_tb, gr.nof_layers);
      return SRSRAN_ERROR;
    }
    const uint32_t lstart = f.cfi + (q->cell.nof_prb < 10 ? 1 : 0);  // SRSRAN_NOF_CTRL_SYMBOLS
    tabs[b]               = get_table(q, g, gr, lstart, f.tti % 10);
    if (!tabs[b].d) {
      return SRSRAN_ERROR;
    }
    if (tabs[b].len != gr.nof_re) {
      fprintf(stderr, "[srsran_pdsch] Error expecting %u symbols but got %u\n", gr.nof_re, tabs[b].len);
      return SRSRAN_ERROR;
    }
    max_re = std::max(max_re, gr.nof_re);
    // power allocation (pdsch.c:485-521, 795-801)
    float scaling = 1.0f, rho_b_inv = 1.0f;
    if (f.cfg->power_scale) {
      const float rho_a = (float)(powf(10.0f, f.cfg->p_a / 20.0f) * (np == 1 ? 1.0 : M_SQRT2));
      if (rho_a != 0.0f && std::isnormal(rho_a)) {
        scaling = rho_a;
      }
      static const float kRatio[2][4] = {{1.0f, 4.0f / 5.0f, 3.0f / 5.0f, 2.0f / 5.0f},
                                         {5.0f / 4.0f, 1.0f, 3.0f / 4.0f, 1.0f / 2.0f}};
      if (f.cfg->p_b > 3) {
        return SRSRAN_ERROR_INVALID_INPUTS;
      }
      const float rho_b = sqrtf(kRatio[np == 1 ? 0 : 1][f.cfg->p_b]);
      if (rho_b != 0.0f && rho_b != 1.0f) {
        rho_b_inv = 1.0f / rho_b;
      }
    }
    PredArgs&      a        = pa[b];
    const uint32_t codebook = gr.nof_tb == 1 ? gr.pmi : gr.pmi + 1;
    if (!pred_setup(a, (int)nrx, (int)np, (int)gr.nof_layers, (int)codebook, (int)gr.tx_scheme, scaling)) {
      fprintf(stderr, "[srsran_pdsch] unsupported: scheme %d, %u ports, %u rx, %u layers\n", (int)gr.tx_scheme, np,
              nrx, gr.nof_layers);
      return SRSRAN_ERROR;
    }
    a.n          = gr.nof_re;
    a.interleave = txd ? 1 : cw1l2 ? 2 : 0;  // the layer demapping fused into the predecoder
    a.noise     = f.cfg->decoder_type == SRSRAN_MIMO_DECODER_ZF ? 0.0f : f.noise;
    a.noise_ptr = f.cfg->decoder_type == SRSRAN_MIMO_DECODER_ZF ? nullptr : f.d_noise;
    a.rho_b_inv = rho_b_inv;
    a.ce_row    = f.ce_full ? 0 : nre;
    const size_t ce_len = f.ce_full ? (size_t)nsf_rows * nre : nre;
    for (uint32_t r = 0; r < nrx; r++) {
      a.y[r] = (const float2*)f.d_grid + (size_t)r * nsf_rows * nre;
      for (uint32_t p = 0; p < np; p++) {
        a.h[p][r] = (const float2*)f.d_ce + (size_t)(p * nrx + r) * ce_len;
      }
    }
    for (uint32_t tb = 0; tb < SRSRAN_MAX_CODEWORDS; tb++) {
      const srsran_ra_tb_t& t = gr.tb[tb];
      if (!t.enabled) {
        continue;
      }
      const uint32_t Qm = srsran_mod_bits_x_symbol(t.mod);
      if (Qm == 0 || t.cw_idx >= gr.nof_tb || t.nof_bits != gr.nof_re * Qm) {
        fprintf(stderr, "[srsran_pdsch] unsupported codeword %u: Qm %u, %u bits for %u REs\n", tb, Qm, t.nof_bits,
                gr.nof_re);
        return SRSRAN_ERROR;
      }
      cws.push_back(Cw{b, tb, t.cw_idx, Qm * (gr.nof_layers != gr.nof_tb ? 2u : 1u), t.nof_bits, (int)t.mod});
    }
  }
  if (max_re == 0) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  // scratch
  const size_t x_sz = align256((size_t)nsf * 2 * max_re * sizeof(float2));
  const size_t c_sz = align256((size_t)nsf * 2 * max_re * sizeof(float));
  const size_t m_sz = align256((size_t)nsf * 2 * sizeof(float));
  const size_t e_sz = align256((size_t)nsf * 2 * max_re * kMaxQm * sizeof(int16_t));
  const uint32_t evm_parts = (2 * max_re + LLR_BLOCK_SYMBOLS - 1) / LLR_BLOCK_SYMBOLS;  // >= blocks of any item
  const size_t   v_sz      = align256((size_t)nsf * 2 * (evm_parts + 1) * sizeof(float));
  if (!grow_dev((void**)&g->d_work, &g->work_cap, x_sz + c_sz + m_sz + e_sz + v_sz)) {
    return SRSRAN_ERROR;
  }
  float* d_evm_part = (float*)(g->d_work + x_sz + c_sz + m_sz + e_sz);
  float* d_evm_out  = d_evm_part + (size_t)nsf * 2 * evm_parts;
  float2*  d_x   = (float2*)g->d_work;
  float*   d_csi = (float*)(g->d_work + x_sz);
  float*   d_max = (float*)(g->d_work + x_sz + c_sz);
  int16_t* d_e   = (int16_t*)(g->d_work + x_sz + c_sz + m_sz);
  for (uint32_t b = 0; b < nsf; b++) {
    PredArgs& a = pa[b];
    a.idx       = tabs[b].d;
    for (int l = 0; l < 2; l++) {
      a.x[l]   = d_x + ((size_t)b * 2 + l) * max_re;
      a.csi[l] = d_csi + ((size_t)b * 2 + l) * max_re;
    }
    a.csi_max = (uint32_t*)(d_max + 2 * b);
  }
  // LLR descriptors, grouped by modulation
  std::vector<LlrItem> li(cws.size());
  std::vector<EvmItem> evs;
  g->last_evm.clear();
  llr.assign(cws.size(), nullptr);
  for (size_t i = 0; i < cws.size(); i++) {
    const Cw&                    c = cws[i];
    const srsran_pdsch_gpu_sf_t& f = sfs[c.sf];
    LlrItem&                     it = li[i];
    it.sym      = (const float*)(d_x + ((size_t)c.sf * 2 + c.cw) * max_re);
    it.csi      = f.cfg->csi_enable ? d_csi + ((size_t)c.sf * 2 + c.cw) * max_re : nullptr;
    it.csi_max  = f.cfg->csi_enable ? d_max + 2 * c.sf + c.cw : nullptr;
    it.llr      = d_e + ((size_t)c.sf * 2 + c.tb) * max_re * kMaxQm;
    it.llr8     = q->llr_is_8bit ? (int8_t*)it.llr : nullptr;  // the 8-bit chain writes int8 into the same slot
    it.n        = f.cfg->grant.nof_re;
    it.seed     = pdsch_seed(f.cfg->rnti, (int)c.cw, 2 * (f.tti % 10), q->cell.id);
    it.bit0     = 0;
    it.scramble = 1;
    llr[i]      = it.llr;
    if (f.cfg->meas_evm_en) {  // srsran_evm_run_s over min(max_bits, nof_bits) bits (evm.h:190-194)
      const uint32_t nbits = std::min(g->evm_max_bits, c.nbits);
      const uint32_t qmod  = srsran_mod_bits_x_symbol((srsran_mod_t)c.mod);
      const size_t   slot  = (size_t)c.sf * 2 + c.tb;
      it.evm_n             = qmod ? nbits / qmod : 0;
      it.evm_part          = d_evm_part + slot * evm_parts;
      evs.push_back(EvmItem{it.evm_part, (it.evm_n + LLR_BLOCK_SYMBOLS - 1) / LLR_BLOCK_SYMBOLS, it.evm_n,
                            d_evm_out + slot});
      g->last_evm.push_back({c.sf, c.tb, d_evm_out + slot});
    }
  }
  // The fused predecode + LLR path (llr_kernel.h FusedItem, one item a subframe), opt-in (SRSRAN_AMD_PDSCH_FUSED=1,
  // read every call) for batches whose subframes are all PORT0, or SM / CDD with two codewords of one modulation on
  // two layers, with int16 LLRs and no EVM: the equalised symbols and CSI stay in registers, the CSI maxima come
  // from a pre-pass over the (subcarrier, parity) pairs.  Both kernels it replaces are issue-bound, not HBM-bound,
  // so the fused one takes their sum (C3, r05m: 7.4 + 33.8 us against 19.0 + 21.8 us) -- off by default.
  const char* fenv  = getenv("SRSRAN_AMD_PDSCH_FUSED");
  bool        fused = !q->llr_is_8bit && fenv && fenv[0] == '1';
  std::vector<int>      sf_mod(nsf, -1);
  std::vector<uint32_t> sf_cw(nsf * 2, 0);  // [sf][layer] -> index into cws
  std::vector<uint8_t>  sf_layers(nsf, 0);  // [sf] bit l: layer l's codeword recorded (once)
  for (size_t i = 0; i < cws.size() && fused; i++) {
    const Cw& c = cws[i];
    fused       = (sf_mod[c.sf] < 0 || sf_mod[c.sf] == c.mod) && c.cw < 2 && !(sf_layers[c.sf] >> c.cw & 1);
    if (fused) {
      sf_mod[c.sf]           = c.mod;
      sf_cw[c.sf * 2 + c.cw] = (uint32_t)i;
      sf_layers[c.sf] |= (uint8_t)(1u << c.cw);
    }
  }
  // every layer the fused kernel writes must have its own codeword (a disabled TB or two TBs on one codeword index
  // would leave a slot pointing at another codeword's buffer): bit 0 for PORT0, bits 0 and 1 for SM / CDD
  for (uint32_t b = 0; b < nsf && fused; b++) {
    const srsran_pdsch_grant_t& gr = sfs[b].cfg->grant;
    fused = sf_mod[b] >= 0 && !sfs[b].cfg->meas_evm_en && pa[b].interleave == 0 &&
            (pa[b].scheme == 0 ? gr.nof_tb == 1 && sf_layers[b] == 1u
                               : (pa[b].scheme == 2 || pa[b].scheme == 3) && gr.nof_tb == 2 && sf_layers[b] == 3u);
  }
  std::vector<uint32_t> order_p(nsf), order_l(fused ? nsf : cws.size()), pos_of(nsf);
  for (uint32_t i = 0; i < nsf; i++) {
    order_p[i] = i;
  }
  for (uint32_t i = 0; i < order_l.size(); i++) {
    order_l[i] = i;
  }
  std::stable_sort(order_p.begin(), order_p.end(), [&](uint32_t x, uint32_t y) { return pa[x].scheme < pa[y].scheme; });
  for (uint32_t i = 0; i < nsf; i++) {
    pos_of[order_p[i]] = i;
  }
  // LLR launches group by modulation (fused: subframes by modulation and predecoder scheme)
  auto lkey = [&](uint32_t x) { return fused ? sf_mod[x] * 8 + pa[x].scheme : cws[x].mod; };
  std::stable_sort(order_l.begin(), order_l.end(), [&](uint32_t x, uint32_t y) { return lkey(x) < lkey(y); });
  const size_t pa_bytes = align256(nsf * sizeof(PredArgs));
  const size_t li_bytes = align256(std::max<size_t>(order_l.size(), 1) * (fused ? sizeof(FusedItem) : sizeof(LlrItem)));
  const size_t ev_bytes = align256(evs.size() * sizeof(EvmItem));
  const size_t pp_bytes = fused ? pa_bytes : 0;  // the fused path's pre-pass descriptors (CSI pairs)
  desc.stop();
  srsran_amd::HostScope wait(srsran_amd::HP_PDSCH_WAIT);
  const bool side   = srsran_amd::stage_side_copy();
  const int  slot   = (int)g->ring_next;
  StageSlot& st     = g->ring[slot];
  g->ring_next = (g->ring_next + 1) % kStageRing;
  if (st.used && (side ? hipEventSynchronize(st.staged) != hipSuccess
                       : !srsran_amd::stage_fence_wait(g->fence, slot, st.seq))) {
    return SRSRAN_ERROR;
  }
  // every slot of the ring grows now, not when it comes round
  if (st.cap < pa_bytes + li_bytes + ev_bytes + pp_bytes) {
    for (StageSlot& r : g->ring) {
      if (!grow_stage(g, r, 2 * (pa_bytes + li_bytes + ev_bytes + pp_bytes))) {
        return SRSRAN_ERROR;
      }
    }
  }
  wait.stop();
  srsran_amd::HostScope launch(srsran_amd::HP_PDSCH_LAUNCH);
  PredArgs*  hp = (PredArgs*)st.h;
  LlrItem*   hl = (LlrItem*)(st.h + pa_bytes);
  FusedItem* hf = (FusedItem*)(st.h + pa_bytes);
  for (uint32_t i = 0; i < nsf; i++) {
    hp[i] = pa[order_p[i]];
  }
  for (uint32_t i = 0; i < order_l.size(); i++) {
    const uint32_t c = order_l[i];
    if (fused) {  // subframe c; its descriptor as uploaded: st.d + pos_of[c] PredArgs
      FusedItem& fi = hf[i];
      fi.pa         = (const PredArgs*)st.d + pos_of[c];
      fi.n          = pa[c].n;
      fi.csi_max    = sfs[c].cfg->csi_enable ? d_max + 2 * c : nullptr;
      for (uint32_t l = 0; l < 2; l++) {
        const LlrItem& it = li[sf_cw[c * 2 + (pa[c].scheme == 0 ? 0 : l)]];
        fi.llr[l]         = it.llr;
        fi.seed[l]        = it.seed;
      }
    } else {
      hl[i] = li[c];
    }
  }
  if (!evs.empty()) {
    memcpy(st.h + pa_bytes + li_bytes, evs.data(), evs.size() * sizeof(EvmItem));
  }
  PredArgs* hpp = (PredArgs*)(st.h + pa_bytes + li_bytes + ev_bytes);
  for (uint32_t i = 0; i < nsf && fused; i++) {
    hpp[i] = hp[i];
    if (hp[i].ce_row) {  // AVERAGE: the CSI pairs of the subframe's table
      const Table& tb = tabs[order_p[i]];
      hpp[i].idx      = tb.d + tb.len;
      hpp[i].n        = tb.npairs;
      hpp[i].pairs    = 1;
    }
  }
  // SRSRAN_AMD_STAGE=side (round 3): the upload on a copy stream once the launches of the batch that last used
  // this slot are done with its device copy, beside the OFDM / estimation stages
  if (side) {
    if (st.used) {
      hipStreamWaitEvent(g->copy, st.read, 0);
    }
    hipMemcpyAsync(st.d, st.h, pa_bytes + li_bytes + ev_bytes + pp_bytes, hipMemcpyHostToDevice, g->copy);
    hipEventRecord(st.staged, g->copy);
    hipStreamWaitEvent(s, st.staged, 0);
  } else {  // in line: a copy kernel reads the pinned slot and then marks it read in the fence (stage_copy.h)
    // ... and zeroes the batch's CSI maxima (no memset launch)
    if (srsran_amd::handoff(g->ho, s) != hipSuccess) {
      return SRSRAN_ERROR;
    }
    st.seq = ++g->fence.seq;
    if (srsran_amd::stage_copy_or_record(st.d, st.hd, pa_bytes + li_bytes + ev_bytes + pp_bytes, s, (uint32_t*)d_max,
                                         nsf * 2, &g->fence, slot, st.seq) != hipSuccess) {
      return SRSRAN_ERROR;
    }
  }
  st.used = true;
  // from here on the slot belongs to this batch: its read event is recorded on every exit, so the upload that
  // next reuses it waits for whatever of this one was enqueued, error paths included
  struct ReadMark {
    StageSlot&  st;
    hipStream_t s;
    bool        on;
    ~ReadMark()
    {
      if (on) {
        hipEventRecord(st.read, s);
      }
    }
  } mark{st, s, side};
  if (side) {
    hipMemsetAsync(d_max, 0, (size_t)nsf * 2 * sizeof(float), s);
  }
  const PredArgs* dp = (const PredArgs*)st.d;
  const LlrItem*  dl = (const LlrItem*)(st.d + pa_bytes);
  if (fused) {
    bool any_csi = false;
    for (uint32_t b = 0; b < nsf; b++) {
      any_csi = any_csi || sfs[b].cfg->csi_enable;
    }
    const PredArgs* dpp = (const PredArgs*)(st.d + pa_bytes + li_bytes + ev_bytes);
    for (uint32_t i = 0; i < nsf && any_csi;) {  // the CSI maxima: one pre-pass launch per predecoder scheme
      uint32_t j = i, mx = 0;
      while (j < nsf && hpp[j].scheme == hpp[i].scheme) {
        mx = std::max(mx, hpp[j].n);
        j++;
      }
      const PredArgs* items = dpp + i;
      const uint32_t  n = j - i, scheme = (uint32_t)hp[i].scheme;
      if (srsran_amd::launch_or_record([=] { return csi_max_batch_launch(items, n, (int)scheme, mx, s); }) !=
          hipSuccess) {
        return SRSRAN_ERROR;
      }
      i = j;
    }
    const FusedItem* df = (const FusedItem*)(st.d + pa_bytes);
    for (uint32_t i = 0; i < nsf;) {  // one launch per (modulation, scheme)
      uint32_t j = i, mx = 0;
      while (j < nsf && lkey(order_l[j]) == lkey(order_l[i])) {
        mx = std::max(mx, hf[j].n);
        j++;
      }
      const int        mod = sf_mod[order_l[i]], scheme = pa[order_l[i]].scheme;
      const FusedItem* items = df + i;
      const uint32_t   n     = j - i;
      if (srsran_amd::launch_or_record([=] { return fused_llr_batch_launch(mod, scheme, items, n, mx, s); }) !=
          hipSuccess) {
        return SRSRAN_ERROR;
      }
      i = j;
    }
    return SRSRAN_SUCCESS;
  }
  for (uint32_t i = 0; i < nsf;) {  // one launch per predecoder scheme
    uint32_t j = i, mx = 0;
    while (j < nsf && hp[j].scheme == hp[i].scheme) {
      mx = std::max(mx, hp[j].n);
      j++;
    }
    const PredArgs* items = dp + i;
    const uint32_t  n = j - i, scheme = (uint32_t)hp[i].scheme;
    if (srsran_amd::launch_or_record([=] { return predecode_batch_launch(items, n, (int)scheme, mx, s); }) !=
        hipSuccess) {
      return SRSRAN_ERROR;
    }
    i = j;
  }
  for (uint32_t i = 0; i < cws.size();) {  // one launch per modulation
    uint32_t j = i, mx = 0;
    while (j < cws.size() && cws[order_l[j]].mod == cws[order_l[i]].mod) {
      mx = std::max(mx, hl[j].n);
      j++;
    }
    const int      mod   = cws[order_l[i]].mod;
    const LlrItem* items = dl + i;
    const uint32_t n     = j - i;
    const bool     b8    = q->llr_is_8bit;
    if (srsran_amd::launch_or_record([=] { return llr_batch_launch(mod, items, n, mx, 1, s, b8); }) != hipSuccess) {
      return SRSRAN_ERROR;
    }
    i = j;
  }
  const EvmItem* d_ev  = (const EvmItem*)(st.d + pa_bytes + li_bytes);
  const uint32_t nev   = (uint32_t)evs.size();
  if (nev && srsran_amd::launch_or_record([=] { return evm_finalize_launch(d_ev, nev, s); }) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  return SRSRAN_SUCCESS;
}

}  // namespace

extern "C" {

int srsran_pdsch_init_ue(srsran_pdsch_t* q, uint32_t max_prb, uint32_t nof_rx_antennas)
{
  if (!q || max_prb == 0 || max_prb > SRSRAN_MAX_PRB || nof_rx_antennas == 0 || nof_rx_antennas > SRSRAN_MAX_PORTS) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  memset(q, 0, sizeof(*q));
  q->nof_rx_antennas = nof_rx_antennas;
  q->max_re          = max_prb * 2 * SRSRAN_CP_NORM_NSYMB * SRSRAN_NRE;
  q->is_ue           = true;
  if (gold_tables_init() != hipSuccess || srsran_sch_init(&q->dl_sch)) {
    fprintf(stderr, "[srsran_pdsch] no HIP device available\n");
    return SRSRAN_ERROR;
  }
  PdschGpu* g = new PdschGpu();
  q->gpu      = g;
  g->evm_max_bits = (uint32_t)std::max(0, srsran_ra_tbs_from_idx(SRSRAN_RA_NOF_TBS_IDX - 1, 6));  // pdsch.c:297
  if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&g->copy, hipStreamNonBlocking) != hipSuccess ||
      !init_ring(g)) {
    srsran_pdsch_free(q);
    return SRSRAN_ERROR;
  }
  return SRSRAN_SUCCESS;
}

void srsran_pdsch_free(srsran_pdsch_t* q)
{
  if (!q) {
    return;
  }
  PdschGpu* g = (PdschGpu*)q->gpu;
  if (g) {
    hipDeviceSynchronize();
    for (auto& kv : g->tables) {
      hipFree(kv.second.d);
    }
    hipFree(g->d_work);
    hipFree(g->d_in);
    for (StageSlot& st : g->ring) {
      hipFree(st.d);
      hipHostFree(st.h);
      if (st.staged) {
        hipEventDestroy(st.staged);
      }
      if (st.read) {
        hipEventDestroy(st.read);
      }
    }
    if (g->stream) {
      hipStreamDestroy(g->stream);
    }
    if (g->copy) {
      hipStreamDestroy(g->copy);
    }
    srsran_amd::stage_fence_free(g->fence);
    srsran_amd::handoff_free(g->ho);
    delete g;
  }
  srsran_sch_free(&q->dl_sch);
  memset(q, 0, sizeof(*q));
}

int srsran_pdsch_enable_coworker(srsran_pdsch_t* q) { return q ? SRSRAN_SUCCESS : SRSRAN_ERROR_INVALID_INPUTS; }

int srsran_pdsch_set_cell(srsran_pdsch_t* q, srsran_cell_t cell)
{
  if (!q || !q->gpu || cell.nof_prb == 0 || cell.nof_prb > SRSRAN_MAX_PRB || cell.nof_ports == 0 ||
      cell.nof_ports == 3 || cell.nof_ports > 4 || cell.id > 503) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (cell.frame_type != SRSRAN_FDD && cell.frame_type != SRSRAN_TDD) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (cell.cp != SRSRAN_CP_NORM && cell.cp != SRSRAN_CP_EXT) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  PdschGpu* g = (PdschGpu*)q->gpu;
  hipDeviceSynchronize();
  for (auto& kv : g->tables) {
    hipFree(kv.second.d);
  }
  g->tables.clear();
  // the EVM buffer grows to the new cell (srsran_evm_buffer_resize keeps the larger of the two, pdsch.c:468-471)
  g->evm_max_bits = std::max(g->evm_max_bits,
                             (uint32_t)std::max(0, srsran_ra_tbs_from_idx(SRSRAN_RA_NOF_TBS_IDX - 1, cell.nof_prb)));
  q->cell   = cell;
  q->max_re = SRSRAN_SF_LEN_RE(cell.nof_prb, cell.cp);
  return SRSRAN_SUCCESS;
}

int srsran_pdsch_decode(srsran_pdsch_t*        q,
                        srsran_dl_sf_cfg_t*    sf,
                        srsran_pdsch_cfg_t*    cfg,
                        srsran_chest_dl_res_t* channel,
                        cf_t*                  sf_symbols[SRSRAN_MAX_PORTS],
                        srsran_pdsch_res_t     data[SRSRAN_MAX_CODEWORDS])
{
  if (!q || !q->gpu || !sf || !cfg || !channel || !sf_symbols || !data) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (q->llr_is_8bit != q->dl_sch.llr_is_8bit) {  // srsUE sets both (cc_worker.cc:108-110)
    fprintf(stderr, "[srsran_pdsch] llr_is_8bit must match dl_sch.llr_is_8bit\n");
    return SRSRAN_ERROR;
  }
  PdschGpu*      g   = (PdschGpu*)q->gpu;
  const uint32_t nrx = q->nof_rx_antennas, np = q->cell.nof_ports, nsym = SRSRAN_SF_LEN_RE(q->cell.nof_prb, q->cell.cp);
  if (cfg->max_nof_iterations) {
    srsran_sch_set_max_noi(&q->dl_sch, cfg->max_nof_iterations);
  }
  if (!grow_dev((void**)&g->d_in, &g->in_cap, (size_t)(nrx + np * nrx) * nsym * sizeof(float2))) {
    return SRSRAN_ERROR;
  }
  for (uint32_t r = 0; r < nrx; r++) {
    if (!sf_symbols[r]) {
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
    hipMemcpyAsync(g->d_in + (size_t)r * nsym, sf_symbols[r], nsym * sizeof(cf_t), hipMemcpyHostToDevice, g->stream);
    for (uint32_t p = 0; p < np; p++) {
      hipMemcpyAsync(g->d_in + (size_t)(nrx + p * nrx + r) * nsym, channel->ce[p][r], nsym * sizeof(cf_t),
                     hipMemcpyHostToDevice, g->stream);
    }
  }
  srsran_pdsch_gpu_sf_t f;
  memset(&f, 0, sizeof(f));
  f.cfg     = cfg;
  f.tti     = sf->tti;
  f.cfi     = sf->cfi;
  f.d_grid  = (const cf_t*)g->d_in;
  f.d_ce    = (const cf_t*)(g->d_in + (size_t)nrx * nsym);
  f.ce_full = 1;
  f.noise   = channel->noise_estimate;
  std::vector<Cw>       cws;
  std::vector<int16_t*> llr;
  int                   ret = enqueue_llr(q, 1, &f, g->stream, cws, llr);
  if (ret) {
    hipStreamSynchronize(g->stream);
    return ret;
  }
  float evm[SRSRAN_MAX_CODEWORDS] = {NAN, NAN};
  for (const auto& e : g->last_evm) {
    if (e.tb < SRSRAN_MAX_CODEWORDS) {
      hipMemcpyAsync(&evm[e.tb], e.d, sizeof(float), hipMemcpyDeviceToHost, g->stream);
    }
  }
  if (hipStreamSynchronize(g->stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  for (size_t i = 0; i < cws.size(); i++) {
    const uint32_t tb = cws[i].tb;
    if (data[tb].crc) {
      continue;  // already acknowledged (pdsch.c:893)
    }
    data[tb].evm = cfg->meas_evm_en ? evm[tb] : NAN;  // pdsch.c:698-713
    if (!cfg->softbuffers.rx[tb] || !data[tb].payload) {
      data[tb].crc = false;
      continue;
    }
    const int r = srsran_dlsch_decode2_dev(&q->dl_sch, cfg, llr[i], data[tb].payload, (int)tb, cfg->grant.nof_layers);
    data[tb].crc                  = r == SRSRAN_SUCCESS;  // pdsch.c:739-747
    data[tb].avg_iterations_block = srsran_sch_last_noi(&q->dl_sch);
  }
  if (cfg->meas_evm_en) {  // pdsch.c:945-951
    for (uint32_t i = 0; i < SRSRAN_MAX_CODEWORDS; i++) {
      if (cfg->grant.tb[i].enabled && !std::isnan(data[i].evm)) {
        q->avg_evm = 0.1f * data[i].evm + (1.0f - 0.1f) * q->avg_evm;  // SRSRAN_VEC_EMA(data, avg, 0.1)
      }
    }
  }
  return SRSRAN_SUCCESS;
}

int srsran_pdsch_gpu_decode_batch(srsran_pdsch_t*              q,
                                  uint32_t                     nof_sf,
                                  const srsran_pdsch_gpu_sf_t* sfs,
                                  int32_t*                     d_result,
                                  float*                       d_avg_noi,
                                  void*                        stream)
{
  if (!q || !q->gpu || (nof_sf && (!sfs || !d_result || !d_avg_noi))) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (nof_sf == 0) {
    return 0;
  }
  if (q->llr_is_8bit != q->dl_sch.llr_is_8bit) {
    return SRSRAN_ERROR;
  }
  hipStream_t s = (hipStream_t)stream;
  std::vector<Cw>       cws;
  std::vector<int16_t*> llr;
  int                   ret = enqueue_llr(q, nof_sf, sfs, s, cws, llr);
  if (ret) {
    return ret;
  }
  PdschGpu* g = (PdschGpu*)q->gpu;
  g->last_llr.clear();
  for (size_t i = 0; i < cws.size(); i++) {
    g->last_llr.push_back({cws[i].sf, cws[i].tb, cws[i].nbits, llr[i]});
  }
  std::vector<srsran_dlsch_gpu_tb_t> tbs(cws.size());
  std::vector<uint32_t>              maxit(cws.size());  // each subframe's own limit (pdsch.c:723 per decode)
  for (size_t i = 0; i < cws.size(); i++) {
    const srsran_pdsch_gpu_sf_t& f = sfs[cws[i].sf];
    const srsran_ra_tb_t&        t = f.cfg->grant.tb[cws[i].tb];
    srsran_dlsch_gpu_tb_t&       e = tbs[i];
    if (!f.cfg->softbuffers.rx[cws[i].tb] || !f.d_payload[cws[i].tb]) {
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
    e.tbs        = (uint32_t)t.tbs;
    e.Qm         = cws[i].Qm;  // Qm * Nl as srsran_dlsch_decode2 passes it (sch.c:587-603)
    e.rv         = (uint32_t)t.rv;
    e.nof_e_bits = t.nof_bits;
    e.d_e_bits   = llr[i];
    e.d_data     = f.d_payload[cws[i].tb];
    e.softbuffer = f.cfg->softbuffers.rx[cws[i].tb];
    e.new_data   = f.new_data[cws[i].tb];
    maxit[i]     = f.cfg->max_nof_iterations;
  }
  ret = dlsch_gpu_decode_batch_limits(&q->dl_sch, (uint32_t)tbs.size(), tbs.data(), maxit.data(), d_result, d_avg_noi,
                                      stream);
  return ret == SRSRAN_SUCCESS ? (int)tbs.size() : ret;
}


int srsran_pdsch_gpu_last_evm(srsran_pdsch_t* q, uint32_t sf, uint32_t tb, const float** d_evm)
{
  if (!q || !q->gpu || !d_evm) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  for (const auto& r : ((PdschGpu*)q->gpu)->last_evm) {
    if (r.sf == sf && r.tb == tb) {
      *d_evm = r.d;
      return SRSRAN_SUCCESS;
    }
  }
  return SRSRAN_ERROR;
}

int srsran_pdsch_gpu_last_llr(srsran_pdsch_t* q, uint32_t sf, uint32_t tb, const int16_t** d_llr, uint32_t* nof_llr)
{
  if (!q || !q->gpu || !d_llr || !nof_llr) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  for (const auto& r : ((PdschGpu*)q->gpu)->last_llr) {
    if (r.sf == sf && r.tb == tb) {
      *d_llr   = r.d;
      *nof_llr = r.n;
      return SRSRAN_SUCCESS;
    }
  }
  return SRSRAN_ERROR;
}

// ---------------- transmitter (pdsch.c:1015-1120, eNB side) ----------------
int srsran_pdsch_init_enb(srsran_pdsch_t* q, uint32_t max_prb)
{
  const int r = srsran_pdsch_init_ue(q, max_prb, 1);
  if (r == SRSRAN_SUCCESS) {
    q->is_ue = false;
  }
  return r;
}

int srsran_pdsch_encode(srsran_pdsch_t*     q,
                        srsran_dl_sf_cfg_t* sf,
                        srsran_pdsch_cfg_t* cfg,
                        uint8_t*            data[SRSRAN_MAX_CODEWORDS],
                        cf_t*               sf_symbols[SRSRAN_MAX_PORTS])
{
  if (!q || !q->gpu || !sf || !cfg || !data || !sf_symbols) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  const srsran_cell_t&        cell = q->cell;
  const srsran_pdsch_grant_t& gr   = cfg->grant;
  const uint32_t              P    = cell.nof_ports;
  for (uint32_t p = 0; p < P; p++) {
    if (!sf_symbols[p]) {
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
  }
  if (gr.nof_tb == 0) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  int scheme;
  if (gr.tx_scheme == SRSRAN_TXSCHEME_PORT0 && P == 1 && gr.nof_tb == 1) {
    scheme = 0;
  } else if (gr.tx_scheme == SRSRAN_TXSCHEME_DIVERSITY && P == 2 && gr.nof_tb == 1) {
    scheme = 1;
  } else if (gr.tx_scheme == SRSRAN_TXSCHEME_DIVERSITY && P == 4 && gr.nof_tb == 1) {
    scheme = 4;
  } else if (gr.tx_scheme == SRSRAN_TXSCHEME_CDD && P == 2 && gr.nof_tb == 2 && gr.nof_layers == 2) {
    scheme = 3;
  } else {
    fprintf(stderr, "[srsran_pdsch] encode: scheme %d with %u ports / %u TBs is not provided\n", (int)gr.tx_scheme, P,
            gr.nof_tb);
    return SRSRAN_ERROR;
  }
  // apply_power_allocation (pdsch.c:485-521, called by srsran_pdsch_encode whatever power_scale says, :1057-1071):
  // the precoder scales by rho_a = 10^(p_a / 20) (x sqrt 2 with more than one port); the rho_b part scales
  // nof_rx_antennas grids, none for the eNB's object (pdsch.c srsran_pdsch_init_enb)
  const float rho_a   = (float)((double)powf(10.0f, cfg->p_a / 20.0f) * (P == 1 ? 1.0 : M_SQRT2));
  const float scaling = rho_a != 0.0f ? rho_a : 1.0f;
  PdschGpu*             g      = (PdschGpu*)q->gpu;
  const uint32_t        lstart = sf->cfi + (cell.nof_prb < 10 ? 1 : 0);
  std::vector<uint32_t> tab    = pdsch_re_table(cell, gr, lstart, sf->tti % 10);
  const uint32_t        nre = (uint32_t)tab.size(), nsf_re = SRSRAN_SF_LEN_RE(cell.nof_prb, cell.cp);
  if (nre != gr.nof_re || nre > q->max_re) {
    fprintf(stderr, "[srsran_pdsch] Error expecting %u symbols but got %u\n", gr.nof_re, nre);
    return SRSRAN_ERROR;
  }
  // device scratch: grids, RE table, payloads, packed e bits, descriptor
  PdschTx                             it;
  std::vector<srsran_dlsch_gpu_enc_t> enc;
  memset(&it, 0, sizeof(it));
  it.nre       = nre;
  it.scheme    = scheme;
  it.scaling   = scaling;
  it.div_scale = scheme == 4 ? (float)(scaling / 1.41421356237309504880) : (float)((double)scaling * 0.70710678118654752440);
  size_t   off = align256((size_t)P * nsf_re * sizeof(float2));
  size_t   o_idx = off;
  off += align256((size_t)nre * sizeof(uint32_t));
  size_t   o_item = off;
  off += align256(sizeof(PdschTx));
  std::vector<size_t> o_data, o_e;
  uint32_t            cw = 0;
  for (uint32_t t = 0; t < SRSRAN_MAX_CODEWORDS; t++) {
    const srsran_ra_tb_t& tb = gr.tb[t];
    if (!tb.enabled) {
      continue;
    }
    const uint32_t Qm = srsran_mod_bits_x_symbol(tb.mod), Nl = gr.nof_layers != gr.nof_tb ? 2 : 1;
    if (!data[t] || Qm == 0 || tb.tbs <= 0 || tb.nof_bits != nre * Qm || cw >= 2) {
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
    o_data.push_back(off);
    off += align256((size_t)tb.tbs / 8);
    o_e.push_back(off);
    off += align256((tb.nof_bits + 7) / 8);
    enc.push_back({(uint32_t)tb.tbs, Qm * Nl, (uint32_t)tb.rv, tb.nof_bits, nullptr, nullptr});
    it.seed[cw] = pdsch_seed(cfg->rnti, (int)tb.cw_idx, 2 * (sf->tti % 10), cell.id);
    it.mod[cw]  = (int)tb.mod;
    cw++;
  }
  if ((scheme == 3) != (cw == 2) || !grow_dev((void**)&g->d_work, &g->work_cap, off) ||
      srsran_amd::handoff(g->ho, g->stream) != hipSuccess) {  // d_work: after the batches queued elsewhere
    return SRSRAN_ERROR;
  }
  char* base = g->d_work;
  for (uint32_t p = 0; p < P; p++) {
    it.grid[p] = (float2*)base + (size_t)p * nsf_re;
  }
  it.idx = (const uint32_t*)(base + o_idx);
  cw     = 0;
  for (uint32_t t = 0; t < SRSRAN_MAX_CODEWORDS; t++) {
    if (!gr.tb[t].enabled) {
      continue;
    }
    enc[cw].d_data   = (const uint8_t*)(base + o_data[cw]);
    enc[cw].d_e_bits = (uint8_t*)(base + o_e[cw]);
    it.e[cw]         = (const uint8_t*)(base + o_e[cw]);
    if (hipMemcpyAsync(base + o_data[cw], data[t], (size_t)gr.tb[t].tbs / 8, hipMemcpyHostToDevice, g->stream) !=
        hipSuccess) {
      return SRSRAN_ERROR;
    }
    cw++;
  }
  // the ports' grids keep what the caller already put there (CRS, control): only PDSCH REs change
  for (uint32_t p = 0; p < P; p++) {
    if (hipMemcpyAsync(it.grid[p], sf_symbols[p], nsf_re * sizeof(float2), hipMemcpyHostToDevice, g->stream) !=
        hipSuccess) {
      return SRSRAN_ERROR;
    }
  }
  if (hipMemcpyAsync(base + o_idx, tab.data(), nre * sizeof(uint32_t), hipMemcpyHostToDevice, g->stream) !=
          hipSuccess ||
      hipMemcpyAsync(base + o_item, &it, sizeof(it), hipMemcpyHostToDevice, g->stream) != hipSuccess ||
      srsran_dlsch_gpu_encode_batch(&q->dl_sch, cw, enc.data(), g->stream) != SRSRAN_SUCCESS ||
      pdsch_tx_launch((const PdschTx*)(base + o_item), 1, nre, g->stream) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  for (uint32_t p = 0; p < P; p++) {
    if (hipMemcpyAsync(sf_symbols[p], it.grid[p], nsf_re * sizeof(float2), hipMemcpyDeviceToHost, g->stream) !=
        hipSuccess) {
      return SRSRAN_ERROR;
    }
  }
  return hipStreamSynchronize(g->stream) == hipSuccess ? SRSRAN_SUCCESS : SRSRAN_ERROR;
}

}  // extern "C"
