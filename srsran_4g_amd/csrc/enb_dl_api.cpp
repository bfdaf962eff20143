// srsran_4g_amd/csrc/enb_dl_api.cpp -- eNB downlink transmit on the GPU (include/srsran_enb_dl.h):
// DL-SCH encoding (srsran_dlsch_gpu_encode_batch), CRS, scrambling + modulation + precoding + RE mapping
// (llr_kernel.hip: pdsch_tx_kernel, crs_put_kernel), the control channels (ctrl_tx_kernel: PSS / SSS,
// PBCH, PCFICH, PDCCH) and the OFDM modulator (ofdm_kernel.hip: ofdm_tx_kernel).  enb_dl.c:300-470,
// pdsch.c:1015-1120, pdcch.c:528-660, pcfich.c:185-235, pbch.c, pss.c / sss.c / gen_sss.c.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/srsran_enb_dl.h"
#include "llr_kernel.h"
#include "pdsch_internal.h"

using namespace srsran_amd;

namespace {

struct EnbDlGpu {
  srsran_sch_t  sch{};
  srsran_ofdm_t ofdm{};
  uint32_t      N = 0, sf_len = 0;
  float2*       d_grid = nullptr;  // [sf][port][2 nsymb][nre]
  size_t        grid_cap = 0;
  uint8_t*      d_e = nullptr;     // packed e bits of every codeword
  size_t        e_cap = 0;
  uint32_t*     d_idx = nullptr;   // RE tables of every subframe
  size_t        idx_cap = 0;
  uint32_t      last_sf = 0;    // subframes in d_grid (srsran_enb_dl_gpu_sf_symbols)
  PdschTx*      d_items = nullptr;
  size_t        items_cap = 0;
  uint32_t*     d_sfidx = nullptr;
  size_t        sfidx_cap = 0;
  // RE tables on the device, keyed by (PRB allocation, symbols a slot, first symbol, subframe): built
  // once, not re-uploaded every batch
  std::unordered_map<std::string, std::pair<uint32_t*, uint32_t>> tabs;
  // control channels: REG tables of the cell, the PBCH REs, the PSS / SSS sequences (built at init)
  srsran_regs_t regs{};
  bool          regs_ok = false;
  uint32_t*     d_ctab  = nullptr;  // [16 PCFICH][PBCH][PDCCH CFI 1][CFI 2][CFI 3]
  uint32_t      pbch_off = 16, pbch_nsym = 0, pdcch_off[3] = {0, 0, 0};
  float2*       d_sync  = nullptr;  // [PSS 72][SSS subframe 0: 72][SSS subframe 5: 72] (5 zero guards each side)
  CtrlTxJob*    d_jobs  = nullptr;
  size_t        jobs_cap = 0;
};

constexpr size_t kTabCache = 512;  // RE tables kept on the device

// Called once before a batch looks up its tables: when the batch could push the cache past its bound,
// the cache is emptied here (after the device is idle), never in the middle of the batch, so every
// table a batch has looked up stays allocated until its launches have run.
void tab_evict(EnbDlGpu* g, uint32_t nof_sf)
{
  if (g->tabs.size() + nof_sf > kTabCache) {
    hipDeviceSynchronize();
    for (auto& kv : g->tabs) {
      hipFree(kv.second.first);
    }
    g->tabs.clear();
  }
}

// (device table, RE count) of a grant, built and cached on first use; {nullptr, 0} on failure
std::pair<uint32_t*, uint32_t> get_tab(EnbDlGpu* g, const srsran_cell_t& cell, const srsran_pdsch_grant_t& gr,
                                       uint32_t lstart, uint32_t sf_idx)
{
  std::string key;
  key.reserve(2 * cell.nof_prb + 8);
  for (uint32_t s = 0; s < 2; s++) {
    for (uint32_t n = 0; n < cell.nof_prb; n++) {
      key.push_back(gr.prb_idx[s][n] ? '1' : '0');
    }
    key.push_back((char)gr.nof_symb_slot[s]);
  }
  key.push_back((char)lstart);
  key.push_back((char)sf_idx);
  auto it = g->tabs.find(key);
  if (it != g->tabs.end()) {
    return it->second;
  }
  const std::vector<uint32_t> t = pdsch_re_table(cell, gr, lstart, sf_idx);
  uint32_t*                   d = nullptr;
  if (hipMalloc((void**)&d, std::max<size_t>(t.size(), 1) * sizeof(uint32_t)) != hipSuccess ||
      hipMemcpy(d, t.data(), t.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
    hipFree(d);
    return {nullptr, 0};
  }
  return g->tabs[key] = std::make_pair(d, (uint32_t)t.size());
}

bool grow(void** p, size_t* cap, size_t need)
{
  if (need <= *cap) {
    return true;
  }
  hipFree(*p);
  *p   = nullptr;
  *cap = 0;
  if (hipMalloc(p, need) != hipSuccess) {
    return false;
  }
  *cap = need;
  return true;
}


// ---- control-channel tables ----
// PSS of N_id_2 (pss.c:341-370: the reference's float / double mix kept), SSS of subframes 0 and 5
// (36.211 6.11.2, gen_sss.c), each as 72 REs: 5 zero guards, 62 symbols, 5 zero guards (pss.c:372-379,
// sss.c:105-119)
void sync_sequences(uint32_t cell_id, std::vector<float2>& out)
{
  out.assign(3 * 72, make_float2(0.f, 0.f));
  static const float root[3] = {25.0f, 29.0f, 34.0f};
  const float        r       = root[cell_id % 3];
  for (int i = 0; i < 62; i++) {
    const double f   = i < 31 ? (double)(float)i * ((float)i + 1.0) : ((float)i + 2.0) * ((float)i + 1.0);
    const float  arg = (float)((double)(float)-1 * M_PI * (double)r * f / 63.0);
    out[5 + i]       = make_float2(cosf(arg), sinf(arg));
  }
  // m-sequences x(i + 5) = f(x) with x(0..4) = 0, 0, 0, 0, 1; tilde sequences 1 - 2 x
  auto mseq = [](int taps, int* t) {
    int x[31] = {0, 0, 0, 0, 1};
    for (int i = 0; i < 26; i++) {
      int v = 0;
      for (int b = 0; b < 5; b++) {
        if (taps & (1 << b)) {
          v ^= x[i + b];
        }
      }
      x[i + 5] = v;
    }
    for (int i = 0; i < 31; i++) {
      t[i] = 1 - 2 * x[i];
    }
  };
  int s_t[31], c_t[31], z_t[31];
  mseq(0x05, s_t);  // x(i+2) + x(i)
  mseq(0x09, c_t);  // x(i+3) + x(i)
  mseq(0x17, z_t);  // x(i+4) + x(i+2) + x(i+1) + x(i)
  const int N1 = (int)cell_id / 3, N2 = (int)cell_id % 3;
  const int qp = N1 / 30, q = (N1 + qp * (qp + 1) / 2) / 30, mp = N1 + q * (q + 1) / 2;
  const int m0 = mp % 31, m1 = (m0 + mp / 31 + 1) % 31;
  for (int n = 0; n < 31; n++) {
    const int s0 = s_t[(n + m0) % 31], s1 = s_t[(n + m1) % 31];
    const int c0 = c_t[(n + N2) % 31], c1 = c_t[(n + N2 + 3) % 31];
    const int z0 = z_t[(n + m0 % 8) % 31], z1 = z_t[(n + m1 % 8) % 31];
    out[72 + 5 + 2 * n]      = make_float2((float)(s0 * c0), 0.f);
    out[72 + 5 + 2 * n + 1]  = make_float2((float)(s1 * c1 * z0), 0.f);
    out[144 + 5 + 2 * n]     = make_float2((float)(s1 * c0), 0.f);
    out[144 + 5 + 2 * n + 1] = make_float2((float)(s0 * c1 * z1), 0.f);
  }
}

// PBCH REs (pbch.c srsran_pbch_cp with put): slot 1, symbols 0..3, the 72 central subcarriers; symbols 0, 1
// (and 3 with the extended CP) skip the CRS positions k mod 3 = cell_id mod 3 of any port count
std::vector<uint32_t> pbch_res(const srsran_cell_t& cell)
{
  const uint32_t nre = 12 * cell.nof_prb, nsymb = SRSRAN_CP_NSYMB(cell.cp), k0 = nre / 2 - 36, v = cell.id % 3;
  std::vector<uint32_t> t;
  for (uint32_t l = 0; l < 4; l++) {
    const bool crs = l < 2 || (l == 3 && cell.cp != SRSRAN_CP_NORM);
    for (uint32_t r = 0; r < 72; r++) {
      if (!crs || (k0 + r) % 3 != v) {
        t.push_back((nsymb + l) * nre + k0 + r);
      }
    }
  }
  return t;
}

bool ctrl_init(EnbDlGpu* g, const srsran_cell_t& cell)
{
  if (srsran_regs_init_opts(&g->regs, cell, 1, false) != SRSRAN_SUCCESS) {
    return false;
  }
  g->regs_ok = true;
  std::vector<uint32_t> tab(g->regs.pcfich_re, g->regs.pcfich_re + 16);
  const std::vector<uint32_t> pb = pbch_res(cell);
  g->pbch_off                    = (uint32_t)tab.size();
  g->pbch_nsym                   = (uint32_t)pb.size();
  tab.insert(tab.end(), pb.begin(), pb.end());
  for (int c = 0; c < 3; c++) {
    g->pdcch_off[c] = (uint32_t)tab.size();
    tab.insert(tab.end(), g->regs.pdcch_re[c], g->regs.pdcch_re[c] + 4 * (size_t)g->regs.pdcch_nregs[c]);
  }
  std::vector<float2> sync;
  sync_sequences(cell.id, sync);
  return hipMalloc((void**)&g->d_ctab, tab.size() * sizeof(uint32_t)) == hipSuccess &&
         hipMemcpy(g->d_ctab, tab.data(), tab.size() * sizeof(uint32_t), hipMemcpyHostToDevice) == hipSuccess &&
         hipMalloc((void**)&g->d_sync, sync.size() * sizeof(float2)) == hipSuccess &&
         hipMemcpy(g->d_sync, sync.data(), sync.size() * sizeof(float2), hipMemcpyHostToDevice) == hipSuccess;
}

// the jobs of one subframe's control channels (enb_dl.c:333-428), appended to `jobs`
int ctrl_jobs(EnbDlGpu* g, const srsran_cell_t& cell, const srsran_enb_dl_gpu_sf_t& s, float2* const* grid,
              std::vector<CtrlTxJob>& jobs)
{
  const srsran_enb_dl_gpu_ctrl_t* c = s.ctrl;
  const uint32_t sf = s.tti % 10, nre = 12 * cell.nof_prb, nsymb = SRSRAN_CP_NSYMB(cell.cp);
  const uint32_t P = cell.nof_ports, cfi = s.cfi;
  auto           base = [&](uint32_t kind) {
    CtrlTxJob j;
    memset(&j, 0, sizeof(j));
    for (uint32_t p = 0; p < P; p++) {
      j.grid[p] = grid[p];
    }
    j.kind   = kind;
    j.nports = P;
    return j;
  };
  if (c->put_base) {
    if (sf == 0 || sf == 5) {  // put_sync: PSS in the last, SSS in the second last symbol of slot 0
      CtrlTxJob j = base(2);
      j.seq       = g->d_sync;
      j.re0       = (nsymb - 1) * nre + nre / 2 - 36;
      j.nsym      = 72;
      jobs.push_back(j);
      j.seq = g->d_sync + (sf == 0 ? 72 : 144);
      j.re0 = (nsymb - 2) * nre + nre / 2 - 36;
      jobs.push_back(j);
    }
    if (sf == 0) {  // put_mib: the MIB of SFN tti / 10, the (sfn mod 4)-th quarter of its rate-matched bits
      CtrlTxJob j = base(0);
      uint8_t   mib[24];
      srsran_cell_t cl = cell;
      srsran_pbch_mib_pack(&cl, s.tti / 10, mib);
      memcpy(j.payload, mib, 24);
      j.nof_bits = 24;
      j.crc_mask = P == 2 ? 0xffffu : P == 4 ? 0x5555u : 0u;  // 36.212 Table 5.3.1.1-1
      j.nsym     = g->pbch_nsym;
      j.E        = 4 * 2 * g->pbch_nsym;
      j.bit0     = ((s.tti / 10) % 4) * 2 * g->pbch_nsym;
      j.seed     = cell.id;  // srsran_sequence_pbch
      j.seq_off  = j.bit0;
      j.re       = g->d_ctab + g->pbch_off;
      jobs.push_back(j);
    }
    CtrlTxJob j = base(1);  // put_pcfich
    j.nof_bits  = cfi;
    j.nsym      = 16;
    j.seed      = (sf + 1) * (2 * cell.id + 1) * 512 + cell.id;  // srsran_sequence_pcfich
    j.re        = g->d_ctab;
    jobs.push_back(j);
  }
  const uint32_t ncce = g->regs.pdcch_nregs[cfi - 1] / 9;
  for (uint32_t d = 0; d < c->nof_dci; d++) {
    const srsran_dci_msg_t& m = c->dci[d];
    const uint32_t          L = m.location.L, n0 = m.location.ncce, ncc = 1u << L;
    if (L > 3 || n0 + ncc > ncce || m.nof_bits >= SRSRAN_DCI_MAX_BITS - 16) {
      fprintf(stderr, "[srsran_enb_dl] illegal DCI message nCCE %u, L %u, nof_cce %u, nof_bits %u\n", n0, L, ncce,
              m.nof_bits);
      return SRSRAN_ERROR;
    }
    CtrlTxJob j = base(0);
    memcpy(j.payload, m.payload, m.nof_bits);
    j.nof_bits = m.nof_bits;
    j.crc_mask = m.rnti;
    j.nsym     = 36 * ncc;
    j.E        = 72 * ncc;
    j.seed     = sf * 512 + cell.id;  // srsran_sequence_pdcch
    j.seq_off  = 72 * n0;
    j.re       = g->d_ctab + g->pdcch_off[cfi - 1] + 36 * n0;
    for (uint32_t e = d + 1; e < c->nof_dci; e++) {  // CCEs a later message rewrites
      const uint32_t a = c->dci[e].location.ncce, b = a + (1u << c->dci[e].location.L);
      for (uint32_t k = 0; k < ncc; k++) {
        if (n0 + k >= a && n0 + k < b) {
          j.skip |= 1u << k;
        }
      }
    }
    jobs.push_back(j);
  }
  return SRSRAN_SUCCESS;
}

}  // namespace

extern "C" {

int srsran_enb_dl_gpu_init(srsran_enb_dl_gpu_t* q, srsran_cell_t cell)
{
  if (!q || cell.nof_prb < 6 || cell.nof_prb > SRSRAN_MAX_PRB || cell.nof_ports == 0 || cell.nof_ports == 3 ||
      cell.nof_ports > 4 ||
      (cell.cp != SRSRAN_CP_NORM && cell.cp != SRSRAN_CP_EXT)) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  memset(q, 0, sizeof(*q));
  q->cell       = cell;
  EnbDlGpu* g   = new EnbDlGpu();
  q->gpu        = g;
  srsran_ofdm_cfg_t oc;
  memset(&oc, 0, sizeof(oc));
  oc.nof_prb   = cell.nof_prb;
  oc.cp        = cell.cp;
  oc.normalize = false;  // enb_dl.c:158
  if (srsran_sch_init(&g->sch) != SRSRAN_SUCCESS || srsran_ofdm_tx_init_cfg(&g->ofdm, &oc) != SRSRAN_SUCCESS) {
    srsran_enb_dl_gpu_free(q);
    return SRSRAN_ERROR;
  }
  g->N      = g->ofdm.cfg.symbol_sz;
  g->sf_len = g->ofdm.sf_sz;
  if (!ctrl_init(g, cell)) {
    srsran_enb_dl_gpu_free(q);
    return SRSRAN_ERROR;
  }
  return SRSRAN_SUCCESS;
}

void srsran_enb_dl_gpu_free(srsran_enb_dl_gpu_t* q)
{
  if (!q) {
    return;
  }
  EnbDlGpu* g = (EnbDlGpu*)q->gpu;
  if (g) {
    hipDeviceSynchronize();
    srsran_sch_free(&g->sch);
    srsran_ofdm_tx_free(&g->ofdm);
    hipFree(g->d_grid);
    hipFree(g->d_e);
    hipFree(g->d_idx);
    hipFree(g->d_items);
    hipFree(g->d_sfidx);
    hipFree(g->d_ctab);
    hipFree(g->d_sync);
    hipFree(g->d_jobs);
    if (g->regs_ok) {
      srsran_regs_free(&g->regs);
    }
    for (auto& kv : g->tabs) {
      hipFree(kv.second.first);
    }
    delete g;
  }
  memset(q, 0, sizeof(*q));
}

int srsran_enb_dl_gpu_tx_batch(srsran_enb_dl_gpu_t*          q,
                               uint32_t                      nof_sf,
                               const srsran_enb_dl_gpu_sf_t* sfs,
                               cf_t*                         d_samples,
                               float                         scale,
                               void*                         stream)
{
  if (!q || !q->gpu || (nof_sf && (!sfs || !d_samples))) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  if (nof_sf == 0) {
    return SRSRAN_SUCCESS;
  }
  EnbDlGpu*           g     = (EnbDlGpu*)q->gpu;
  hipStream_t         st    = (hipStream_t)stream;
  const srsran_cell_t& cell = q->cell;
  const uint32_t      P     = cell.nof_ports, nre_sf = SRSRAN_SF_LEN_RE(cell.nof_prb, cell.cp);
  std::vector<std::pair<uint32_t*, uint32_t>> tables(nof_sf);
  std::vector<PdschTx>               items(nof_sf);
  std::vector<srsran_dlsch_gpu_enc_t> enc;
  std::vector<size_t>                 e_off;
  std::vector<uint32_t>               sfidx(nof_sf);
  size_t                              e_tot = 0;
  uint32_t                            max_nre = 0;
  tab_evict(g, nof_sf);
  // the subframes with a PDSCH: items[0..npd) (pdsch_tx_kernel's grid.y), sfidx per subframe (CRS)
  uint32_t npd = 0;
  std::vector<uint32_t> pd_sf;
  for (uint32_t b = 0; b < nof_sf; b++) {
    const srsran_enb_dl_gpu_sf_t& s   = sfs[b];
    const srsran_pdsch_cfg_t*     cfg = s.cfg;
    if (s.cfi < 1 || s.cfi > 3) {
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
    sfidx[b] = s.tti % 10;
    if (!cfg) {
      continue;
    }
    const srsran_pdsch_grant_t& gr = cfg->grant;
    int                         scheme;
    if (gr.tx_scheme == SRSRAN_TXSCHEME_PORT0 && P == 1 && gr.nof_tb == 1) {
      scheme = 0;
    } else if (gr.tx_scheme == SRSRAN_TXSCHEME_DIVERSITY && P == 2 && gr.nof_tb == 1) {
      scheme = 1;
    } else if (gr.tx_scheme == SRSRAN_TXSCHEME_DIVERSITY && P == 4 && gr.nof_tb == 1) {
      scheme = 4;
    } else if (gr.tx_scheme == SRSRAN_TXSCHEME_CDD && P == 2 && gr.nof_tb == 2 && gr.nof_layers == 2) {
      scheme = 3;
    } else {
      fprintf(stderr, "[srsran_enb_dl] transmission scheme %d with %u ports / %u TBs is not provided\n",
              (int)gr.tx_scheme, P, gr.nof_tb);
      return SRSRAN_ERROR;
    }
    const uint32_t lstart = s.cfi + (cell.nof_prb < 10 ? 1 : 0);  // SRSRAN_NOF_CTRL_SYMBOLS
    tables[npd]           = get_tab(g, cell, gr, lstart, sfidx[b]);
    if (!tables[npd].first) {
      return SRSRAN_ERROR;
    }
    const uint32_t nre = tables[npd].second;
    max_nre            = std::max(max_nre, nre);
    PdschTx& it        = items[npd];
    memset(&it, 0, sizeof(it));
    it.nre       = nre;
    it.scheme    = scheme;
    it.scaling   = s.pdsch_scaling > 0.0f ? s.pdsch_scaling : 1.0f;
    // scaling * M_SQRT1_2 (2 ports); scaling /= M_SQRT2 (4 ports, precoding.c:1962)
    it.div_scale = scheme == 4 ? (float)(it.scaling / 1.41421356237309504880)
                               : (float)((double)it.scaling * 0.70710678118654752440);
    uint32_t cw = 0;
    for (uint32_t t = 0; t < SRSRAN_MAX_CODEWORDS; t++) {
      const srsran_ra_tb_t& tb = gr.tb[t];
      if (!tb.enabled) {
        continue;
      }
      const uint32_t Qm = srsran_mod_bits_x_symbol(tb.mod), Nl = gr.nof_layers != gr.nof_tb ? 2 : 1;
      if (!s.d_data[t] || Qm == 0 || tb.nof_bits != nre * Qm || tb.tbs <= 0 || cw >= 2) {
        fprintf(stderr, "[srsran_enb_dl] TB %u: nof_bits %u does not match %u REs x Qm %u\n", t, tb.nof_bits, nre, Qm);
        return SRSRAN_ERROR_INVALID_INPUTS;
      }
      e_off.push_back(e_tot);
      enc.push_back({(uint32_t)tb.tbs, Qm * Nl, (uint32_t)tb.rv, tb.nof_bits, s.d_data[t], nullptr});
      it.seed[cw] = pdsch_seed(cfg->rnti, (int)tb.cw_idx, 2 * sfidx[b], cell.id);
      it.mod[cw]  = (int)tb.mod;
      e_tot += ((tb.nof_bits + 7) / 8 + 15) & ~(size_t)15;
      cw++;
    }
    if ((scheme == 3) != (cw == 2)) {
      return SRSRAN_ERROR_INVALID_INPUTS;
    }
    pd_sf.push_back(b);
    npd++;
  }
  const size_t grid_bytes = (size_t)nof_sf * P * nre_sf * sizeof(float2);
  if (!grow((void**)&g->d_grid, &g->grid_cap, grid_bytes) || !grow((void**)&g->d_e, &g->e_cap, e_tot + 16) ||
      !grow((void**)&g->d_items, &g->items_cap, nof_sf * sizeof(PdschTx)) ||
      !grow((void**)&g->d_sfidx, &g->sfidx_cap, nof_sf * sizeof(uint32_t))) {
    return SRSRAN_ERROR;
  }
  // device pointers of the codewords, tables and grids
  size_t k = 0;
  for (uint32_t i = 0; i < npd; i++) {
    PdschTx&       it = items[i];
    const uint32_t b  = pd_sf[i];
    it.idx            = tables[i].first;
    for (uint32_t p = 0; p < P; p++) {
      it.grid[p] = g->d_grid + ((size_t)b * P + p) * nre_sf;
    }
    const uint32_t ncw = it.scheme == 3 ? 2 : 1;
    for (uint32_t c = 0; c < ncw; c++, k++) {
      enc[k].d_e_bits = g->d_e + e_off[k];
      it.e[c]         = g->d_e + e_off[k];
    }
  }
  // control channels of every subframe: one launch
  std::vector<CtrlTxJob> jobs;
  for (uint32_t b = 0; b < nof_sf; b++) {
    if (!sfs[b].ctrl) {
      continue;
    }
    float2* grid[4] = {nullptr, nullptr, nullptr, nullptr};
    for (uint32_t p = 0; p < P; p++) {
      grid[p] = g->d_grid + ((size_t)b * P + p) * nre_sf;
    }
    if ((sfs[b].ctrl->nof_dci && !sfs[b].ctrl->dci) || ctrl_jobs(g, cell, sfs[b], grid, jobs) != SRSRAN_SUCCESS) {
      return SRSRAN_ERROR;
    }
  }
  if (!grow((void**)&g->d_jobs, &g->jobs_cap, std::max<size_t>(jobs.size(), 1) * sizeof(CtrlTxJob))) {
    return SRSRAN_ERROR;
  }
  if ((!enc.empty() && srsran_dlsch_gpu_encode_batch(&g->sch, (uint32_t)enc.size(), enc.data(), st) != SRSRAN_SUCCESS) ||
      hipMemsetAsync(g->d_grid, 0, grid_bytes, st) != hipSuccess ||
      (npd && hipMemcpyAsync(g->d_items, items.data(), npd * sizeof(PdschTx), hipMemcpyHostToDevice, st) != hipSuccess) ||
      hipMemcpyAsync(g->d_sfidx, sfidx.data(), nof_sf * sizeof(uint32_t), hipMemcpyHostToDevice, st) != hipSuccess ||
      (!jobs.empty() &&
       hipMemcpyAsync(g->d_jobs, jobs.data(), jobs.size() * sizeof(CtrlTxJob), hipMemcpyHostToDevice, st) != hipSuccess) ||
      crs_put_launch(g->d_grid, cell.nof_prb, cell.id, P, SRSRAN_CP_NSYMB(cell.cp), g->d_sfidx, nof_sf, st) != hipSuccess ||
      ctrl_tx_launch(g->d_jobs, (uint32_t)jobs.size(), st) != hipSuccess ||
      pdsch_tx_launch(g->d_items, npd, max_nre, st) != hipSuccess) {
    return SRSRAN_ERROR;
  }
  g->last_sf = nof_sf;
  const float sc = scale > 0.0f ? scale : 0.05f / sqrtf((float)cell.nof_prb);  // enb_dl_get_norm_factor
  return srsran_ofdm_tx_gpu(&g->ofdm, (const cf_t*)g->d_grid, d_samples, P, nof_sf, sc, st);
}

// ---------------- enb_dl.h: the reference's per-subframe object over the batched transmitter ----------------
}  // extern "C"

namespace {
struct EnbDlRef {
  srsran_enb_dl_gpu_t           tx{};
  bool                          tx_ok = false;
  hipStream_t                   stream = nullptr;
  // the subframe being recorded (srsran_enb_dl_put_* until srsran_enb_dl_gen_signal)
  bool                          base = false, pdsch = false;
  std::vector<srsran_dci_msg_t> dci;
  srsran_pdsch_cfg_t            cfg{};
  uint8_t*                      d_data[SRSRAN_MAX_CODEWORDS] = {nullptr, nullptr};
  size_t                        data_cap = 0;
  cf_t*                         d_samples = nullptr;
  size_t                        samples_cap = 0;
  uint32_t                      max_prb = 0;
};

void enb_ref_release(EnbDlRef* g)
{
  if (g->tx_ok) {
    srsran_enb_dl_gpu_free(&g->tx);
    g->tx_ok = false;
  }
}
}  // namespace

extern "C" {

int srsran_enb_dl_init(srsran_enb_dl_t* q, cf_t* out_buffer[SRSRAN_MAX_PORTS], uint32_t max_prb)
{
  if (!q || !out_buffer || max_prb < 6 || max_prb > SRSRAN_MAX_PRB) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  memset(q, 0, sizeof(*q));
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    fprintf(stderr, "[srsran_enb_dl] no HIP device\n");
    return SRSRAN_ERROR;
  }
  EnbDlRef* g = new EnbDlRef();
  g->max_prb  = max_prb;
  q->gpu      = g;
  const size_t nre = SRSRAN_SF_LEN_RE(max_prb, SRSRAN_CP_NORM);
  for (int p = 0; p < SRSRAN_MAX_PORTS; p++) {
    q->out_buffer[p] = out_buffer[p];
    q->sf_symbols[p] = (cf_t*)calloc(nre, sizeof(cf_t));
    if (!q->sf_symbols[p]) {
      srsran_enb_dl_free(q);
      return SRSRAN_ERROR;
    }
  }
  if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess) {
    srsran_enb_dl_free(q);
    return SRSRAN_ERROR;
  }
  return SRSRAN_SUCCESS;
}

void srsran_enb_dl_free(srsran_enb_dl_t* q)
{
  if (!q) {
    return;
  }
  EnbDlRef* g = (EnbDlRef*)q->gpu;
  if (g) {
    if (g->stream) {
      hipStreamSynchronize(g->stream);
      hipStreamDestroy(g->stream);
    }
    enb_ref_release(g);
    for (auto& d : g->d_data) {
      hipFree(d);
    }
    hipFree(g->d_samples);
    delete g;
  }
  if (q->cell.nof_prb) {
    srsran_regs_free(&q->regs);
  }
  for (int p = 0; p < SRSRAN_MAX_PORTS; p++) {
    free(q->sf_symbols[p]);
  }
  memset(q, 0, sizeof(*q));
}

int srsran_enb_dl_set_cell(srsran_enb_dl_t* q, srsran_cell_t cell)
{
  if (!q || !q->gpu || cell.nof_prb < 6 || cell.nof_prb > ((EnbDlRef*)q->gpu)->max_prb) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  EnbDlRef* g = (EnbDlRef*)q->gpu;
  if (q->cell.nof_prb) {
    srsran_regs_free(&q->regs);
  }
  enb_ref_release(g);
  if (srsran_enb_dl_gpu_init(&g->tx, cell) != SRSRAN_SUCCESS) {
    memset(&q->cell, 0, sizeof(q->cell));
    return SRSRAN_ERROR;
  }
  g->tx_ok = true;
  q->cell  = cell;
  if (srsran_regs_init(&q->regs, cell) != SRSRAN_SUCCESS) {
    return SRSRAN_ERROR;
  }
  // the PDCCH object's host fields (srsran_pdcch_set_cell's, pdcch.c:143-185): its locations are all a caller reads
  memset(&q->pdcch, 0, sizeof(q->pdcch));
  q->pdcch.cell = cell;
  q->pdcch.regs = &q->regs;
  for (int c = 0; c < 3; c++) {
    q->pdcch.nof_regs[c] = (q->regs.pdcch_nregs[c] / 9) * 9;
    q->pdcch.nof_cce[c]  = q->pdcch.nof_regs[c] / 9;
  }
  q->pdcch.max_bits = q->pdcch.nof_regs[2] * 8;
  for (uint32_t cfi = 1; cfi <= 3; cfi++) {  // enb_dl.c:226-230
    q->nof_common_locations[cfi - 1] =
        srsran_pdcch_common_locations(&q->pdcch, q->common_locations[cfi - 1], SRSRAN_MAX_CANDIDATES_COM, cfi);
  }
  return SRSRAN_SUCCESS;
}

bool srsran_enb_dl_location_is_common_ncce(srsran_enb_dl_t* q, const srsran_dci_location_t* loc)
{
  if (!q || !loc || q->dl_sf.cfi < 1 || q->dl_sf.cfi > 3) {
    return false;
  }
  return srsran_location_find_location(q->common_locations[q->dl_sf.cfi - 1], q->nof_common_locations[q->dl_sf.cfi - 1],
                                       loc);
}

void srsran_enb_dl_put_base(srsran_enb_dl_t* q, srsran_dl_sf_cfg_t* dl_sf)
{
  if (!q || !q->gpu || !dl_sf) {
    return;
  }
  EnbDlRef* g = (EnbDlRef*)q->gpu;
  q->dl_sf    = *dl_sf;
  g->base     = true;  // clear_sf + sync + CRS + MIB + PCFICH (enb_dl.c:372-382), generated with the subframe
  g->pdsch    = false;
  g->dci.clear();
}

static int put_dci(srsran_enb_dl_t* q, const srsran_dci_msg_t& m)
{
  EnbDlRef* g = (EnbDlRef*)q->gpu;
  if (q->dl_sf.cfi < 1 || q->dl_sf.cfi > 3 || m.location.L > 3 ||
      m.location.ncce + (1u << m.location.L) > q->pdcch.nof_cce[q->dl_sf.cfi - 1]) {
    fprintf(stderr, "[srsran_enb_dl] DCI location L=%u ncce=%u outside the control region of CFI %u\n",
            m.location.L, m.location.ncce, q->dl_sf.cfi);
    return SRSRAN_ERROR;  // srsran_pdcch_encode refuses it too (pdcch.c:626-631)
  }
  g->dci.push_back(m);
  return SRSRAN_SUCCESS;
}

int srsran_enb_dl_put_pdcch_dl(srsran_enb_dl_t* q, srsran_dci_cfg_t* dci_cfg, srsran_dci_dl_t* dci_dl)
{
  if (!q || !q->gpu || !dci_dl) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  srsran_dci_msg_t m;
  memset(&m, 0, sizeof(m));
  if (srsran_dci_msg_pack_pdsch(&q->cell, &q->dl_sf, dci_cfg, dci_dl, &m)) {
    fprintf(stderr, "[srsran_enb_dl] Error packing DL DCI\n");  // enb_dl.c:397-399: reported, then encoded
  }
  return put_dci(q, m);
}

int srsran_enb_dl_put_pdcch_ul(srsran_enb_dl_t* q, srsran_dci_cfg_t* dci_cfg, srsran_dci_ul_t* dci_ul)
{
  if (!q || !q->gpu || !dci_ul) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  srsran_dci_msg_t m;
  memset(&m, 0, sizeof(m));
  if (srsran_dci_msg_pack_pusch(&q->cell, &q->dl_sf, dci_cfg, dci_ul, &m)) {
    fprintf(stderr, "[srsran_enb_dl] Error packing UL DCI\n");
  }
  return put_dci(q, m);
}

int srsran_enb_dl_put_pdsch(srsran_enb_dl_t* q, srsran_pdsch_cfg_t* pdsch, uint8_t* data[SRSRAN_MAX_CODEWORDS])
{
  if (!q || !q->gpu || !pdsch || !data) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  EnbDlRef* g = (EnbDlRef*)q->gpu;
  size_t    need = 0;
  for (uint32_t t = 0; t < SRSRAN_MAX_CODEWORDS; t++) {
    if (pdsch->grant.tb[t].enabled) {
      if (!data[t] || pdsch->grant.tb[t].tbs <= 0) {
        return SRSRAN_ERROR_INVALID_INPUTS;
      }
      need = std::max(need, (size_t)pdsch->grant.tb[t].tbs / 8);
    }
  }
  if (need > g->data_cap) {
    hipStreamSynchronize(g->stream);
    for (auto& d : g->d_data) {
      hipFree(d);
      d = nullptr;
    }
    g->data_cap = 0;
    for (auto& d : g->d_data) {
      if (hipMalloc((void**)&d, need + 64) != hipSuccess) {
        return SRSRAN_ERROR;
      }
    }
    g->data_cap = need;
  }
  hipStreamSynchronize(g->stream);  // the previous subframe's encoder is done with the payload buffers
  for (uint32_t t = 0; t < SRSRAN_MAX_CODEWORDS; t++) {
    if (pdsch->grant.tb[t].enabled &&
        hipMemcpy(g->d_data[t], data[t], (size_t)pdsch->grant.tb[t].tbs / 8, hipMemcpyHostToDevice) != hipSuccess) {
      return SRSRAN_ERROR;
    }
  }
  g->cfg   = *pdsch;
  g->pdsch = true;
  return SRSRAN_SUCCESS;
}

void srsran_enb_dl_gen_signal(srsran_enb_dl_t* q)
{
  if (!q || !q->gpu || !q->cell.nof_prb) {
    return;
  }
  EnbDlRef*      g  = (EnbDlRef*)q->gpu;
  const uint32_t P  = q->cell.nof_ports;
  const uint32_t N  = ((EnbDlGpu*)g->tx.gpu)->N, sf_len = ((EnbDlGpu*)g->tx.gpu)->sf_len;
  const size_t   nre = SRSRAN_SF_LEN_RE(q->cell.nof_prb, q->cell.cp);
  (void)N;
  if (q->dl_sf.sf_type == SRSRAN_SF_MBSFN) {
    fprintf(stderr, "[srsran_enb_dl] MBSFN subframes are not generated (SURVEY section 8f)\n");
    return;
  }
  if (!g->base) {
    fprintf(stderr, "[srsran_enb_dl] srsran_enb_dl_put_base was not called for this subframe\n");
  }
  const size_t bytes = (size_t)P * sf_len * sizeof(cf_t);
  if (bytes > g->samples_cap) {
    hipFree(g->d_samples);
    g->d_samples   = nullptr;
    g->samples_cap = 0;
    if (hipMalloc((void**)&g->d_samples, bytes) != hipSuccess) {
      fprintf(stderr, "[srsran_enb_dl] device allocation failed\n");
      return;
    }
    g->samples_cap = bytes;
  }
  srsran_enb_dl_gpu_ctrl_t ctrl;
  memset(&ctrl, 0, sizeof(ctrl));
  ctrl.put_base = g->base ? 1u : 0u;
  ctrl.nof_dci  = (uint32_t)g->dci.size();
  ctrl.dci      = g->dci.empty() ? nullptr : g->dci.data();
  srsran_enb_dl_gpu_sf_t sf;
  memset(&sf, 0, sizeof(sf));
  sf.tti  = q->dl_sf.tti;
  sf.cfi  = q->dl_sf.cfi;
  sf.cfg  = g->pdsch ? &g->cfg : nullptr;
  sf.ctrl = &ctrl;
  for (uint32_t t = 0; t < SRSRAN_MAX_CODEWORDS && g->pdsch; t++) {
    sf.d_data[t] = g->cfg.grant.tb[t].enabled ? g->d_data[t] : nullptr;
  }
  if (g->pdsch) {  // srsran_pdsch_encode's rho_a (pdsch.c:492: 10^(p_a / 20), x sqrt 2 with more than one port)
    sf.pdsch_scaling = (float)((double)powf(10.0f, g->cfg.p_a / 20.0f) * (P == 1 ? 1.0 : M_SQRT2));
  }
  int ret = srsran_enb_dl_gpu_tx_batch(&g->tx, 1, &sf, g->d_samples, 0.0f, g->stream);
  for (uint32_t p = 0; p < P && ret == SRSRAN_SUCCESS; p++) {
    if ((q->out_buffer[p] && hipMemcpyAsync(q->out_buffer[p], g->d_samples + (size_t)p * sf_len, sf_len * sizeof(cf_t),
                                            hipMemcpyDeviceToHost, g->stream) != hipSuccess) ||
        hipMemcpyAsync(q->sf_symbols[p], srsran_enb_dl_gpu_sf_symbols(&g->tx) + (size_t)p * nre, nre * sizeof(cf_t),
                       hipMemcpyDeviceToHost, g->stream) != hipSuccess) {
      ret = SRSRAN_ERROR;
    }
  }
  if (ret != SRSRAN_SUCCESS || hipStreamSynchronize(g->stream) != hipSuccess) {
    fprintf(stderr, "[srsran_enb_dl] Error generating the subframe\n");
  }
  g->base  = false;
  g->pdsch = false;
  g->dci.clear();
}

float srsran_enb_dl_get_maximum_signal_power_dBfs(uint32_t nof_prb)
{
  // srsran_convert_amplitude_to_dB(0.05 / sqrt(N_RB)) + srsran_convert_power_to_dB(N_RB x 12) + 3 (enb_dl.c:691-695)
  return 20.0f * log10f(0.05f / sqrtf((float)nof_prb)) + 10.0f * log10f((float)nof_prb * SRSRAN_NRE) + 3.0f;
}

const cf_t* srsran_enb_dl_gpu_sf_symbols(srsran_enb_dl_gpu_t* q)
{
  return q && q->gpu && ((EnbDlGpu*)q->gpu)->last_sf ? (const cf_t*)((EnbDlGpu*)q->gpu)->d_grid : nullptr;
}

void srsran_pbch_mib_pack(srsran_cell_t* cell, uint32_t sfn, uint8_t* payload)
{
  // 36.331 MasterInformationBlock: dl-Bandwidth (3), phich-Duration (1), phich-Resource (2), SFN / 4 (8),
  // spare (10)
  const uint32_t bw  = cell->nof_prb <= 6 ? 0 : cell->nof_prb <= 15 ? 1 : 1 + cell->nof_prb / 25;
  uint32_t       res = 0;
  switch (cell->phich_resources) {
    case SRSRAN_PHICH_R_1_6:
      res = 0;
      break;
    case SRSRAN_PHICH_R_1_2:
      res = 1;
      break;
    case SRSRAN_PHICH_R_1:
      res = 2;
      break;
    case SRSRAN_PHICH_R_2:
      res = 3;
      break;
  }
  const uint32_t v = (bw << 21) | ((cell->phich_length == SRSRAN_PHICH_EXT ? 1u : 0u) << 20) | (res << 18) |
                     (((sfn >> 2) & 0xffu) << 10);
  for (int i = 0; i < 24; i++) {
    payload[i] = (uint8_t)((v >> (23 - i)) & 1u);
  }
}

}  // extern "C"
