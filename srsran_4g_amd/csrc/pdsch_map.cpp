// srsran_4g_amd/csrc/pdsch_map.cpp -- PDSCH resource-element map (host side).
//
// srsran_pdsch_get / srsran_pdsch_cp (pdsch.c:136-220) walk the subframe grid and copy every
// PDSCH RE of a grant into a contiguous symbol array, skipping the control region, the CRS
// (prb_cp_ref, prb_dl.c:46-77) and the PSS/SSS/PBCH centre PRBs (pdsch_cp_skip_symbol,
// pdsch.c:83-112).  Here that walk runs once per (cell, grant, CFI, subframe) on the host and
// records, for every PDSCH RE in order, its grid index; the predecoder kernel gathers
// through the table, so the extracted symbol / estimate arrays never exist in HBM.
// Bit 31 of an entry marks REs of CRS-bearing symbols (the ones apply_power_allocation scales
// by 1/rho_b, pdsch.c:498-517).
#include <cstdint>
#include <vector>

#include "../../include/srsran_ue_dl.h"

namespace srsran_amd {

// SRSRAN_SYMBOL_HAS_REF (phy_common.h): l = 0 and l = nsymb - 3 of each slot (+ l = 1 with 4 ports)
static bool symbol_has_ref(uint32_t l, uint32_t nsymb, uint32_t nof_ports)
{
  return (l == 1 && nof_ports == 4) || l == 0 || l == nsymb - 3;
}

static bool skip_symbol(const srsran_cell_t& cell, const srsran_pdsch_grant_t& g, uint32_t sf_idx, uint32_t s,
                        uint32_t l, uint32_t n)
{
  if (n >= cell.nof_prb / 2 - 3 && n < cell.nof_prb / 2 + 3 + (cell.nof_prb % 2)) {
    if (cell.frame_type == SRSRAN_FDD) {
      if (s == 0 && (sf_idx == 0 || sf_idx == 5) && l >= g.nof_symb_slot[s] - 2) {
        return true;  // PSS / SSS
      }
    } else {
      if (s == 1 && (sf_idx == 0 || sf_idx == 5) && l >= g.nof_symb_slot[s] - 1) {
        return true;  // TDD SSS
      }
      if (s == 0 && (sf_idx == 1 || sf_idx == 6) && l == 2) {
        return true;  // TDD PSS
      }
    }
    if (s == 1 && sf_idx == 0 && l < 4) {
      return true;  // PBCH
    }
  }
  return false;
}

// prb_cp_ref in "get" direction: the input pointer skips the reference REs
static void cp_ref(uint32_t& in, std::vector<uint32_t>& out, uint32_t flag, int offset, int nof_refs,
                   int nof_intervals)
{
  const int ref_interval = (SRSRAN_NRE / nof_refs) - 1;
  for (int k = 0; k < offset; k++) {
    out.push_back((in++) | flag);
  }
  for (int i = 0; i < nof_intervals - 1; i++) {
    in++;
    for (int k = 0; k < ref_interval; k++) {
      out.push_back((in++) | flag);
    }
  }
  if (ref_interval - offset > 0) {
    in++;
    for (int k = 0; k < ref_interval - offset; k++) {
      out.push_back((in++) | flag);
    }
  }
}

std::vector<uint32_t> pdsch_re_table(const srsran_cell_t& cell, const srsran_pdsch_grant_t& g, uint32_t lstart_grant,
                                     uint32_t sf_idx)
{
  std::vector<uint32_t> out;
  const uint32_t        nof_refs = cell.nof_ports == 1 ? 2 : 4;
  for (uint32_t s = 0; s < 2; s++) {
    const uint32_t lstart = s == 0 ? lstart_grant : 0;
    for (uint32_t l = lstart; l < g.nof_symb_slot[s]; l++) {
      const bool     has_crs = symbol_has_ref(l, SRSRAN_CP_NSYMB(cell.cp), cell.nof_ports);
      const uint32_t flag    = has_crs ? 0x80000000u : 0u;
      const uint32_t crs_off = !has_crs ? 0 : cell.nof_ports == 1 ? (l == 0 ? cell.id % 6 : (cell.id + 3) % 6) : cell.id % 3;
      const uint32_t lp      = l + s * g.nof_symb_slot[0];
      for (uint32_t n = 0; n < cell.nof_prb; n++) {
        if (!g.prb_idx[s][n]) {
          continue;
        }
        uint32_t in = (lp * cell.nof_prb + n) * SRSRAN_NRE;
        if (!skip_symbol(cell, g, sf_idx, s, l, n)) {
          if (has_crs) {
            cp_ref(in, out, flag, (int)crs_off, (int)nof_refs, (int)nof_refs);
          } else {
            for (uint32_t k = 0; k < SRSRAN_NRE; k++) {
              out.push_back(in++);
            }
          }
        } else if (cell.nof_prb % 2 != 0) {  // odd PRB count: half of the centre PRBs carry PDSCH
          if (n == cell.nof_prb / 2 - 3) {
            if (has_crs) {
              cp_ref(in, out, flag, (int)crs_off, (int)nof_refs, (int)nof_refs / 2);
            } else {
              for (uint32_t k = 0; k < SRSRAN_NRE / 2; k++) {
                out.push_back(in++);
              }
            }
          } else if (n == cell.nof_prb / 2 + 3) {
            in += SRSRAN_NRE / 2;
            if (has_crs) {
              cp_ref(in, out, flag, (int)crs_off, (int)nof_refs, (int)nof_refs / 2);
            } else {
              for (uint32_t k = 0; k < SRSRAN_NRE / 2; k++) {
                out.push_back(in++);
              }
            }
          }
        }
      }
    }
  }
  return out;
}

}  // namespace srsran_amd

// added: the table as a C entry point (tests, external schedulers).  Returns the number of PDSCH
// REs and writes up to max_len grid indices (bit 31: CRS-bearing symbol).
extern "C" int srsran_pdsch_re_table(const srsran_cell_t*        cell,
                                     const srsran_pdsch_grant_t* grant,
                                     uint32_t                    lstart,
                                     uint32_t                    sf_idx,
                                     uint32_t*                   idx,
                                     uint32_t                    max_len)
{
  if (!cell || !grant) {
    return SRSRAN_ERROR_INVALID_INPUTS;
  }
  const std::vector<uint32_t> t = srsran_amd::pdsch_re_table(*cell, *grant, lstart, sf_idx);
  for (size_t i = 0; idx && i < t.size() && i < max_len; i++) {
    idx[i] = t[i];
  }
  return (int)t.size();
}
