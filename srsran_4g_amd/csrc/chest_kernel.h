// srsran_4g_amd/csrc/chest_kernel.h -- DL channel estimation (CRS, srsUE default configuration).
#ifndef SRSRAN_AMD_CHEST_KERNEL_H
#define SRSRAN_AMD_CHEST_KERNEL_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srsran_amd {

static constexpr int CHEST_MAX_PRB  = 110;
static constexpr int CHEST_MAX_NREF = 2 * CHEST_MAX_PRB;  // pilots per CRS symbol

struct ChestArgs {
  const float2* grid;      // [rx][14 * nre] received subframe grids
  const float2* pilots;    // [port pair][4 * nref] CRS of this subframe (ports 2/3: 2 symbols)
  float2*       ce;        // [port][rx][ce_stride] estimates
  float*        stats;     // [rx][port][4]: noise, rsrp, rssi, cfo-sum (re) ; cfo-sum (im) at [4*..+3]
  uint32_t      nof_prb;
  uint32_t      cell_id;
  uint32_t      nports;
  uint32_t      nrx;
  uint32_t      ce_stride; // float2 per (port, rx): nre (one row) or 14 * nre (full grid)
  uint32_t      full_grid; // write all 14 symbols (srsran_chest_dl_res_t layout)
  float         filter[8]; // smoothing filter (srsran_chest_set_smooth_filter_gauss)
  uint32_t      filter_len;
  uint32_t      filter_auto; // Gauss order 4, stddev = 200 * noise of the (port, rx) (chest_dl.c:703-704)
};

hipError_t chest_launch(const ChestArgs& a, hipStream_t stream);

}  // namespace srsran_amd
#endif
