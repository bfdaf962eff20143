// srsran_4g_amd/csrc/chest_kernel.h -- DL channel estimation (CRS, srsUE default configuration).
#ifndef SRSRAN_AMD_CHEST_KERNEL_H
#define SRSRAN_AMD_CHEST_KERNEL_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srsran_amd {

static constexpr int CHEST_MAX_PRB  = 110;
static constexpr int CHEST_MAX_NREF = 2 * CHEST_MAX_PRB;  // pilots per CRS symbol

struct ChestArgs {
  const float2* grid;      // [rx][2 nsymb * nre] received subframe grids
  const float2* pilots;    // [port pair][4 * nref] CRS of this subframe (ports 2/3: 2 symbols)
  float2*       ce;        // [port][rx][ce_stride] estimates
  float*        stats;     // [rx][port][4]: noise, rsrp, rssi, cfo-sum (re) ; cfo-sum (im) at [4*..+3]
  uint32_t      nof_prb;
  uint32_t      cell_id;
  uint32_t      nports;
  uint32_t      nrx;
  uint32_t      ce_stride; // float2 per (port, rx): nre (one row) or 2 nsymb * nre (full grid)
  uint32_t      full_grid; // write all 2 nsymb symbols (srsran_chest_dl_res_t layout)
  uint32_t      nsymb;     // symbols per slot: 7 (normal CP) or 6 (extended CP)
  float         filter[8]; // smoothing filter (srsran_chest_set_smooth_filter_gauss)
  uint32_t      filter_len;
  uint32_t      filter_auto; // Gauss order 4, stddev = 200 * noise of the (port, rx) (chest_dl.c:703-704)
  // ---- batches of subframes (gridDim.y = nof subframes) ----
  const uint32_t* sf_idx;     // [b] subframe index (tti % 10): pilots + sf_idx[b] * CHEST_PILOTS_PER_SF; null = as given
  size_t          grid_sf_stride; // float2 between subframes of `grid`
  size_t          ce_sf_stride;   // float2 between subframes of `ce`
};

static constexpr size_t CHEST_PILOTS_PER_SF = 2 * 4 * CHEST_MAX_NREF;  // float2 (both port pairs)
static constexpr size_t CHEST_STATS_PER_SF  = 4 * 4 * 8;               // floats of stats per subframe

hipError_t chest_launch(const ChestArgs& a, hipStream_t stream, uint32_t nsf = 1);
// device-side reduction of the per-(rx, port) stats of nsf subframes into out[b][4] =
// {noise_estimate, rsrp, rssi, cfo} (fill_res, chest_dl.c:962-986)
hipError_t chest_finalize_launch(const float* stats, uint32_t np, uint32_t nrx, uint32_t nof_prb, float symbol_sz,
                                 uint32_t nsymb, float* out, uint32_t nsf, hipStream_t stream);

}  // namespace srsran_amd
#endif
