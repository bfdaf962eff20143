// srsran_4g_amd/csrc/chest_kernel.h -- DL channel estimation (CRS, srsUE default configuration).
#ifndef SRSRAN_AMD_CHEST_KERNEL_H
#define SRSRAN_AMD_CHEST_KERNEL_H
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "stage_jobs.h"

namespace srsran_amd {

static constexpr int CHEST_MAX_PRB  = 110;
static constexpr int CHEST_MAX_NREF = 2 * CHEST_MAX_PRB;  // pilots per CRS symbol
static constexpr int CHEST_INLINE_SF = 512;  // subframe indices a batch launch carries in its arguments

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
  uint32_t      filter_none; // SRSRAN_CHEST_FILTER_NONE: no average_pilots -- the LS estimates interpolated as they
                             // are (chest_dl.c:724-725); TRIANGLE is filter[] = {w, 1 - 2w, w} (chest_common.c:62-68)
  const float2* mbsfn_pilots; // chest_mbsfn_kernel: the MBSFN reference signals of the subframe, [3][6 nof_prb]
  // ---- estimator options beyond srsUE's defaults (chest_dl.c:437-555, 402-433, 703-745) ----
  uint32_t        estimator;  // 0 AVERAGE (one row, copied), 1 INTERPOLATE (full_grid: every row its own)
  uint32_t        noise_alg;  // 0 REFS (pilot residuals), 1 PSS, 2 EMPTY (subframes 0 / 5 only)
  const float2*   pss;        // the 62 PSS values of N_id_2 (noise_alg 1)
  const float*    noise_in;   // [rx][port] (4 x 4) kept noise estimates: the automatic filter's input and the
                              // result of PSS / EMPTY outside subframes 0 / 5 (q->noise_estimate)
  uint32_t        sf_index;   // tti % 10 when sf_idx (below) is null
  // TDD special subframes (refsignal_dl.c:169-226): bit i of special_mask = subframe index i is special; its DwPTS
  // holds ss_nsym[0] CRS symbols of ports 0 / 1 and ss_nsym[1] of ports 2 / 3 (every other subframe: 4 / 2)
  uint32_t        special_mask;
  uint32_t        ss_nsym[2];
  // ---- batches of subframes (gridDim.y = nof subframes) ----
  const uint32_t* sf_idx;     // [b] subframe index (tti % 10): pilots + sf_idx[b] * CHEST_PILOTS_PER_SF; null = as given
  size_t          grid_sf_stride; // float2 between subframes of `grid`
  size_t          ce_sf_stride;   // float2 between subframes of `ce`
  // subframe indices carried in the launch arguments (batches of <= CHEST_INLINE_SF subframes, sf_inl = 1): no
  // host buffer for the GPU to read, so no ring slot and no event to free it
  uint32_t        sf_inl;
  uint8_t         sf_inline[CHEST_INLINE_SF];
  // staging copies of the batch's PDSCH / DL-SCH descriptors fused into the launch (stage_jobs.h; n = 0: none):
  // their PCIe reads go out with the pilot loads and are stored at the end
  CopyJobs        jobs;
};

// CRS symbols of `port` in subframe index sfi (srsran_refsignal_cs_nof_symbols)
__host__ __device__ inline uint32_t chest_crs_nsym(const ChestArgs& a, uint32_t sfi, uint32_t port)
{
  return ((a.special_mask >> sfi) & 1u) ? a.ss_nsym[port < 2 ? 0 : 1] : (port < 2 ? 4u : 2u);
}

static constexpr size_t CHEST_PILOTS_PER_SF = 2 * 4 * CHEST_MAX_NREF;  // float2 (both port pairs)
static constexpr size_t CHEST_STATS_PER_SF  = 4 * 4 * 8;               // floats of stats per subframe
// stats per (rx, port): [0] noise, [1] rsrp, [2] rssi, [3] / [4] CFO phase sum, [5] 1 when [0] is a new PSS / EMPTY
// estimate (subframes 0 / 5), 0 when it is noise_in

hipError_t chest_launch(const ChestArgs& a, hipStream_t stream, uint32_t nsf = 1);
// estimate_port_mbsfn (chest_dl.c:836-865) of one MBSFN subframe (host-synchronous path): one workgroup per
// (port, rx); ce rows 0..11 of the (port, rx) estimate written, stats [0] = noise (REFS, or noise_in), rest 0
hipError_t chest_mbsfn_launch(const ChestArgs& a, hipStream_t stream);
// diagnostic build (-DCHEST_STAMPS) only: phase clock stamps of every chest_kernel workgroup into d_buf
hipError_t chest_set_stamps(void* d_buf);
// device-side reduction of the per-(rx, port) stats of nsf subframes into out[b][4] =
// {noise_estimate, rsrp, rssi, cfo} (fill_res, chest_dl.c:962-986); a subframe without 4 CRS symbols (TDD special)
// keeps the CFO before it, from *cfo_state (device, may be null: 0) across calls, which is updated
hipError_t chest_finalize_launch(const float* stats, uint32_t np, uint32_t nrx, uint32_t nof_prb, float symbol_sz,
                                 uint32_t nsymb, float* out, uint32_t nsf, hipStream_t stream,
                                 float* cfo_state = nullptr);
// the same for PSS / EMPTY noise over a batch, in subframe order: a subframe without a new estimate takes the
// (rx, port) value left by the subframes before it, starting from state[rx * 4 + port], which holds the last
// values afterwards (q->noise_estimate across calls)
hipError_t chest_finalize_kept_launch(float* stats, uint32_t np, uint32_t nrx, uint32_t nof_prb, float symbol_sz,
                                      uint32_t nsymb, float* state, float* out, uint32_t nsf, hipStream_t stream,
                                      float* cfo_state = nullptr);

// correct_sync_error (chest_dl.c:750-804), device side of the host-synchronous path: per (rx, port) the LS
// estimates' per-CRS-symbol phase sums sum(x[i] conj(x[i-1])) and their power sum -> out[(rx * 4 + port) * 10 ..]:
// 4 complex sums, then the power sum (the host finishes with the reference's scalar arithmetic)
hipError_t chest_sync_sums_launch(const ChestArgs& a, float* out, hipStream_t stream, uint32_t nsf = 1);
static constexpr size_t CHEST_SYNC_PER_SF = 4 * 4 * 10;  // floats of phase sums per subframe
// the batch's correction (chest_dl.c:750-804): per (rx, subframe) the reference's arithmetic on the sums of
// chest_sync_sums_launch, the sync error of every (rx, port) into serr[b][rx * 4 + port], and where |error| > 0.05
// samples every row of that rx grid (grid + b * a.grid_sf_stride) rotated in place by srsran_vec_apply_cfo's phasors
hipError_t chest_sync_apply_launch(const ChestArgs& a, const float* sums, float* serr, float2* grid, float symbol_sz,
                                   uint32_t nsf, hipStream_t stream);
// rows (2 nsymb of every rx grid) multiplied in place by the phasor table tab[nre] (srsran_vec_apply_cfo per row)
hipError_t grid_rotate_launch(float2* grid, const float2* tab, uint32_t nre, uint32_t nrows, hipStream_t stream);

}  // namespace srsran_amd
#endif
