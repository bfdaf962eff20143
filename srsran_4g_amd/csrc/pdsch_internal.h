// srsran_4g_amd/csrc/pdsch_internal.h -- host helpers shared by the PHCH / PDSCH / UE DL C-ABI files.
#ifndef SRSRAN_AMD_PDSCH_INTERNAL_H
#define SRSRAN_AMD_PDSCH_INTERNAL_H
#include <stdint.h>

#include <vector>

#include "../../include/srsran_ue_dl.h"
#include "eq_kernel.h"
#include "stage_jobs.h"

namespace srsran_amd {

// predecoder scheme + norm for srsran_predecoding_type's arguments (phch_api.cpp)
bool pred_setup(PredArgs& a, int nrx, int nports, int nlayers, int codebook, int type, float scaling);
// sequence_pdsch_seed (sequences.c:62-65)
uint32_t pdsch_seed(uint16_t rnti, int q, uint32_t nslot, uint32_t cell_id);
// PDSCH RE gather table (pdsch_map.cpp)
std::vector<uint32_t> pdsch_re_table(const srsran_cell_t& cell, const srsran_pdsch_grant_t& g, uint32_t lstart,
                                     uint32_t sf_idx);

// srsran_dlsch_gpu_decode_batch with the descriptor upload on the DL-SCH object's copy stream (sch_api.cpp),
// for callers whose stream has work queued in front of the decode
int dlsch_gpu_decode_batch_early_copy(srsran_sch_t* q, uint32_t nof_tb, const srsran_dlsch_gpu_tb_t* tbs,
                                      int32_t* d_result, float* d_avg_noi, void* stream);
// the same with a per-TB iteration limit (0: the object's current one): one batch per distinct limit, each TB's
// result in its own slot; q is left at the last TB's limit, as after sequential decodes
int dlsch_gpu_decode_batch_limits(srsran_sch_t* q, uint32_t nof_tb, const srsran_dlsch_gpu_tb_t* tbs,
                                  const uint32_t* max_noi, int32_t* d_result, float* d_avg_noi, void* stream);

// srsran_chest_dl_gpu_estimate_batch_cfg with the nsf <= CHEST_INLINE_SF subframe indices h_sf[b] = tti % 10 given on
// the host and carried in the launch's arguments, and the batch's staging copies fused in (chest_api.cpp)
int chest_dl_gpu_estimate_batch_inline(srsran_chest_dl_t*           q,
                                       const srsran_chest_dl_cfg_t* cfg,
                                       const uint8_t*               h_sf,
                                       const CopyJobs*              jobs,  // fused staging copies (may be null)
                                       uint32_t                     nsf,
                                       const cf_t*                  d_grid,
                                       size_t                       grid_sf_stride,
                                       cf_t*                        d_ce,
                                       size_t                       ce_sf_stride,
                                       int                          full_grid,
                                       float*                       d_res,
                                       void*                        stream);
// the estimator options the batch estimator takes (the same check it makes, without launching anything; prints
// the reason when it returns false)
bool chest_batch_cfg_supported(const srsran_chest_dl_t* q, const srsran_chest_dl_cfg_t* cfg, int full_grid);

}  // namespace srsran_amd
#endif
