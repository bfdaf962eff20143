// srsran_4g_amd/csrc/sch_kernel.h -- launch interface of the DL-SCH kernels.
//
// A DL-SCH batch is a set of transport blocks; each TB owns C consecutive "slots"
// (one per code block).  Three kernels run in order on one stream:
//   1. rm_rx_kernel     rate de-matching of every slot into its HARQ soft buffer
//                       (srsran_rm_turbo_rx_lut, rm_turbo.c:390-483)
//   2. tdec_kernel<ES>  turbo decode with CRC early stop (decode_tb_cb, sch.c:420-456)
//   3. tb_kernel        TB assembly, CB bookkeeping, TB CRC (sch.c:458-573)
#ifndef SRSRAN_AMD_SCH_KERNEL_H
#define SRSRAN_AMD_SCH_KERNEL_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srsran_amd {

static constexpr int SCH_SLOT_BYTES = 768;  // decision bytes per slot (K <= 6144)
static constexpr int SCH_MAX_CB     = 32;   // SRSRAN_MAX_CODEBLOCKS (phy_common.h:64)
static constexpr int TB_MAX_CHUNKS  = 32;
static constexpr int RM_LDS_MAX_E   = 24576;  // E LLRs a CB may have for the LDS de-matcher (48 KB)   // 1 KB CRC chunks per TB (>= 32 * 6144 / 8 / 1024)

struct RmSlot {
  const short*    e;     // the CB's E rate-matched LLRs (device)
  short*          sb;    // the CB's soft buffer (device)
  const uint8_t*  skip;  // soft buffer cb_crc flag: set -> not de-matched (sch.c:392)
  const uint16_t* inv;   // layout position -> circular-buffer index, 0xFFFF for padding
  uint32_t        E;
  uint32_t        len;   // positions in the soft buffer layout (3K+12 or 3(K+32)+12)
  uint32_t        N;     // 3K+12: period of the circular buffer after dummy removal
  uint32_t        overwrite;  // new transmission: sb = sum (the reset buffer is zero), flag ignored
};

struct SchTb {
  uint8_t*       data;      // TB payload (device)
  const uint8_t* cbout;     // decision bytes per slot (SCH_SLOT_BYTES apart)
  const uint8_t* noi;       // per slot: half-iterations (0 = skipped)
  const uint8_t* crc_ok;    // per slot
  uint8_t*       cb_crc;    // soft buffer flags (device, max_cb)
  uint8_t*       tb_crc;    // soft buffer TB flag (device)
  uint8_t*       saved;     // soft buffer saved payloads (device)
  int32_t*       result;    // decode_tb return value (device)
  float*         avg;       // avg_iterations (device)
  short*         sbuf;      // soft buffer arena (sb_stride int16 per CB), for new-transmission resets
  uint32_t       saved_stride;
  uint32_t       sb_stride;
  uint32_t       max_cb;
  uint32_t       nof_cb_reset;  // CBs srsran_softbuffer_rx_reset_tbs clears (softbuffer.c:146-150)
  uint32_t       new_data;
  uint32_t       slot0;
  uint32_t       C, C1, K1, K2, tbs;
  int32_t        status;    // 1: decoded; otherwise the return value of a host-side check
};

// max_e: the largest E of the batch (the LDS de-matcher takes E <= RM_LDS_MAX_E)
hipError_t rm_rx_launch(const RmSlot* d_slots, uint32_t nslots, uint32_t max_len, uint32_t max_e,
                        hipStream_t stream);
// max_tbs: the largest TBS of the batch (sizes the assembly grid)
hipError_t tb_launch(const SchTb* d_tbs, uint32_t ntb, uint32_t max_tbs, hipStream_t stream);

// UL-SCH channel de-interleaver without RI bits (sch.c:661-682, 994-1021):
// g[(j N_symb + i) Qm + k] = q[(i rows + j) Qm + k], rows = H' / N_symb
hipError_t ul_deint_launch(const int16_t* q, int16_t* g, uint32_t Qm, uint32_t H_prime_total, uint32_t N_symb,
                           hipStream_t stream);
struct UlDeint {
  const int16_t* q;
  int16_t*       g;
  uint32_t       rows, cols, Qm;
  // RI multiplexed (sch.c:994-1021 with ri_present): column i holds RI in its last ri_rows[i]
  // rows, which the de-interleaver skips; srsran_vec_lut_sis maps every skipped position to
  // g[0], so the last one (q[g0_src]) ends there.  ri_rows all 0 / g0_src < 0 without RI.
  uint16_t ri_rows[14];
  int32_t  g0_src;
};
// many TBs in one launch (grid.y = TB); d_desc on the device; cols <= 14, Qm <= 8
hipError_t ul_deint_batch_launch(const UlDeint* d_desc, uint32_t ntb, uint32_t max_rows, hipStream_t stream);

}  // namespace srsran_amd
#endif
