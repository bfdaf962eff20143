// srsran_4g_amd/csrc/nr_sch_kernel.h -- NR SCH receive kernels: LDPC rate de-matching and TB assembly.
#ifndef SRSRAN_AMD_NR_SCH_KERNEL_H
#define SRSRAN_AMD_NR_SCH_KERNEL_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srsran_amd {

// One code block's rate de-matching (srsran_ldpc_rm_rx_c, ldpc_rm.c:675-706) into its soft buffer.
struct NrRmCb {
  const int8_t*  e;      // the TB's rate-matched LLRs (device)
  uint8_t*       flags;  // the TB's cb_crc flags (device): a set flag skips the block and its E
  int8_t*        buf;    // soft buffer of the block (device, >= Ncb bytes)
  uint32_t       r;      // block index in the TB
  uint32_t       E0, E1, jthr;  // E_r = r <= jthr ? E0 : E1 (sch_nr.c:178-189)
  uint32_t       Qm, k0, Ncb, ini, end;  // bit selection: start, circular length, filler range
  uint8_t*       data;        // saved payload of the block (device)
  uint32_t       data_bytes;  // bytes of it a new transmission clears
  uint32_t       fresh;       // new data: flags, soft bits [0, Ncb) and payload of the TB's blocks start from zero
};

// One TB's assembly (sch_nr.c:692-748).
struct NrTb {
  const uint8_t* flags;   // cb_crc[C] (device)
  const uint8_t* data;    // packed code block bits, block r at data + r * data_stride (device)
  const uint8_t* iters;   // iterations per block (device)
  uint8_t*       payload; // A / 8 bytes (device)
  uint8_t*       crc_out; // 1: TB CRC ok
  float*         avg_out; // average iterations
  uint32_t*      scratch; // 2 dwords (CRC accumulator, finished slices), zero between launches
  uint32_t       data_stride, C, A, Kp, L_cb, L_tb;
};

// TB assembly slices: each workgroup copies and CRCs NR_TB_SLICE payload bytes of one TB
constexpr uint32_t NR_TB_THREADS = 256;
constexpr uint32_t NR_TB_BYTES   = 16;  // contiguous bytes per thread
constexpr uint32_t NR_TB_SLICE   = NR_TB_THREADS * NR_TB_BYTES;

hipError_t nr_rm_launch(const NrRmCb* d_cbs, uint32_t ncb, hipStream_t stream);
// slices = max over the TBs of ceil(payload bytes / NR_TB_SLICE) (at least 1)
hipError_t nr_tb_launch(const NrTb* d_tbs, uint32_t ntb, uint32_t slices, hipStream_t stream);

}  // namespace srsran_amd
#endif
