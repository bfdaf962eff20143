// srsran_4g_amd/csrc/tdec_kernel.h -- launch interface of the HIP turbo decoder.
#ifndef SRSRAN_AMD_TDEC_KERNEL_H
#define SRSRAN_AMD_TDEC_KERNEL_H
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace srsran_amd {

static constexpr int TDEC_W       = 32;  // beta checkpoint window (must match the kernel)
static constexpr int TDEC_OVERLAP = 40;  // sliding-window training length

// One code block of a DL-SCH decode (launch-index order).
struct TdecCb {
  const short*   in;    // soft buffer of the block (rate de-matched LLRs)
  const uint8_t* skip;  // soft buffer cb_crc flag: set -> block already decoded (sch.c:392)
  uint32_t       slot;  // index into out / noi_out / crc_ok
  uint32_t       crc_a; // 1 -> CRC24A over tbs+24 (single-CB TB), 0 -> CRC24B (sch.c:440-446)
};
// slot of a padding descriptor: decodes nothing, writes nothing.  The host inserts one where two
// neighbouring blocks of a launch lie too far apart to share the lane-pair decoder's workgroup
// (one buffer resource over both), so the pair starts with the next block instead.
static constexpr uint32_t TDEC_PAD_SLOT = 0xffffffffu;
// the two blocks of a lane-pair workgroup must lie within this many bytes of each other
static constexpr uint64_t TDEC_PAIR_SPAN = ((uint64_t)1 << 31) - ((uint64_t)1 << 16);
static constexpr uint32_t TDEC_GROUP     = 8;  // blocks per workgroup of the largest such decoder (tdec8s)

struct TdecArgs {
  const short*    in;        // ncb code blocks, in_stride int16 apart (device)
  uint32_t        in_stride;
  int             layout_sb; // 0: natural 3K+12, 1: rm_turbo sub-block layout
  uint32_t        K;
  uint32_t        ncb;
  int             n_start;   // first half-iteration index to run
  int             n_end;     // one past the last half-iteration index
  uint8_t*        out;       // ncb * K/8 hard-decision bytes (device)
  const uint16_t* tfwd;      // slot of pi(n(q))    (device, K entries, q order)
  const uint16_t* trev;      // slot of pi^-1(n(q)) (device, K entries, q order)
  const uint16_t* tfwd_nat;  // slot of pi(n)       (device, K entries, natural order)
  const uint16_t* trev_nat;  // slot of pi^-1(n)    (device, K entries, natural order)
  short*          state;     // optional ncb * 2 * xyw saved LLR/AUX state (device) or nullptr
  uint32_t        L;         // sub-block length (K for the generic decoder)
  uint32_t        Ls;        // LDS slot stride per sub-block
  uint32_t        xyw;       // LDS words per code block
  uint32_t        M;         // beta checkpoints per sub-block
  uint32_t        magicL;    // ceil(2^32 / L)
  uint32_t        magicLs;   // ceil(2^32 / Ls)
  // ---- DL-SCH mode (decode_tb_cb, sch.c:391-456): enabled when cbs != nullptr ----
  const struct TdecCb* cbs;  // per launch index: input pointer, skip flag, output slot, CRC type
  uint32_t        out_stride; // bytes between output slots
  uint8_t*        noi_out;   // per slot: half-iterations run (0 = skipped, CRC already OK)
  uint8_t*        crc_ok;    // per slot: 1 if the block's CRC passed (or it was skipped)
  const uint32_t* xpow_a;    // x^(8m) mod CRC24A, m = 0..768 (device)
  const uint32_t* xpow_b;    // x^(8m) mod CRC24B
  int             min_iters; // early stop needs at least this many half-iterations (sch.c:35)
};

static constexpr uint32_t LTE_CRC24A = 0x1864CFB;  // phy_common.h:72
static constexpr uint32_t LTE_CRC24B = 0x1800063;  // phy_common.h:73

hipError_t tdec_launch(int nsb, const TdecArgs& a, hipStream_t stream);
// ngroups descriptors of one decoder class (device array) in one launch; d_first[g] = first
// workgroup of group g (ascending); lds = the largest tdec_lds_bytes of the groups
hipError_t tdec_multi_launch(int nsb, const TdecArgs* d_groups, const uint32_t* d_first, int ngroups,
                             uint32_t nblocks, size_t lds, hipStream_t stream);
int        tdec_cpw(int nsb);  // code blocks per workgroup

// tdec16_kernel.hip: the lane-pair decoder of the 16-sub-block class on the SB input layout
// (every plain / DL-SCH launch of K >= 816 without state save/restore)
bool       tdec16_eligible(int nsb, const TdecArgs& a);
bool       tdec16_pays(uint32_t ncb);  // enough blocks in one launch for the lane-pair kernel
void       tdec16_set_min_cb(uint32_t n);
uint32_t   tdec16_min_cb();
hipError_t tdec16_launch(const TdecArgs& a, hipStream_t stream);
hipError_t tdec16_multi_launch(const TdecArgs* d_groups, const uint32_t* d_first, int ngroups, uint32_t nblocks,
                               size_t lds, hipStream_t stream);
size_t     tdec16_lds_bytes(const TdecArgs& a);
int        tdec16_cpw();
// tdecs_kernel.hip: one lane per sub-block (64 / NSB blocks a workgroup), the window classes of large
// batches (16 sub-blocks: eligible where tdec16_eligible is, chosen from tdec16s_min_cb() blocks a
// launch; 8 sub-blocks: tdec8s_eligible)
#define SRSRAN_TDECS_API(ns)                                                                               \
  namespace ns {                                                                                           \
  hipError_t launch(const TdecArgs& a, hipStream_t stream);                                                \
  hipError_t multi_launch(const TdecArgs* d_groups, const uint32_t* d_first, int ngroups, uint32_t nblocks, \
                          size_t lds, hipStream_t stream);                                                 \
  size_t     lds_bytes(const TdecArgs& a);                                                                 \
  int        cpw();                                                                                        \
  }
SRSRAN_TDECS_API(tdecs16)
SRSRAN_TDECS_API(tdecs8)
SRSRAN_TDECS_API(tdecs16w8)  // the same built with 8-step windows (fewer registers, more checkpoints)
SRSRAN_TDECS_API(tdecs8w8)
SRSRAN_TDECS_API(tdecs1)  // tdec1s_kernel.hip: the generic decoder (K <= 400), one lane per block and side
#undef SRSRAN_TDECS_API
#ifdef TDECS_STAMPS  // diagnostic build (Makefile `stamps`): phase-boundary clock stamps of the single-lane kernels
namespace tdecs16 { hipError_t set_stamps(void* d_buf); }
namespace tdecs8 { hipError_t set_stamps(void* d_buf); }
namespace tdecs16w8 { hipError_t set_stamps(void* d_buf); }
namespace tdecs8w8 { hipError_t set_stamps(void* d_buf); }
#endif
bool       tdec8s_eligible(int nsb, const TdecArgs& a);
bool       tdec1s_eligible(int nsb, const TdecArgs& a);
// srsran_tdec_gpu_set_w8_max_k(): window classes of K up to this size run the 8-step-window build
void       tdecs_set_w8_max_k(uint32_t k);
// srsran_tdec_gpu_set_w8_fused_max_k(): the 16-sub-block class's cut in fused multi-size launches
void       tdecs_set_w8_fused_max_k(uint32_t k);
uint32_t   tdecs_w8_fused_max_k();
uint32_t   tdecs_w8_max_k();
void       tdec8s_set_min_cb(uint32_t n);
uint32_t   tdec8s_min_cb();
void       tdec1s_set_min_cb(uint32_t n);
uint32_t   tdec1s_min_cb();
void       tdec16s_set_min_cb(uint32_t n);
uint32_t   tdec16s_min_cb();
// the kernel the 16-sub-block class runs for a launch of ncb blocks on the SB layout: 2 = single lane
// per sub-block (tdec16s), 1 = lane pair (tdec16), 0 = quad (tdec_kernel<16>)
int        tdec16_choice(uint32_t ncb);
size_t     tdec_lds_bytes(int nsb, int xyw, int M);
// x^(8m) mod poly for m = 0..nm-1 (host helper for the CRC combine tables)
void crc24_xpow_table(uint32_t poly, uint32_t* out, int nm);

// DL-SCH decode of ncb code blocks of size K (tdec_api.cpp): AUTO decoder, soft
// buffer layout (SB for K >= 408), CRC early stop after >= 2 half-iterations, at
// most n_end half-iterations; decisions to d_out + slot * out_stride.
int tdec_sch_enqueue(uint32_t      K,
                     const TdecCb* d_cbs,
                     uint32_t      ncb,
                     uint8_t*      d_out,
                     uint32_t      out_stride,
                     uint8_t*      d_noi,
                     uint8_t*      d_crc_ok,
                     int           n_end,
                     hipStream_t   stream);
// the same with llr_is_8bit for K > 800 (tdec8bit_kernel.hip's 8-bit window decoders; int8 soft buffers in the
// 8-bit decoder's layout)
int tdec8_sch_enqueue(uint32_t K, const TdecCb* d_cbs, uint32_t ncb, uint8_t* d_out, uint32_t out_stride,
                      uint8_t* d_noi, uint8_t* d_crc_ok, int n_end, hipStream_t stream);
// Appends the n blocks of `src` to `dst` so that every aligned group of TDEC_GROUP consecutive entries
// counted from `dst_group_start` (a workgroup of the lane-pair or single-lane decoder) lies within
// TDEC_PAIR_SPAN: padding entries close a group before a block too far from the group's others.
// Returns the padding entries added.
uint32_t tdec_pair_cbs(const TdecCb* src, uint32_t n, size_t dst_group_start, void* dst_vec);
// name of the last turbo-decoder kernel this thread launched ("" before the first)
const char* tdec_last_kernel();
void        tdec_set_last_kernel(const char* name);
int tdec_cb_index(uint32_t K);

}  // namespace srsran_amd
#endif
