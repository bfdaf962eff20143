// srsran_4g_amd/csrc/ldpc_kernel.h -- launch interface of the HIP NR LDPC decoder.
#ifndef SRSRAN_AMD_LDPC_KERNEL_H
#define SRSRAN_AMD_LDPC_KERNEL_H
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace srsran_amd {

static constexpr int LDPC_MAX_EDGES = 316;  // BG1 (BG2: 197)
static constexpr int LDPC_WG        = 384;  // threads per workgroup upper bound
static constexpr int LDPC_LDS_HDR   = LDPC_MAX_EDGES * 4 + 128;  // shift table + scaling table

enum LdpcScale { LDPC_SCALE_C = 0, LDPC_SCALE_SIMD = 1 };

// One code block of an NR SCH transport block (CB mode, sch_nr.c:611-690): per-codeword input,
// number of layers, CRC type, skip flag and outputs.
struct LdpcCw {
  const int8_t* in;        // rate de-matched LLRs (the soft buffer of the code block, device)
  uint8_t*      data;      // packed message bits (cb_len of them) written when the CRC passes
  uint8_t*      flag;      // cb_crc: set -> skipped (already decoded); set to 1 when the CRC passes
  uint8_t*      iters;     // iterations used (ret == 0 ? max_iter : ret), 0 when skipped
  uint16_t      n_layers;  // from the rate-matched length (ldpc_decoder.c:70)
  uint16_t      cb_len;    // Kp - L_cb
  uint32_t      crc;       // 0: CRC24B (C > 1), 1: CRC24A, 2: CRC16 (TB CRC of single-CB TBs)
};

// One batch of codewords of one (base graph, lifting size), all decoded alike.
struct LdpcArgs {
  const void*     in;          // ncw x (liftN - 2 ls) LLRs (int8, or int16 if llr_bits == 16), in_stride bytes apart
  int             llr_bits;    // 8 (types C, C_AVX2, C_AVX512) or 16 (type S)
  uint32_t        in_stride;
  uint8_t*        out;         // ncw x liftK bytes (0/1) or liftK/8 packed bytes (device)
  uint32_t        out_stride;
  int             out_packed;  // 1: MSB-first packed bits (liftK/8 bytes, liftK % 8 == 0)
  uint8_t*        ret;         // optional per codeword: decode_crc_c's return (iterations; 0 = CRC failed)
  uint32_t        ncw;
  int             ls;
  int             cw_per_wg;   // codewords per workgroup (ls threads each)
  int             n_layers;    // layers processed (rate-matched length, ldpc_decoder.c:70); CB mode: the
                               // codewords' largest (selects the kernel instantiation)
  int             max_iter;
  int             scale_mode;  // LdpcScale
  int             sf;          // scaling factor as the mode's integer (65535ths or 100ths)
  const uint8_t*  scale_lut;   // scale(m), m = 0..127, in the decoder's arithmetic (device)
  const uint32_t* xpow;        // x^n mod P, n = 0 .. liftK (device), nullptr: no CRC early stop
  uint32_t        crc_poly;    // with its x^order bit
  int             crc_order;   // 16 or 24
  const uint32_t* sh;          // V mod ls per edge of the base graph, edge order (device)
  const LdpcCw*   cws;         // CB mode (nullptr: plain batch): per codeword descriptors
  const uint32_t* xpow3[3];    // CB mode: x^n mod P tables for CRC24B, CRC24A, CRC16 (device)
  uint32_t        magic_ls;    // ceil(2^32 / ls): i / ls = umulhi(i, magic_ls) for i < 2^16
};

constexpr int LDPC_FEW_LAYERS = 8;  // layer bound of the reduced-state instantiations

hipError_t ldpc_launch(int bg, const LdpcArgs& a, hipStream_t stream);
int        ldpc_cw_per_wg(int ls, int bits);
int        ldpc_threads_per_cw(int ls, int bits);
size_t     ldpc_lds_bytes(int bg, int ls, int bits);  // per workgroup

}  // namespace srsran_amd
#endif
