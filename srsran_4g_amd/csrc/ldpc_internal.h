// srsran_4g_amd/csrc/ldpc_internal.h -- entry points of the LDPC decoder for other modules of the
// library (NR SCH): code-block mode launches over a decoder object.
#ifndef SRSRAN_AMD_LDPC_INTERNAL_H
#define SRSRAN_AMD_LDPC_INTERNAL_H
#include <vector>
#include "../../include/srsran_ldpc.h"
#include "ldpc_kernel.h"

namespace srsran_amd {

// layers processed for a rate-matched length (ldpc_decoder.c:48-70)
int ldpc_layers_for(const srsran_ldpc_decoder_t* q, uint32_t cdwd_rm_length);
// n code blocks described by d_cws (device) through decoder q (8-bit types), CRC early stop per block
// max_layers: the largest n_layers of the descriptors (0: unknown)
int ldpc_launch_cws(srsran_ldpc_decoder_t* q, const LdpcCw* d_cws, uint32_t n, const uint32_t* const xpow3[3],
                    uint32_t max_layers,
                    hipStream_t stream);
// x^n mod P, n = 0 .. nmax (P with its x^order bit)
std::vector<uint32_t> ldpc_xpow_table(uint32_t poly, int order, int nmax);

}  // namespace srsran_amd
#endif
