/* oracle/phy_oracle.h -- CPU restatement of the PDSCH LLR stages (test infrastructure only). */
#ifndef ORACLE_PHY_H
#define ORACLE_PHY_H
#include <stdint.h>

int      oracle_demod_soft_s(int mod, const float* sym, int16_t* llr, int n);
void     oracle_sequence_bits(uint32_t seed, uint8_t* c, uint32_t len);
void     oracle_sequence_apply_s(const int16_t* in, int16_t* out, uint32_t len, uint32_t seed);
uint32_t oracle_pdsch_seed(uint16_t rnti, int q, uint32_t nslot, uint32_t cell_id);
int      oracle_predecode(int scheme, int nrx, int nports, int nlayers, int codebook, const float* y, const float* h,
                          float* x, float* csi, int n, float scaling, float noise);
void     oracle_csi_correction(int mod, const float* csi, int16_t* e, uint32_t nof_bits);
#endif
