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
int      oracle_demod_soft_b(int mod, const float* sym, int8_t* llr, int n);
void     oracle_sequence_apply_c(const int8_t* in, int8_t* out, uint32_t len, uint32_t seed);
void     oracle_csi_correction_b(int mod, const float* csi, int8_t* e, uint32_t nof_bits);
void     oracle_crs_pilots(uint32_t cell_id, uint32_t nof_prb, uint32_t pp, uint32_t sf, float* out);
uint32_t oracle_gauss_filter(float* f, uint32_t order, float std_dev);
void     oracle_conv_same(const float* in, const float* f, float* out, uint32_t N, uint32_t M);
int      oracle_chest_dl(const float* grid, uint32_t nof_prb, uint32_t cell_id, uint32_t nports, uint32_t nrx,
                         uint32_t sf_idx, uint32_t symbol_sz, float* ce, float* out);
int      oracle_chest_dl_cp(const float* grid, uint32_t nof_prb, uint32_t cell_id, uint32_t nports, uint32_t nrx,
                            uint32_t sf_idx, uint32_t symbol_sz, uint32_t cp, float* ce, float* out);
void     oracle_crs_pilots_cp(uint32_t cell_id, uint32_t nof_prb, uint32_t pp, uint32_t sf, uint32_t cp, float* out);
int      oracle_chest_dl_tdd(const float* grid, uint32_t nof_prb, uint32_t cell_id, uint32_t nports, uint32_t nrx,
                             uint32_t sf_idx, uint32_t symbol_sz, uint32_t cp, uint32_t nsym01, uint32_t nsym23,
                             float* ce, float* out);
#endif
