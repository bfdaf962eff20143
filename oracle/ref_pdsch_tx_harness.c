/*
 * oracle/ref_pdsch_tx_harness.c -- TEST INFRASTRUCTURE ONLY (linked into oracle/_ref/libsrsref.so).
 *
 * Pins the GPU transmitter's PDSCH symbols (srsran_4g_amd/csrc/enc_kernel.hip pdsch_tx_kernel) to the
 * reference's own building blocks, compiled from /root/reference: bit scrambling
 * (srsran_sequence_pdsch_apply_pack, phch/sequences.c:72-81), modulation (srsran_mod_modulate_bytes over
 * srsran_modem_table_lte + srsran_modem_table_bytes, modem/mod.c:135, modem_table.c), layer mapping
 * (srsran_layermap_type, mimo/layermap.c:83) and precoding (srsran_precoding_type, mimo/precoding.c).
 * pdsch.c itself is not buildable here (generated headers); its srsran_pdsch_encode /
 * srsran_pdsch_codeword_encode sequence (pdsch.c:1017-1120, 960-1015) is restated below around those
 * calls.  The coded bits come from the caller (the oracle encoder, itself pinned to turbocoder.c /
 * rm_turbo.c); the RE mapping is pinned separately (ref_pdsch_map_harness.c).
 */
#include <complex.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "srsran/phy/common/phy_common.h"
#include "srsran/phy/common/sequence.h"
#include "srsran/phy/mimo/layermap.h"
#include "srsran/phy/mimo/precoding.h"
#include "srsran/phy/utils/vector.h"
#include "srsran/phy/modem/mod.h"
#include "srsran/phy/modem/modem_table.h"

/* 64-byte aligned, zeroed (the reference's SIMD precoders use aligned loads: srsran_vec_cf_malloc) */
static cf_t* cf_zalloc(size_t n)
{
  void* p = NULL;
  if (posix_memalign(&p, 64, n * sizeof(cf_t) + 64)) {
    return NULL;
  }
  memset(p, 0, n * sizeof(cf_t) + 64);
  return (cf_t*)p;
}

/* ncw codewords of nbits[c] coded bits each (one bit a byte in e[c * e_stride ...]), modulation mod[c]
 * (srsran_mod_t), scrambled with the codeword index cw_idx[c]; tx_scheme srsran_tx_scheme_t; nof_re
 * REs a port.  out: [nof_ports][nof_re] complex symbols (the q->symbols the reference maps to the REs).
 * Returns 0, or -1 on bad arguments. */
/* scaling: srsran_pdsch_encode's rho_a (pdsch.c:1057-1071, apply_power_allocation, pdsch.c:485-521) */
int ref_pdsch_tx_symbols_sc(uint32_t       ncw,
                            const uint8_t* e,
                            uint32_t       e_stride,
                            const uint32_t* nbits,
                            const uint32_t* mod,
                            const uint32_t* cw_idx,
                            uint16_t        rnti,
                            uint32_t        sf_idx,
                            uint32_t        cell_id,
                            int             tx_scheme,
                            uint32_t        nof_ports,
                            uint32_t        nof_layers,
                            uint32_t        pmi,
                            uint32_t        nof_re,
                            float           scaling,
                            float*          out)
{
  if (ncw == 0 || ncw > SRSRAN_MAX_CODEWORDS || nof_ports == 0 || nof_ports > SRSRAN_MAX_PORTS || nof_layers == 0 ||
      nof_layers > SRSRAN_MAX_LAYERS || nof_re == 0) {
    return -1;
  }
  int      ret = -1;
  cf_t*    d[SRSRAN_MAX_CODEWORDS] = {NULL};
  cf_t*    xl[SRSRAN_MAX_LAYERS]   = {NULL};
  cf_t*    y[SRSRAN_MAX_PORTS]     = {NULL};
  uint8_t* packed                  = NULL;
  const size_t nsym                = (size_t)nof_re * SRSRAN_MAX_LAYERS;
  for (uint32_t c = 0; c < SRSRAN_MAX_CODEWORDS; c++) {
    d[c] = cf_zalloc(nsym);
  }
  for (uint32_t l = 0; l < SRSRAN_MAX_LAYERS; l++) {
    xl[l] = cf_zalloc(nsym);
  }
  for (uint32_t p = 0; p < SRSRAN_MAX_PORTS; p++) {
    y[p] = cf_zalloc(nsym);
  }
  packed = calloc(e_stride / 8 + 16, 1);
  if (!packed) {
    goto out;
  }
  for (uint32_t i = 0; i < SRSRAN_MAX_LAYERS; i++) {
    if (!d[i % SRSRAN_MAX_CODEWORDS] || !xl[i] || !y[i % SRSRAN_MAX_PORTS]) {
      goto out;
    }
  }
  /* srsran_pdsch_codeword_encode (pdsch.c:960-1015): scrambling of the packed coded bits, then mapping */
  for (uint32_t c = 0; c < ncw; c++) {
    if (!d[c] || nbits[c] > e_stride || mod[c] >= SRSRAN_MOD_NITEMS) {
      goto out;
    }
    memset(packed, 0, e_stride / 8 + 16);
    for (uint32_t i = 0; i < nbits[c]; i++) {
      packed[i / 8] |= (uint8_t)((e[(size_t)c * e_stride + i] & 1) << (7 - i % 8));
    }
    srsran_sequence_pdsch_apply_pack(packed, packed, rnti, (int)cw_idx[c], 2 * sf_idx, cell_id, nbits[c]);
    srsran_modem_table_t tab;
    if (srsran_modem_table_lte(&tab, (srsran_mod_t)mod[c])) {
      goto out;
    }
    srsran_modem_table_bytes(&tab);
    srsran_mod_modulate_bytes(&tab, packed, d[cw_idx[c]], nbits[c]);
    srsran_modem_table_free(&tab);
  }
  /* srsran_pdsch_encode (pdsch.c:1066-1125): layer mapping and precoding with `scaling` */
  if (nof_ports > 1) {
    int   nof_symbols;
    cf_t* x[SRSRAN_MAX_LAYERS] = {NULL};
    if (nof_layers == ncw) {
      for (uint32_t i = 0; i < nof_layers; i++) {
        x[i] = d[i];
      }
      nof_symbols = (int)nof_re;
    } else {
      for (uint32_t i = 0; i < nof_layers; i++) {
        x[i] = xl[i];
      }
      nof_symbols = srsran_layermap_type(d, x, (int)ncw, (int)nof_layers, (int[SRSRAN_MAX_CODEWORDS]){nof_re, nof_re},
                                         (srsran_tx_scheme_t)tx_scheme);
    }
    const int codebook_idx = ncw == 1 ? (int)pmi : (int)pmi + 1;
    if (srsran_precoding_type(x, y, (int)nof_layers, (int)nof_ports, codebook_idx, nof_symbols, scaling,
                              (srsran_tx_scheme_t)tx_scheme) < 0) {
      goto out;
    }
  } else if (scaling == 1.0f) {
    memcpy(y[0], d[0], nof_re * sizeof(cf_t));
  } else {
    srsran_vec_sc_prod_cfc(d[0], scaling, y[0], nof_re);
  }
  for (uint32_t p = 0; p < nof_ports; p++) {
    memcpy(out + (size_t)2 * p * nof_re, y[p], nof_re * sizeof(cf_t));
  }
  ret = 0;
out:
  for (uint32_t c = 0; c < SRSRAN_MAX_CODEWORDS; c++) {
    free(d[c]);
  }
  for (uint32_t l = 0; l < SRSRAN_MAX_LAYERS; l++) {
    free(xl[l]);
  }
  for (uint32_t p = 0; p < SRSRAN_MAX_PORTS; p++) {
    free(y[p]);
  }
  free(packed);
  return ret;
}

/* the composition at scaling 1 (the batched transmitter's default, srsran_enb_dl_gpu_sf_t::pdsch_scaling unset) */
int ref_pdsch_tx_symbols(uint32_t ncw, const uint8_t* e, uint32_t e_stride, const uint32_t* nbits, const uint32_t* mod,
                         const uint32_t* cw_idx, uint16_t rnti, uint32_t sf_idx, uint32_t cell_id, int tx_scheme,
                         uint32_t nof_ports, uint32_t nof_layers, uint32_t pmi, uint32_t nof_re, float* out)
{
  return ref_pdsch_tx_symbols_sc(ncw, e, e_stride, nbits, mod, cw_idx, rnti, sf_idx, cell_id, tx_scheme, nof_ports,
                                 nof_layers, pmi, nof_re, 1.0f, out);
}

/* ---- PDSCH EVM (pdsch.c:698-713): the reference's own srsran_evm_run_s (modem/evm.h:175-212, static inline,
 * compiled here) on the equalised symbols of a codeword and its demodulated (pre-scrambling) int16 LLRs, with an
 * EVM buffer of max_bits bits (srsran_evm_buffer_alloc / _resize, pdsch.c:297, 468-471). ---- */
#include "srsran/phy/modem/evm.h"

float ref_evm_run_s(int mod, const cf_t* symbols, const int16_t* llr, uint32_t nof_bits, uint32_t max_bits)
{
  srsran_modem_table_t t;
  srsran_modem_table_init(&t);
  if (srsran_modem_table_lte(&t, (srsran_mod_t)mod)) {
    return NAN;
  }
  srsran_modem_table_bytes(&t);
  srsran_evm_buffer_t* b = srsran_evm_buffer_alloc(max_bits);
  const float          e = srsran_evm_run_s(b, &t, symbols, llr, nof_bits);
  srsran_evm_free(b);
  srsran_modem_table_free(&t);
  return e;
}

/* The 8-bit form, srsran_evm_run_b (evm.h:214-217 instantiation), on int8 demodulated LLRs. */
float ref_evm_run_b(int mod, const cf_t* symbols, const int8_t* llr, uint32_t nof_bits, uint32_t max_bits)
{
  srsran_modem_table_t t;
  srsran_modem_table_init(&t);
  if (srsran_modem_table_lte(&t, (srsran_mod_t)mod)) {
    return NAN;
  }
  srsran_modem_table_bytes(&t);
  srsran_evm_buffer_t* b = srsran_evm_buffer_alloc(max_bits);
  const float          e = srsran_evm_run_b(b, &t, symbols, llr, nof_bits);
  srsran_evm_free(b);
  srsran_modem_table_free(&t);
  return e;
}

/* ---- csi_correction (pdsch.c:523-618, static there) restated around the reference's own srsran_vec_max_fi and
 * built with the reference's release flags (oracle/Makefile REFFLAGS: -Ofast -mavx2 ...), so that the compiler's
 * treatment of its float expressions -- the scalar loops' division by csi_max in particular -- is the one a
 * reference build gets.  e: nof_bits LLRs, int8 when llr8 else int16, corrected in place. ---- */
#include <immintrin.h>
#include "srsran/phy/utils/vector.h"

void ref_csi_correction(int mod, const float* csi, void* e, uint32_t nof_bits, int llr8)
{
  const uint32_t qm = srsran_mod_bits_x_symbol((srsran_mod_t)mod);
  if (qm == 0) {
    return;
  }
  const uint32_t ns   = nof_bits / qm;
  const uint32_t imax = srsran_vec_max_fi(csi, ns);
  float          cmax = 1.0f;
  if (imax < ns) {
    cmax = csi[imax];
  }
  const float* cv = csi;
  if (llr8) {
    int8_t* eb = e;
    for (uint32_t i = 0; i < ns; i++) {
      const float c = *(cv++) / cmax;
      for (uint32_t k = 0; k < qm; k++, eb++) {
        *eb = (int8_t)((float)*eb * c);
      }
    }
    return;
  }
  int16_t* es = e;
  uint32_t i  = 0;
  __m128   sc = _mm_set1_ps(INT16_MAX / cmax);
  __m64*   v  = (__m64*)e;
  if (mod == SRSRAN_MOD_QPSK) { /* 4 LLRs = 2 symbols: lanes 0,1 <- symbol 1, lanes 2,3 <- symbol 0 (blend 3) */
    for (; i + 3 < nof_bits; i += 4) {
      __m128 a = _mm_set1_ps(*(cv++));
      __m128 b = _mm_set1_ps(*(cv++));
      *v       = _mm_mulhi_pi16(*v, _mm_cvtps_pi16(_mm_mul_ps(_mm_blend_ps(a, b, 3), sc)));
      v++;
    }
  } else if (mod == SRSRAN_MOD_16QAM) {
    for (; i + 3 < nof_bits; i += 4) {
      *v = _mm_mulhi_pi16(*v, _mm_cvtps_pi16(_mm_mul_ps(_mm_set1_ps(*(cv++)), sc)));
      v++;
    }
  } else if (mod == SRSRAN_MOD_64QAM) { /* 12 LLRs = 2 symbols over three 4-lane words */
    for (; i + 11 < nof_bits; i += 12) {
      __m128 a = _mm_mul_ps(_mm_set1_ps(*(cv++)), sc);
      __m128 b = _mm_mul_ps(_mm_set1_ps(*(cv++)), sc);
      v[0]     = _mm_mulhi_pi16(v[0], _mm_cvtps_pi16(a));
      v[1]     = _mm_mulhi_pi16(v[1], _mm_cvtps_pi16(_mm_blend_ps(a, b, 3)));
      v[2]     = _mm_mulhi_pi16(v[2], _mm_cvtps_pi16(b));
      v += 3;
    }
  } else if (mod == SRSRAN_MOD_256QAM) {
    for (; i + 7 < nof_bits; i += 8) {
      __m64 c = _mm_cvtps_pi16(_mm_mul_ps(_mm_set1_ps(*(cv++)), sc));
      v[0]    = _mm_mulhi_pi16(v[0], c);
      v[1]    = _mm_mulhi_pi16(v[1], c);
      v += 2;
    }
  }
  i /= qm;
  for (; i < ns; i++) {
    const float c = csi[i] / cmax;
    for (uint32_t k = 0; k < qm; k++) {
      es[qm * i + k] = (int16_t)((float)es[qm * i + k] * c);
    }
  }
}
