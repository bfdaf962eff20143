// srsran_4g_amd/csrc/ofdm_kernel.h -- OFDM demodulation (CP removal, CFO, FFT, subcarrier map).
#ifndef SRSRAN_AMD_OFDM_KERNEL_H
#define SRSRAN_AMD_OFDM_KERNEL_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srsran_amd {

static constexpr int OFDM_MAX_N      = 2048;
static constexpr int OFDM_MAX_STAGES = 6;

struct OfdmArgs {
  const float2* in;        // [sf][rx][sf_len] time-domain samples
  float2*       out;       // [sf][rx][2 nsymb][nre] resource grid
  const float2* tw;        // exp(-2 pi i m / N), m = 0..N-1
  uint32_t      N;         // FFT size (symbol_sz)
  uint32_t      cp0, cp;   // first / other cyclic prefix lengths of a slot
  uint32_t      nsymb;     // symbols per slot: 7 (normal CP) or 6 (extended CP, cp0 = cp)
  uint32_t      nre;       // 12 * nof_prb
  uint32_t      sf_len;    // samples per subframe and antenna
  uint32_t      nrx;
  float         norm;      // 1 or 1/sqrt(N) (srsran_ofdm_cfg_t.normalize)
  const float2* cfo_tab;   // srsran_vec_apply_cfo's phasor of every sample of a subframe (cfo_table_launch,
                           // sf_len entries), applied as z = x * tab[n], n from the subframe start; nullptr = off
  // MBSFN subframes (ofdm_rx_slot_mbsfn, ofdm.c:522-535): slot 0's symbols start at mbsfn_off[i] (the non-MBSFN
  // region's normal cyclic prefixes, the guard, then extended ones); 0 = every slot as cp0 / cp say
  uint32_t      mbsfn;
  uint32_t      mbsfn_off[7];
  // srsran_ofdm_cfg_t options (ofdm.c:151-157, 228-230): every non-MBSFN symbol's DFT window starts `win` samples
  // into its cyclic prefix (rx_window_offset; the phase ramp it leaves is ofdm_rx_post's); dc0 = 1: the subcarriers
  // start at bin 0 (keep_dc, or a frequency shift), 0: the DC bin is skipped
  uint32_t      win;
  uint32_t      dc0;
  // int16 I/Q input (srsran_ofdm_rx_gpu_sc16): when set, sample n is (in16[n].x, in16[n].y) x in_scale, the
  // float product the host conversion of the radio's sc16 samples computes; `in` is then not read
  const short2* in16;
  float         in_scale;
  int           nstages;
  int           radix[OFDM_MAX_STAGES];
  uint32_t      ns_magic[OFDM_MAX_STAGES];  // ceil(2^32 / Ns) of every stage (j / Ns by __umulhi)
};

// grid: (2 nsymb, nrx, nsf) workgroups
hipError_t ofdm_rx_launch(const OfdmArgs& a, uint32_t nsf, hipStream_t stream);

// modulator: in = grid [sf][port][2 nsymb][nre], out = samples [sf][port][sf_len], nrx = ports, norm = scale;
// grid (2 nsymb, ports, nsf) workgroups
hipError_t ofdm_tx_launch(const OfdmArgs& a, uint32_t nsf, hipStream_t stream);

// rx_window_offset's phase ramp and phase compensation on the receiver's grids (ofdm_rx_slot, ofdm.c:491-512):
// grid [rows][nre], row = (sf x nrx) x 2 nsymb + sym; x *= wo[bin(k)] (wo: N entries, nullptr = none), then
// x *= ph[sym] (ph: 2 nsymb entries, the conjugate compensation phasors, nullptr = none); mbsfn: slot 0's rows
// (ofdm_rx_slot_mbsfn, neither applied) untouched
hipError_t ofdm_rx_post_launch(float2* grid, uint32_t rows, const OfdmArgs& a, const float2* wo, const float2* ph,
                               hipStream_t stream);
// the modulator's phase compensation and frequency shift on its samples (ofdm_tx_slot / srsran_ofdm_tx_sf,
// ofdm.c:625-636, 687-689): out [rows][sf_len], x *= ph[symbol of n] (cyclic prefix included: it is copied after the
// product), then x *= shift[n] (sf_len entries); either nullptr = none
hipError_t ofdm_tx_post_launch(float2* out, uint32_t rows, const OfdmArgs& a, const float2* ph, const float2* shift,
                               hipStream_t stream);

// factor N into radices 8/4/3/2 (largest first); returns the number of stages or -1
int ofdm_plan(uint32_t N, int* radix);
int ofdm_plan(uint32_t N, int* radix, uint32_t* ns_magic);

// srsran_vec_apply_cfo (vector_simd.c:1723-1774, the AVX2 + FMA build srsUE runs) as a phasor table: tab[n] is
// the phase the reference multiplies sample n by -- 8 lane phases 1, w, w^2 .. w^7 advanced by w^8 once per
// 8 samples, then a scalar tail advanced by w -- every product rounded as the reference's FMA sequence.
// (c, s) = sincosf(2 pi f) computed on the host by cfo_phasor (the reference's cexpf(I * TWOPI * cfo)).
void       cfo_phasor(float f, float* c, float* s);
hipError_t cfo_table_launch(float c, float s, float2* tab, uint32_t len, hipStream_t stream);
// standalone srsran_cfo_correct: out[n] = in[n] * tab[n] with the reference's complex product
hipError_t cfo_launch(const float2* in, float2* out, const float2* tab, uint32_t n, hipStream_t stream);

}  // namespace srsran_amd
#endif
