# experiment: the 16-sub-block mid part on a build with registers for two waves a SIMD (SRSRAN_AMD_TDEC_MID_O2=1)
set -o pipefail
A="--steps 30 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0"
bash tools/gpu_run.sh r06z \
  bench:warm:"--steps 10 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0" bench:def1:"$A" \
  benche:o2:SRSRAN_AMD_TDEC_MID_O2=1:"$A" benche:o2m4096:SRSRAN_AMD_TDEC_MID_O2=1,SRSRAN_AMD_TDEC_MIDCUT=4096:"$A" \
  benche:o2w2048:SRSRAN_AMD_TDEC_MID_O2=1:"$A --w8-fused-max-k 2048" bench:def2:"$A"
