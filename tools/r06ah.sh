# the mid part (1536 < K <= 3072) as a persistent grid of 2 (or 1, 3) workgroups a CU: the all-188 step
set -o pipefail
A="--steps 30 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0"
bash tools/gpu_run.sh r06ah bench:warm:"--steps 10 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0" bench:def1:"$A" \
  benche:p2:SRSRAN_AMD_TDEC_MID_PERSIST=2:"$A" benche:p1:SRSRAN_AMD_TDEC_MID_PERSIST=1:"$A" bench:def2:"$A" \
  benche:p2b:SRSRAN_AMD_TDEC_MID_PERSIST=2:"$A" benche:p3:SRSRAN_AMD_TDEC_MID_PERSIST=3:"$A"
