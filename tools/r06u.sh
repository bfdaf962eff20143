# all-188 step against the 16-step part's mid cut (SRSRAN_AMD_TDEC_MIDCUT) and the 8-step part's upper K
set -o pipefail
A="--steps 30 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0"
bash tools/gpu_run.sh r06u bench:m3072:"$A" benche:m2560:SRSRAN_AMD_TDEC_MIDCUT=2560:"$A" \
  benche:m3584:SRSRAN_AMD_TDEC_MIDCUT=3584:"$A" benche:m4096:SRSRAN_AMD_TDEC_MIDCUT=4096:"$A" \
  bench:w1536:"$A --w8-fused-max-k 1536" bench:w2560:"$A --w8-fused-max-k 2560" bench:m3072b:"$A"
