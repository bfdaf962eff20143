# all-188 step: the 8-step part's upper K (--w8-fused-max-k) around 1536, with the mid cut; default repeated
set -o pipefail
A="--steps 30 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0"
bash tools/gpu_run.sh r06v bench:warm:"--steps 10 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0" bench:def1:"$A" bench:w1536a:"$A --w8-fused-max-k 1536" \
  bench:w1024:"$A --w8-fused-max-k 1024" bench:w1792:"$A --w8-fused-max-k 1792" \
  benche:w1536m2560:SRSRAN_AMD_TDEC_MIDCUT=2560:"$A --w8-fused-max-k 1536" benche:w1536m3584:SRSRAN_AMD_TDEC_MIDCUT=3584:"$A --w8-fused-max-k 1536" \
  bench:def2:"$A" bench:w1536b:"$A --w8-fused-max-k 1536"
