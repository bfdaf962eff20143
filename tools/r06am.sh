# all-188 step: the generic class (K <= 400) on the single-lane decoder (tdec1s) instead of the quad one
set -o pipefail
A="--steps 30 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0"
bash tools/gpu_run.sh r06am bench:warm:"--steps 10 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0" bench:def1:"$A" \
  bench:g1s:"$A --generic-single-min-cb 0" bench:def2:"$A" bench:g1s2:"$A --generic-single-min-cb 0"
