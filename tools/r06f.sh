set -o pipefail
A="--steps 10 --warmup 3 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0"
bash tools/gpu_run.sh r06f \
 "benche:m0a:SRSRAN_AMD_TDEC_MIDCUT=0:$A" \
 "benche:m3072a:SRSRAN_AMD_TDEC_MIDCUT=3072:$A" \
 "benche:m0b:SRSRAN_AMD_TDEC_MIDCUT=0:$A" \
 "benche:m3072b:SRSRAN_AMD_TDEC_MIDCUT=3072:$A" \
 "benche:m4096:SRSRAN_AMD_TDEC_MIDCUT=4096:$A" \
 "benche:m2560:SRSRAN_AMD_TDEC_MIDCUT=2560:$A" \
 "benche:m3072nogate:SRSRAN_AMD_TDEC_MIDCUT=3072,SRSRAN_AMD_TDEC_GATE=0:$A" \
 "benche:m5120:SRSRAN_AMD_TDEC_MIDCUT=5120:$A"
