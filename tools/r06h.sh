set -o pipefail
A="--steps 10 --warmup 3 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0"
bash tools/gpu_run.sh r06h \
 "benche:m3072a:SRSRAN_AMD_TDEC_MIDCUT=3072:$A" \
 "benche:m3328:SRSRAN_AMD_TDEC_MIDCUT=3328:$A" \
 "benche:m3584:SRSRAN_AMD_TDEC_MIDCUT=3584:$A" \
 "benche:m2816:SRSRAN_AMD_TDEC_MIDCUT=2816:$A" \
 "benche:m3072q8:SRSRAN_AMD_TDEC_MIDCUT=3072,GPU_MAX_HW_QUEUES=8:$A" \
 "benche:m3072b:SRSRAN_AMD_TDEC_MIDCUT=3072:$A"
