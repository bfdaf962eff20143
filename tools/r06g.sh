set -o pipefail
A="--steps 4 --warmup 2 --cpu-seconds 0 --pdsch-steps 0 --pdsch-low-snr 0"
bash tools/gpu_run.sh r06g "prof:mid3072:$A" && python tools/trace_step.py gpurun_out/r06g/prof_mid3072/run_kernel_trace.csv tdec
