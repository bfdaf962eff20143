# kernel trace of the C3 chain with its 3 workers (timeline analysis: decoder busy fraction, gaps)
set -o pipefail
bash tools/gpu_run.sh r06aa "prof:chain3:--workload pdsch --steps 30 --cpu-seconds 0"
