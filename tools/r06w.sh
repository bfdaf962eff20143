# PMC traffic of the round-6 schedule: the all-188 16-sub-block class (three launches: K > 3072, 1536 < K <= 3072,
# K <= 1536 on 8-step windows), C1, and the C3 chain
set -o pipefail
bash tools/gpu_run.sh r06w "pmc:all188:--workload all188 --launches 3" "pmc:k6144:--workload k6144 --launches 3" \
  "pmcb:pdsch:pdsch --pdsch-workers 1"
