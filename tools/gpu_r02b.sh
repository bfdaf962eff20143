set -o pipefail
export TMPDIR=/tmp
bash tools/pmc.sh r02_pmc_all188 all188 --pdsch-steps 0 || exit 1
python tools/pmc_summary.py gpurun_out/r02_pmc_all188 all188 gpurun_out/r02_pmc_all188/summary.json || exit 1
SRSRAN_TDEC16_MIN_CB=1000 timeout -k 10 200 python bench.py --workload pdsch --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/r02_pdsch_t16.json 2>gpurun_out/r02_pdsch_t16.err || exit 1
timeout -k 10 200 python bench.py --workload pdsch --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/r02_pdsch_q.json 2>gpurun_out/r02_pdsch_q.err || exit 1
python - <<'PY'
import json
for f in ("r02_pdsch_t16","r02_pdsch_q"):
    d=json.load(open(f"gpurun_out/{f}.json")); print(f, d["value"], d["roofline"]["avg_launch_ms"])
PY
