#!/bin/bash
# round 3: split variant parity + timing, PCIe loop probe, bench-workload PMC passes
set -o pipefail
bash tools/gpu_r03h.sh || exit 1
mkdir -p gpurun_out/r03g
timeout -k 10 240 python tools/h2d_probe.py > gpurun_out/r03g/h2d_probe.jsonl 2> gpurun_out/r03g/h2d_probe.err || { tail -5 gpurun_out/r03g/h2d_probe.err; exit 1; }
cat gpurun_out/r03g/h2d_probe.jsonl
bash tools/gpu_pmc_bench_r03.sh
