#!/bin/bash
# Timing ablations of tdec16_kernel.hip (rebuilds the library with -DT16_ABL=N on the box, runs the
# k6144 bench; outputs are wrong by construction).  Usage: tools/ablate16.sh TAG "1 2 4 7"
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for A in $1; do
  make -C srsran_4g_amd/csrc -j16 -B ../lib/tdec16_kernel.o CXXFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -DT16_ABL=$A" > $OUT/build$A.log 2>&1 && make -C srsran_4g_amd/csrc >> $OUT/build$A.log 2>&1 || exit 1
  timeout -k 10 120 python bench.py --workload k6144 --steps 10 --warmup 2 --cpu-seconds 0 > $OUT/k$A.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/k$A.json'));print('abl $A', d['value'], d['roofline']['avg_launch_ms'])"
done
