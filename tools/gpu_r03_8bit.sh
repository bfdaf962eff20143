#!/bin/bash
# round 3: the 8-bit turbo decoder on the GPU -- parity tests, then its C1-shape timing and a rocprof summary
set -o pipefail
OUT=gpurun_out/${R8OUT:-r03_8bit}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_tdec8bit.py -m gpu -v -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
cat > $OUT/b8.py <<'PY'
import json, os, sys
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
import torch, bench
print(json.dumps(bench.bench_8bit(torch, torch.device("cuda:0"), 1024)))
PY
timeout -k 10 300 python $OUT/b8.py > $OUT/b8.json 2> $OUT/b8.err || { tail -5 $OUT/b8.err; exit 1; }
cat $OUT/b8.json
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/$OUT/b8.py > $R/$OUT/b8_prof.json 2> $R/$OUT/b8_prof.err || { tail -5 $R/$OUT/b8_prof.err; exit 1; }
echo done
