"""PDSCH batch workers 3 against 4 (R06BB_WORKERS: other counts; own hardware queues), alternated in one process,
60 timed steps each."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = ["bench.py", "--workload", "pdsch", "--cpu-seconds", "0"]
import bench  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

args = bench.parse()
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
for rep in range(3):
    for nw in tuple(int(x) for x in os.environ.get("R06BB_WORKERS", "3,4").split(",")):
        args.pdsch_workers = nw
        r = bench.run_pdsch(args, torch, dist, 1, 0, dev, steps=60, warmup=2, cpu_seconds=0, emit=False)
        print(json.dumps({"workers": nw, "sf_per_s": r["config"]["subframes_per_s"], "ms": r["ms_per_step"]}),
              flush=True)
