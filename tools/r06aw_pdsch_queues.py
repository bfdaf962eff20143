"""PDSCH batch workers (bench.run_pdsch, 3 workers on streams of their own) on HIP's shared hardware queues vs on
streams with a hardware queue each (CU-masked, every CU): is the chain's step spread queue sharing?"""
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


def pdsch(tag, steps):
    args.worker_queues = tag
    r = bench.run_pdsch(args, torch, dist, 1, 0, dev, steps=steps, warmup=2, cpu_seconds=0, emit=False)
    print(json.dumps({"case": tag, "steps": steps, "sf_per_s": r["config"]["subframes_per_s"], "ms": r["ms_per_step"],
                      "gpu_ms": r["step_spread"]["gpu_ms"]}), flush=True)


# A/B in one process through bench --worker-queues (the default line times 20 steps)
for rep in range(3):
    for tag in ("shared", "own"):
        for steps in (20, 60):
            pdsch(tag, steps)
