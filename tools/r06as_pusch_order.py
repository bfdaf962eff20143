"""PUSCH worker rate vs what ran before it in the same process (the default line runs it after the
PDSCH legs): standalone, after pinned host buffers, after a PDSCH run; per-stage times of worker 0."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = ["bench.py", "--workload", "pusch", "--cpu-seconds", "0", "--pusch-workers", "2"]
import bench  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

args = bench.parse()
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)


def pusch(tag, nw=2):
    args.pusch_workers = nw
    r = bench.run_pusch(args, torch, dist, 1, 0, dev, steps=20, warmup=2, cpu_seconds=0, emit=False)
    st = {k: v["ms_per_step"] for k, v in r["stages"].items()}
    print(json.dumps({"case": tag, "workers": nw, "ue_sf_per_s": r["config"]["ue_subframes_per_s"],
                      "ms": r["ms_per_step"], "stages": st}), flush=True)


pusch("first")
pusch("first", 1)
pinned = [torch.from_numpy(np.zeros(10 << 20, np.float32)).pin_memory() for _ in range(6)]
pusch("after_pinned_240MB")
del pinned
bench.run_pdsch(args, torch, dist, 1, 0, dev, steps=20, warmup=2, cpu_seconds=0, emit=False)
pusch("after_pdsch")
pusch("after_pdsch", 1)
torch.cuda.synchronize()
torch.cuda.empty_cache()
pusch("after_pdsch_empty_cache")
