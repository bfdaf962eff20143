"""One-line digest of a bench.py JSON line (tools/gpu_run.sh)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
out = {k: d.get(k) for k in ("value", "unit", "n_gpus", "ms_per_step")}
out.update({"kernel": r.get("kernel"), "avg_launch_ms": r.get("avg_launch_ms"), "frac": r.get("frac")})
for k in ("pdsch_subframes_per_s", "k6144_mbps", "mbps_16_half_its"):
    if k in d:
        out[k] = d[k]
if "pdsch" in d:
    out["pdsch_ms"] = d["pdsch"].get("ms_per_step")
if "c1_cpu" in d:
    c = d["c1_cpu"]
    out["c1_cpu"] = {k: c.get(k) for k in ("cpu_1thread_mbps", "cpu_share_mbps", "cpu_host_estimate_mbps",
                                            "gpu_over_1thread", "gpu_over_share", "gpu_over_host_estimate")}
if "output_check" in d:
    out["mismatched"] = d["output_check"]["mismatched"]
print(json.dumps(out))
