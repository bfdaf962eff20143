"""Summarise tools/pmc.sh passes: per-kernel average counters per dispatch, and HBM traffic per
launch corrected as MI355X_MICROARCH.md prescribes (FETCH_SIZE x 2 on gfx950, WRITE_SIZE as is;
both in KiB).  Per kernel the MEDIAN over its dispatches: a workload that also launches the kernel with other
settings (the default line's 16-half-iteration launches, warm-up) does not shift the figure.  Usage: python tools/pmc_summary.py gpurun_out/pmc_X WORKLOAD out.json"""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def short(name):
    """kernel name as bench.py / srsran_tdec_gpu_last_kernel report it: no argument list, no namespace"""
    n = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    head, sep, tail = n.partition("<")
    return head.split("::")[-1] + sep + tail


def main(d, workload, out):
    # per kernel and grid size: a call that launches one kernel twice with different grids (the all-188 step's
    # 16-step part cut at SRSRAN_AMD_TDEC_MIDCUT) is reported as the SUM of its launches' medians, per call
    acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(list)))
    for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][int(r.get("Grid_Size") or 0)][r["Counter_Name"]].append(
                float(r["Counter_Value"]))
    kernels = {}
    for k, grids in acc.items():
        if "rocclr" in k or "at::native" in k:
            continue
        parts = {}
        for g, cs in grids.items():
            avg = {c: statistics.median(v) for c, v in cs.items()}
            if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
                avg["hbm_bytes_per_launch"] = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
            parts[g] = avg
        tot = collections.defaultdict(float)
        for avg in parts.values():
            for c, v in avg.items():
                tot[c] += v
        kernels[k] = {c: round(v, 1) for c, v in tot.items()}
        if len(parts) > 1:
            kernels[k]["launches_per_call"] = len(parts)
            kernels[k]["parts_by_grid"] = {str(g): {c: round(v, 1) for c, v in a.items()} for g, a in parts.items()}
    json.dump({"workload": workload, "source": d, "kernels": kernels}, open(out, "w"), indent=1)
    print(json.dumps({k: v.get("hbm_bytes_per_launch") for k, v in kernels.items()}))


if __name__ == "__main__":
    main(*sys.argv[1:4])
