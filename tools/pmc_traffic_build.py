"""Build profiles/pmc_traffic.json (bench.py's roofline.traffic table) from the committed PMC summaries
of the given rounds (tools/pmc_summary.py output copied to profiles/<round>_pmc_<workload>.json); per
workload the first round listed that has a summary wins.

  python tools/pmc_traffic_build.py r04,r03

Per workload and kernel: bytes = HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, KiB -> bytes),
units = the work items of that launch in the profiled run (bench.py scales by its own count),
valu_insts = SQ_INSTS_VALU of the launch, source = the summary file."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# work items per launch of the profiled runs (tools/pmc.sh: bench defaults; tools/pmc_tdec.sh: 1024 a size)
UNITS = {
    "all188": 1024 * 110,  # the 16-sub-block class of the fused launch: 110 sizes x 1024 blocks
    "k6144": 1024,
    "class8": 1024 * 32,
    "dlsch": 156 * 13,     # 78 subframes x 2 TBs x 13 code blocks
    "ulsch": 156 * 13,
    "pdsch": 78 * 26,
    "pusch": 78,           # UEs
    "ldpc": 4096,          # codewords
    "nrsch": 64 * 35,      # code blocks
}

DOC = ("HBM bytes per launch from rocprofv3 PMC (tools/pmc.sh / tools/pmc_tdec.sh -> tools/pmc_summary.py -> "
       "tools/pmc_traffic_build.py): 2 x FETCH_SIZE + WRITE_SIZE.  The x 2 is calibrated on this hardware for "
       "the access widths these kernels use (profiles/r03_fetch_calibration.json, tools/fetch_calib.hip: coalesced "
       "reads of 2, 4, 8 and 16 bytes a lane over 1 GiB all read back as FETCH_SIZE = bytes / 2; WRITE_SIZE = "
       "bytes for every width; re-reads of a 64 MiB slice held in the Infinity Cache are NOT counted, so the "
       "figure is DRAM traffic).  units = work items of the measured launch; bench.py scales by its own batch.  "
       "valu_insts = SQ_INSTS_VALU of the same launch (roofline.valu_issue_frac).")


def all188_units(cut):
    """blocks per launch of the two parts of the 16-sub-block class in tools/tdec_kernels.py's all-188
    workload (1024 a size), cut at srsran_tdec_gpu_get_w8_fused_max_k = `cut`"""
    sys.path.insert(0, ROOT)
    from oracle.oracle import CB_SIZES, nof_subblocks
    k16 = [k for k in CB_SIZES if nof_subblocks(k) == 16]
    return {"tdec16s_multi_kernel": 1024 * sum(1 for k in k16 if k > cut),
            "tdec16sw8_multi_kernel": 1024 * sum(1 for k in k16 if k <= cut),
            "tdec8sw8_multi_kernel": 1024 * sum(1 for k in CB_SIZES if nof_subblocks(k) == 8),
            "tdec_multi_kernel<1>": 1024 * sum(1 for k in CB_SIZES if nof_subblocks(k) == 0)}  # generic: no sub-blocks


def main(rounds, cut=2048):
    out = {"_doc": DOC}
    for wl, units in UNITS.items():
        found = [f"profiles/{r}_pmc_{wl}.json" for r in rounds.split(",")
                 if os.path.exists(os.path.join(ROOT, f"profiles/{r}_pmc_{wl}.json"))]
        if not found:
            continue
        src = found[0]
        path = os.path.join(ROOT, src)
        ks = json.load(open(path))["kernels"]
        ent = {}
        for k, c in ks.items():
            head, sep, tail = k.partition("<")
            k = head.split("::")[-1] + sep + tail  # as bench.py names kernels (no namespace)
            if "hbm_bytes_per_launch" not in c:
                continue
            if wl == "all188" and "multi_kernel" not in k:
                continue  # the default line's other launches (C1, 8-bit, PDSCH / PUSCH): their own workloads
            u = all188_units(cut).get(k, units) if wl == "all188" and len(ks) > 1 else units
            e = {"bytes": int(c["hbm_bytes_per_launch"]), "fetch_raw_kib": c.get("FETCH_SIZE"), "units": u,
                 "source": src}
            if "SQ_INSTS_VALU" in c:
                e["valu_insts"] = int(c["SQ_INSTS_VALU"])
            ent[k] = e
        if wl == "all188" and {"tdec16s_multi_kernel", "tdec16sw8_multi_kernel"} <= set(ent):
            # the 16-sub-block class as bench.py times it: both parts, launched concurrently
            a, b = ent["tdec16s_multi_kernel"], ent["tdec16sw8_multi_kernel"]
            ent["tdec16s_multi_kernel+tdec16sw8_multi_kernel"] = {
                "bytes": a["bytes"] + b["bytes"], "units": a["units"] + b["units"], "source": src,
                "valu_insts": a.get("valu_insts", 0) + b.get("valu_insts", 0), "cut_k": cut}
        out[wl] = ent
    json.dump(out, open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w"), indent=1)
    print({wl: sorted(v) for wl, v in out.items() if wl != "_doc"})


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r03", int(sys.argv[2]) if len(sys.argv) > 2 else 2048)
