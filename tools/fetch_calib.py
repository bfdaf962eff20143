"""Summarise tools/fetch_calib.hip under rocprofv3 (developer tool): FETCH_SIZE and WRITE_SIZE per launch
against the bytes each launch moves, per access width.

  python tools/fetch_calib.py OUT_DIR   (OUT_DIR: fetch.log / write.log = the program's stdout of the two
                                         passes, pf/ and pw/ = their rocprofv3 --pmc output)
-> OUT_DIR/calibration.json: per (op, width, passes) the counter in bytes, the true bytes and the factor
   true / counter by which a counter reading of that access pattern is multiplied."""
import csv
import glob
import json
import os
import sys


def dispatches(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and ("read_kernel" in r["Kernel_Name"] or "write_kernel" in r["Kernel_Name"]):
                rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    return [v for _, v in sorted(rows)]


def main(d):
    res = []
    for counter, log, sub, op in (("FETCH_SIZE", "fetch.log", "pf", "read"), ("WRITE_SIZE", "write.log", "pw", "write")):
        launches = [json.loads(l) for l in open(os.path.join(d, log)) if l.startswith("{")]
        vals = dispatches(os.path.join(d, sub), counter)
        assert len(vals) == len(launches), (counter, len(vals), len(launches))
        for L, v in zip(launches, vals):
            if L["op"] != op:
                continue
            got = v * 1024  # KiB
            res.append(dict(L, counter=counter, counter_bytes=int(got), factor=round(L["bytes"] / got, 3) if got else None))
    json.dump({"_doc": __doc__.split("\n\n")[0], "source": d, "launches": res}, open(os.path.join(d, "calibration.json"), "w"),
              indent=1)
    for r in res:
        print(r)


if __name__ == "__main__":
    main(sys.argv[1])
