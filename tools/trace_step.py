"""Timeline of the decoder launches of one bench step from a rocprofv3 --kernel-trace CSV (developer tool):
  python tools/trace_step.py <kernel_trace.csv> [PATTERN] [STEP_FROM_END]
prints, for the STEP_FROM_END-th last group of multi-kernel dispatches (default 2: the last full timed step), each
dispatch's kernel, start and end in ms from the group's first start, and the group's span."""
import csv
import sys


def main(path, pat="tdec", back=2):
    rows = [r for r in csv.DictReader(open(path)) if pat in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # group dispatches into steps: a new step starts after a gap of > 0.5 ms with nothing running
    steps, cur, end = [], [], 0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if cur and s > end + 500_000:
            steps.append(cur)
            cur = []
        cur.append(r)
        end = max(end, e) if cur[:-1] else e
    if cur:
        steps.append(cur)
    st = steps[-int(back)] if len(steps) >= int(back) else steps[-1]
    t0 = min(int(r["Start_Timestamp"]) for r in st)
    t1 = max(int(r["End_Timestamp"]) for r in st)
    for r in st:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("::")[-1]
        print(f"{name:40s} grid {r.get('Grid_Size_X', r.get('Grid_Size', '?')):>8s} lds {r.get('LDS_Block_Size', r.get('Lds_Size', '?')):>6s}  "
              f"{(int(r['Start_Timestamp']) - t0) / 1e6:8.3f} -> {(int(r['End_Timestamp']) - t0) / 1e6:8.3f} ms")
    print(f"span {(t1 - t0) / 1e6:.3f} ms over {len(st)} dispatches ({len(steps)} groups)")


if __name__ == "__main__":
    main(*sys.argv[1:])
