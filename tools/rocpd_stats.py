"""Kernel statistics from a rocprofv3 SQLite output (`run_results.db`, the default output format when
--output-format is not given):
  python tools/rocpd_stats.py <results.db> <out.csv>                  the columns of --stats' kernel_stats.csv
  python tools/rocpd_stats.py <results.db> <out.json> --dispatches PAT  every dispatch of the kernels whose
                                                                       name contains PAT, in launch order"""
import csv
import json
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    con = sqlite3.connect(db)
    if len(sys.argv) > 4 and sys.argv[3] == "--dispatches":
        rows = con.execute("select name, start, duration, grid_x, workgroup_x, lds_size, stream_id from kernels "
                           "where name like ? order by start", (f"%{sys.argv[4]}%",)).fetchall()
        t0 = rows[0][1] if rows else 0
        recs = [{"kernel": n, "start_ms": round((s - t0) / 1e6, 3), "duration_ms": round(d / 1e6, 4), "grid_x": gx,
                 "workgroup_x": wx, "lds_bytes": lds, "stream_id": sid} for n, s, d, gx, wx, lds, sid in rows]
        with open(out, "w") as f:
            json.dump(recs, f, indent=1)
        print(f"{len(recs)} dispatches -> {out}")
        return
    rows = con.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for name, calls, total, avg, pct in rows:
            # top_kernels reports microseconds
            w.writerow([name, calls, round(total * 1e3), round(avg * 1e3), round(pct, 4)])
    print(f"{len(rows)} kernels -> {out}")


if __name__ == "__main__":
    main()
