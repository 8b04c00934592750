"""Summarise a rocprofv3 SQLite output (rocpd schema) into small CSVs for
profiles/: per-kernel call count / mean / min duration, and per-kernel mean
PMC counter values when counters were collected, and per-range call count /
mean duration of roctx ranges when markers were traced (--marker-trace), and per-call
host time of runtime API calls when traced (--hip-runtime-trace).

    python tools/rocpd_summary.py gpurun_out/prof/xxx_results.db profiles/name
"""

import csv
import sqlite3
import sys


def short(name: str, n: int = 110) -> str:
    return name if len(name) <= n else name[: n - 3] + "..."


def main():
    db, prefix = sys.argv[1], sys.argv[2]
    con = sqlite3.connect(db)
    cur = con.cursor()
    rows = list(cur.execute(
        "select name, count(*), avg(end - start), min(end - start) from kernels group by name "
        "order by sum(end - start) desc"))
    if rows:
        with open(prefix + "_kernels.csv", "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "calls", "mean_us", "min_us"])
            for name, n, avg, mn in rows:
                w.writerow([short(name), n, round(avg / 1e3, 2), round(mn / 1e3, 2)])
    try:
        pm = list(cur.execute(
            "select kernel_name, counter_name, avg(value), count(*) from counters_collection "
            "group by kernel_name, counter_name order by kernel_name"))
    except sqlite3.Error:
        pm = []
    if pm:
        with open(prefix + "_counters.csv", "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "counter", "mean_value", "dispatches"])
            for name, c, v, n in pm:
                w.writerow([short(name), c, v, n])
    # roctx ranges (--marker-trace): the kernel broker's per-op ranges
    try:
        rg = list(cur.execute(
            "select json_extract(extdata, '$.message') as m, count(*), avg(end - start), min(end - start), "
            "sum(end - start) from regions where category like 'MARKER%' group by m order by sum(end - start) desc"))
    except sqlite3.Error:
        rg = []
    if rg:
        with open(prefix + "_ranges.csv", "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["range", "calls", "mean_us", "min_us", "total_ms"])
            for m, n, avg, mn, tot in rg:
                w.writerow([m, n, round(avg / 1e3, 2), round(mn / 1e3, 2), round(tot / 1e6, 2)])
    # runtime API calls (--hip-runtime-trace / --hsa-*-trace): host time per call
    try:
        api = list(cur.execute(
            "select category, name, count(*), avg(end - start), sum(end - start) from regions "
            "where category not like 'MARKER%' group by category, name order by sum(end - start) desc"))
    except sqlite3.Error:
        api = []
    if api:
        with open(prefix + "_api.csv", "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["category", "api", "calls", "mean_us", "total_ms"])
            for cat, name, n, avg, tot in api:
                w.writerow([cat, name, n, round(avg / 1e3, 2), round(tot / 1e6, 2)])
    print(f"{len(rows)} kernels, {len(pm)} counter rows, {len(rg)} ranges, {len(api)} api rows -> {prefix}_*.csv")


if __name__ == "__main__":
    main()
