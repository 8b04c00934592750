"""Per-kernel means of rocprofv3 --pmc counters (its counter_collection.csv):
one row per kernel name (truncated), dispatches and the mean of every
counter per dispatch.

    python tools/probe/pmc_by_kernel.py DIR [DIR ...] [--match SUBSTR ...]
"""

import argparse
import collections
import csv
import glob
import os


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dirs", nargs="+")
    p.add_argument("--match", nargs="*", default=[])
    a = p.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r.get("Kernel_Name", "")
                if a.match and not any(m in name for m in a.match):
                    continue
                key = (name[:70], r.get("Dispatch_Id"))
                vals[name[:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, cs in sorted(vals.items()):
        cols = " ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items()))
        n = max(len(v) for v in cs.values())
        print(f"| {name} | {n} | {cols} |")


if __name__ == "__main__":
    main()
