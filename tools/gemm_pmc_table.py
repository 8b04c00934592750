"""Per-wave, per-K-tile cycle table of GEMM kernels from rocprofv3 PMC runs
(rocpd SQLite output of ``rocprofv3 --kernel-trace --pmc ...``):

    python tools/gemm_pmc_table.py SIZE NAME=gpurun_out/dir [NAME=dir ...]

Counters expected: GRBM_GUI_ACTIVE, SQ_WAVES, SQ_WAVE_CYCLES, SQ_WAIT_ANY,
SQ_WAIT_INST_ANY (SQ_WAIT_INST_LDS, SQ_VALU_MFMA_BUSY_CYCLES if present).
SQ_* wave counters count quad-cycles (MI355X_MICROARCH.md); the effective
clock is GRBM_GUI_ACTIVE / 8 XCDs / kernel time.  Prints a markdown table.
"""

import glob
import os
import sqlite3
import sys


def load(d):
    db = sorted(glob.glob(os.path.join(d, "**", "*results.db"), recursive=True))
    if not db:
        return None
    con = sqlite3.connect(db[0])
    cur = con.cursor()
    gemm = lambda k: "gemm" in k or "Cijk" in k  # noqa: E731
    vals = {c: v for k, c, v in cur.execute(
        "select kernel_name, counter_name, avg(value) from counters_collection group by kernel_name, counter_name")
        if gemm(k)}
    durs = [x for k, x in cur.execute("select name, avg(end - start) from kernels group by name") if gemm(k)]
    return (vals, durs[0]) if vals and durs else None


def main():
    size = int(sys.argv[1])
    ktiles = size // 64
    print("| kernel | us | GHz | wave cycles / K-tile | SQ_WAIT_ANY | SQ_WAIT_INST_ANY | SQ_WAIT_INST_LDS | MFMA busy |")
    print("|---|---|---|---|---|---|---|---|")
    for arg in sys.argv[2:]:
        name, d = arg.split("=", 1)
        r = load(d)
        if r is None:
            print(f"| {name} | (no data) | | | | | | |")
            continue
        v, dur = r
        waves = v["SQ_WAVES"]
        per = lambda c: v[c] * 4 / waves / ktiles if c in v else float("nan")  # noqa: E731
        ghz = v["GRBM_GUI_ACTIVE"] / 8 / dur
        busy = v.get("SQ_VALU_MFMA_BUSY_CYCLES", float("nan")) / (v["GRBM_GUI_ACTIVE"] / 8 * 256 * 4)
        print(f"| {name} | {dur / 1e3:.1f} | {ghz:.2f} | {per('SQ_WAVE_CYCLES'):.0f} | {per('SQ_WAIT_ANY'):.0f} | "
              f"{per('SQ_WAIT_INST_ANY'):.0f} | {per('SQ_WAIT_INST_LDS'):.0f} | {busy:.3f} |")


if __name__ == "__main__":
    main()
