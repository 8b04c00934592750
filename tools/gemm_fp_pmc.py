"""Table of the f64 / f32 GEMM counter passes (tools/gemm_fp_pmc.sh):
per-wave cycles by state, MFMA busy share, instruction mix -- beekern's
kernel against torch.matmul's on the same operands.

    python tools/gemm_fp_pmc.py gpurun_out DTYPE SIZE
"""

import glob
import os
import sqlite3
import sys


def load(d):
    dbs = sorted(glob.glob(os.path.join(d, "**", "*results.db"), recursive=True))
    out, dur = {}, None
    for db in dbs:
        con = sqlite3.connect(db)
        cur = con.cursor()
        rows = list(cur.execute("select kernel_name, counter_name, avg(value) from counters_collection "
                                "group by kernel_name, counter_name"))
        # the GEMM: the kernel with the most wave cycles (torch's fills are tiny)
        by_k = {}
        for k, c, v in rows:
            by_k.setdefault(k, {})[c] = v
        if not by_k:
            continue
        k = max(by_k, key=lambda n: by_k[n].get("SQ_WAVE_CYCLES", by_k[n].get("GRBM_GUI_ACTIVE", 0)))
        out.update(by_k[k])
        durs = {n: x for n, x in cur.execute("select name, avg(end - start) from kernels group by name")}
        dur = durs.get(k, dur)
        out["_kernel"] = k
    return out, dur


def main():
    root, dt, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    impls = sys.argv[4:] or ["bk", "torch"]
    print("| impl | kernel | us | GHz | wave cyc | busy | wait_any | wait_inst | wait_lds | MFMA busy | VALU insts/wave "
          "| LDS insts/wave | LDS bank-conflict / active | VMEM insts/wave |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|---|---|")
    mem = []
    for impl in impls:
        v, dur = {}, None
        for p in (1, 2, 3, 4):
            d = os.path.join(root, f"pmc_{dt}_{n}_{impl}_{p}")
            if not os.path.isdir(d):
                continue
            a, du = load(d)
            v.update(a)
            dur = dur or du
        if not v or not dur:
            print(f"| {impl} | (no data) |")
            continue
        waves = v.get("SQ_WAVES", 1)
        nan = float("nan")
        q = lambda c: v.get(c, nan) * 4 / waves  # noqa: E731  (quad-cycles -> cycles per wave)
        clk = v["GRBM_GUI_ACTIVE"] / 8
        busy = v.get("SQ_VALU_MFMA_BUSY_CYCLES", nan) / (clk * 256 * 4)
        conf = v.get("SQ_LDS_BANK_CONFLICT", nan) / v.get("SQ_LDS_IDX_ACTIVE", nan)
        print(f"| {impl} | {v['_kernel'][:48]} | {dur / 1e3:.1f} | {clk / dur:.2f} | {q('SQ_WAVE_CYCLES'):.0f} | "
              f"{q('SQ_BUSY_CYCLES'):.0f} | {q('SQ_WAIT_ANY'):.0f} | {q('SQ_WAIT_INST_ANY'):.0f} | "
              f"{q('SQ_WAIT_INST_LDS'):.0f} | {busy:.3f} | {v.get('SQ_INSTS_VALU', nan) / waves:.0f} | "
              f"{v.get('SQ_INSTS_LDS', nan) / waves:.0f} | {conf:.3f} | {v.get('SQ_INSTS_VMEM', nan) / waves:.0f} |")
        if "TCC_HIT_sum" in v:
            hit = v["TCC_HIT_sum"] / max(1.0, v["TCC_HIT_sum"] + v.get("TCC_MISS_sum", 0))
            lat = v.get("SQ_INST_LEVEL_VMEM", nan) / max(1.0, v.get("SQ_INSTS_VMEM_RD", nan))
            mem.append(f"| {impl} | L2 hit {hit:.3f} | EA read req {v.get('TCC_EA0_RDREQ_sum', nan):.3e} | "
                       f"VMEM level/read {lat:.1f} | TA busy {v.get('TA_BUSY_avr', nan):.3e} |")


    if mem:
        print()
        print("| impl | L2 | HBM | VMEM latency (level / reads) | TA |")
        print("|---|---|---|---|---|")
        print("\n".join(mem))


if __name__ == "__main__":
    main()
