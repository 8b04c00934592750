"""Tabulate tools/gemm_fp_sweep.sh output: per dtype / shape, each variant's
median us, ratio to torch.matmul, error and race screen.

    python tools/sweep_table.py gpurun_out/gemm_fp_sweep.jsonl
"""
import json
import sys
from collections import defaultdict

rows = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
by = defaultdict(list)
for r in rows:
    by[(r["dtype"], r["shape"], r.get("ta"), r.get("tb"))].append(r)
for (dt, shape, ta, tb), rs in by.items():
    print(f"{dt} {shape}{' ta' if ta else ''}{' tb' if tb else ''}")
    for r in rs:
        print(f"   {r.get('label', '-'):>10}  bk {r['beekern_us_median']:8.1f} us  torch {r['torch_us_median']:8.1f}"
              f"  ratio {r['ratio_median']:.3f}  err {r['max_rel_err_beekern']:.1e}  racy {r['racy_repeats']}")
