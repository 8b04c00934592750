"""Instruction mix per kernel in a hipcc --save-temps .s file (GEMM lab)."""
import sys, re
s = open(sys.argv[1]).read().split('\n')
pat = sys.argv[2] if len(sys.argv) > 2 else 'w4'
cur = None; body = []
funcs = []
for l in s:
    m = re.match(r'^([_A-Za-z0-9]+):\s*(;.*)?$', l)
    if m and not l.startswith('.') and m.group(1).startswith('_Z'):
        cur = m.group(1); body = []
        continue
    if cur:
        if 's_endpgm' in l:
            funcs.append((cur, body)); cur = None
        else:
            body.append(l.strip())
for name, body in funcs:
    if pat not in name: continue
    ins = [l for l in body if l and not l.startswith(('.', ';')) and not l.endswith(':')]
    c = lambda p: sum(1 for l in ins if re.match(p, l))
    print(name[-40:], "insts", len(ins), "mfma", c(r'v_mfma'), "acc_rd", c(r'v_accvgpr_read'), "acc_wr", c(r'v_accvgpr_write'),
          "ds_read", c(r'ds_read'), "ds_write", c(r'ds_write'), "glds", c(r'global_load_lds|buffer_load.*lds'), "scratch", c(r'scratch_'), "waitcnt", c(r's_waitcnt'), "barrier", c(r's_barrier'), "waterfall_loops", sum(1 for l in body if 'Inner Loop Header' in l))
