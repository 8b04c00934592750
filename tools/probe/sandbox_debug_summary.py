import sys,json,statistics as S
rows=[]
for l in sys.stdin:
    if not l.startswith('{'): continue
    d=json.loads(l); st=[x for x in d['debug'] if x.startswith('STAMPS')]
    s=json.loads(st[0][7:]) if st else {}
    t=d['timings']; rows.append((s,t))
for name,sel in (("prefaulted",lambda s:s.get('cow_prefault_pages',0)>0),("plain",lambda s:s.get('cow_prefault_pages',0)==0)):
    g=[(s,t) for s,t in rows if sel(s)]
    if not g: continue
    m=lambda f:round(S.median([f(s,t) for s,t in g]),3)
    print(name,len(g),'pool_cpu',m(lambda s,t:s.get('cpu_pool_ms',0)),'pool_flt',m(lambda s,t:s.get('minflt_pool',0)),'w_cpu',m(lambda s,t:t.get('w_cpu',0)),'w_flt',m(lambda s,t:t.get('w_minflt',0)),'run',m(lambda s,t:t.get('run',0)),'script',m(lambda s,t:t.get('w_script',0)),'setup',m(lambda s,t:t.get('w_setup',0)),'svc',m(lambda s,t:t.get('service_total',0)),'pf_pages',m(lambda s,t:s.get('cow_prefault_pages',0)),'pf_ms',m(lambda s,t:s.get('cow_prefault_ms',0)))
for s,t in rows:
    if 'cow_learned_pages' in s: print('learner', {k:v for k,v in s.items() if k.startswith('cow_')})
