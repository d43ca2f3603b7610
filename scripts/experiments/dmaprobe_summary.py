import json, collections, statistics, sys
d=collections.defaultdict(list); irq=collections.defaultdict(list)
for l in open(sys.argv[1]):
    r=json.loads(l)
    if r["rep"]==0: continue
    if "writer_irqs" in r: irq[r["variant"]].append(r["writer_irqs"]); continue
    d[r["variant"]].append((r["GB/s"], r["writer_cpu_s_per_gib"], r["wait_s_per_gib"]))
for k,v in d.items():
    print(f"  {k:12s} GB/s med {statistics.median(x[0] for x in v):6.2f} cpu/GiB {statistics.median(x[1] for x in v):.4f} wait {statistics.median(x[2] for x in v):.4f} {[x[0] for x in v]} irqs {irq[k]}")
