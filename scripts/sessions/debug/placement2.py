"""Read-path placement x ring-geometry matrix on the GPU box (GPU sink, verify
on), repeated in interleaved rounds so run-to-run spread is visible."""
import itertools
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import custom_go_client_benchmark_amd as pkg  # noqa: E402
from custom_go_client_benchmark_amd.parallel import affinity  # noqa: E402

n = pkg._native
size = int(os.environ.get("SIZE", 256 << 20))
reads = int(os.environ.get("READS", 8))
rounds = int(os.environ.get("ROUNDS", 3))


def physical(cpus):
    """One logical CPU per physical core (drop SMT siblings)."""
    seen, out = set(), []
    for c in cpus:
        try:
            sib = open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
        except OSError:
            sib = str(c)
        if sib not in seen:
            seen.add(sib)
            out.append(c)
    return out


cpus = affinity.gpu_local_cpus(0)
groups = affinity.l3_groups(cpus)
pl = affinity.plan(0, "same")
g = pl["client"]
gi = next(i for i, x in enumerate(groups) if x[0] == g[0])
g2 = groups[(gi + 1) % len(groups)]
ph = physical(g)
placements = {
    "same16": (g, g),
    "l3split_phys": (ph[: len(ph) // 2], ph[len(ph) // 2:]),
    "l3split_smt": ([c for c in g if c not in ph[len(ph) // 2:]], ph[len(ph) // 2:]),
    "cross_l3": (g, g2),
}
print(json.dumps({k: v for k, v in placements.items()}), flush=True)
geoms = [(1 << 20, 8), (2 << 20, 8), (4 << 20, 4), (8 << 20, 4)]
res = {}
for rnd in range(rounds):
    for name, (ccpu, scpu) in placements.items():
        srv = n.Server({"port": 0, "md5": False, "cpus": scpu})
        srv.start()
        srv.add_synthetic("b", "o", "", 0, 1, size)
        for proto, (slot, nslots) in itertools.product(["grpc", "http"], geoms):
            run = n.Runner({"protocol": proto, "endpoint": srv.url, "bucket": "b", "object_prefix": "o", "workers": 1,
                            "reads_per_worker": 2, "sink": "gpu", "ring_slot_bytes": slot, "ring_slots": nslots,
                            "keep_records": False, "cpus": ccpu})
            run.start()
            run.wait()
            run.reset_stats()
            run.set_reads_per_worker(reads)
            run.start()
            run.wait()
            s = run.summary()
            key = f"{name}/{proto}/{slot >> 20}MiBx{nslots}"
            gbs = size / (s["p50_ms"] / 1e3) / 1e9
            res.setdefault(key, []).append(gbs)
            print(json.dumps({"round": rnd, "key": key, "p50_ms": round(s["p50_ms"], 2),
                              "GB/s@p50": round(gbs, 2), "errors": s["errors"]}), flush=True)
        srv.stop()
print("=== summary (GB/s at p50: median / min / max over rounds)")
for k, v in sorted(res.items(), key=lambda kv: -statistics.median(kv[1])):
    print(f"{k:40s} {statistics.median(v):6.2f} {min(v):6.2f} {max(v):6.2f}")
