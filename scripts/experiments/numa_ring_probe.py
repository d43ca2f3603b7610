#!/usr/bin/env python3
"""Where do the pinned ring slots land?  Creates GpuSinks from a thread pinned
to the GPU's NUMA node (as the bench's worker is) and prints each slot's pages
by node, for both ring allocators (GCSB_RING_ALLOC is read once per process:
run the script once per value)."""
import json
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import custom_go_client_benchmark_amd as pkg  # noqa: E402
from custom_go_client_benchmark_amd.parallel import affinity  # noqa: E402

n = pkg._native
plan = affinity.plan(0, "pair")
out = {}


def work():
    n.pin_current_thread(plan["client"])
    out["node_of_thread"] = n.current_numa_node()
    sinks = [n.GpuSink({"device": 0, "ring_slot_bytes": 2 << 20, "ring_slots": 8}) for _ in range(3)]
    out["slots"] = [[{str(i): c for i, c in enumerate(k[:-1]) if c} | ({"absent": k[-1]} if k[-1] else {})
                     for k in s.ring_numa()] for s in sinks]


t = threading.Thread(target=work)
t.start()
t.join()
print(json.dumps({"alloc": os.environ.get("GCSB_RING_ALLOC", "default"), "gpu_node": affinity.gpu_numa_node(0),
                  "client": plan["client"], **out}))
