"""Read-path matrix on the GPU box: placement x protocol (GPU sink, verify on)."""
import sys, os, time, json, itertools
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import custom_go_client_benchmark_amd as pkg
from custom_go_client_benchmark_amd.parallel import affinity
n = pkg._native
size = int(os.environ.get("SIZE", 256 << 20))
reads = int(os.environ.get("READS", 10))
print(affinity.visible_gpu_summary())
for mode in ["none", "same", "split", "numa"]:
    pl = affinity.plan(0, mode)
    print("plan", json.dumps(pl))
    srv = n.Server({"port": 0, "md5": False, "cpus": pl["server"]})
    srv.start()
    srv.add_synthetic("b", "o", "", 0, 1, size)
    for proto, slot in itertools.product(["http", "grpc"], [4 << 20, 8 << 20, 16 << 20]):
        run = n.Runner({"protocol": proto, "endpoint": srv.url, "bucket": "b", "object_prefix": "o", "workers": 1,
                        "reads_per_worker": 2, "sink": "gpu", "ring_slot_bytes": slot, "ring_slots": 4,
                        "keep_records": False, "cpus": pl["client"]})
        run.start(); run.wait()
        run.reset_stats(); run.set_reads_per_worker(reads)
        run.start(); run.wait()
        s = run.summary()
        print(json.dumps({"mode": mode, "proto": proto, "slot_MiB": slot >> 20,
                          "p50_ms": round(s["p50_ms"], 2), "p99_ms": round(s["p99_ms"], 2),
                          "min_ms": round(s["min_ms"], 2), "GiB/s@p50": round(size / (s["p50_ms"] / 1e3) / 2**30, 2),
                          "errors": s["errors"], "wait_s": round(s["gpu"]["slot_wait_s"], 4)}), flush=True)
    srv.stop()
