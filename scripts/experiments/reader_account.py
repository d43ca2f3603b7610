"""Cross-checks the HTTP/2 reader's time split against wall time on the
list-read geometry (8 workers x 1 MiB objects on one gRPC connection, GPU
sink through the connection ring): samples the process's thread names while
the timed pass runs, so a second connection reader would show."""
import json
import os
import threading
import time

import custom_go_client_benchmark_amd._native as n
from custom_go_client_benchmark_amd.utils import cpuacct

B, P = "bkt", "lr/file_"
srv = n.Server({"port": 0, "md5": False})
srv.start()
srv.add_synthetic(B, P, "", 0, 1000, 1 << 20)
names = [f"{P}{i}" for i in range(1000)]
if os.environ.get("LISTER") == "1":
    # as bench.py's list_read block: a client lists the objects first
    lister = n.Client({"protocol": "grpc", "endpoint": srv.url, "retry_initial_s": 0.05})
    names = [o["name"] for o in lister.list_all(B, P, 1000)]
    del lister
out = {}
SINKS = os.environ.get("SINKS", "gpu,discard").split(",")
for sink in SINKS:
    cfg = {"protocol": "grpc", "endpoint": srv.url, "bucket": B, "object_prefix": P, "workers": 8,
           "object_names": names, "reads_per_worker": 125, "sink": sink, "host_crc": sink != "gpu",
           "grpc_conn_pool_size": 1, "keep_records": False, "ring_slots": 2, "ring_slot_bytes": 1 << 20}
    r = n.Runner(cfg)
    r.start()
    r.wait()
    r.reset_stats()
    seen = {}
    stop = threading.Event()

    def sample():
        while not stop.is_set():
            for t in os.listdir("/proc/self/task"):
                try:
                    with open(f"/proc/self/task/{t}/comm") as f:
                        c = f.read().strip()
                except OSError:
                    continue
                if c.startswith("gcsb-h2"):
                    seen.setdefault(c, set()).add(t)
            time.sleep(0.002)

    th = threading.Thread(target=sample)
    th.start()
    h0 = n.h2_reader_stats()
    c0 = cpuacct.thread_cpu()
    t0 = time.perf_counter()
    r.start()
    r.wait()
    el = time.perf_counter() - t0
    c1 = cpuacct.thread_cpu()
    h1 = n.h2_reader_stats()
    stop.set()
    th.join()
    s = r.summary()
    d = {k: h1[k] - h0[k] for k in h1}
    cpu = cpuacct.delta_by_name(c0, c1)
    out[sink] = {"elapsed_s": round(el, 4), "bytes": s["bytes"], "mib_s": round(s["bytes"] / el / 2**20, 1),
                 "reader_threads_seen": {k: len(v) for k, v in seen.items()},
                 "wait_s": round(d["header_wait_ns"] / 1e9, 4), "data_s": round(d["data_ns"] / 1e9, 4),
                 "headers_s": round(d["headers_ns"] / 1e9, 4), "other_s": round(d["other_ns"] / 1e9, 4),
                 "frames": d["frames"], "reader_cpu_s": round(cpu.get("gcsb-h2-reader", 0.0), 4)}
    print(json.dumps({sink: out[sink]}), flush=True)
    del r
srv.stop()
