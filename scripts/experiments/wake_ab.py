"""A/B: deferred discard sink wake-ups (every message vs two blocks) on the
reference's 48 x 1 MiB gRPC pool-1 experiment, interleaved."""
import json, sys, time, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch  # noqa
import custom_go_client_benchmark_amd as pkg
from custom_go_client_benchmark_amd.parallel import affinity
from custom_go_client_benchmark_amd.utils import cpuacct
n = pkg._native
pl = affinity.plan(0, "same", 0)
srv = n.Server({"port": 0, "md5": False, "cpus": pl["server"], "retain_uploads": False})
srv.start()
srv.add_synthetic("b", "w/f_", "", 0, 48, 1 << 20)
cfg = {"protocol": "grpc", "endpoint": srv.url, "bucket": "b", "object_prefix": "w/f_", "workers": 48,
       "reads_per_worker": 2, "sink": "discard", "host_crc": True, "keep_records": False, "cpus": pl["client"],
       "grpc_conn_pool_size": 1, "tcp_congestion": "cubic", "loopback_rto_min": True}
r = n.Runner(cfg)
r.start(); r.wait()
for rep in range(6):
    for mode in (0, 2):
        n.set_deferred_wake_blocks(mode)
        r.reset_stats(); r.set_reads_per_worker(50)
        t0 = cpuacct.thread_cpu(); w0 = time.perf_counter()
        r.start(); r.wait()
        el = time.perf_counter() - w0
        d = cpuacct.delta_by_name(t0, cpuacct.thread_cpu()); s = r.summary(); gib = s["bytes"] / (1 << 30)
        print(json.dumps({"rep": rep, "wake_blocks": mode, "mib_s": round(s["bytes"] / el / (1 << 20)),
                          "p50_ms": round(s["p50_ms"], 3), "p99_ms": round(s["p99_ms"], 3),
                          "reader": round(d.get("gcsb-h2-reader", 0) / gib, 4),
                          "worker": round(s.get("worker_cpu_s", 0) / gib, 4), "errors": s["errors"]}), flush=True)
srv.stop()
