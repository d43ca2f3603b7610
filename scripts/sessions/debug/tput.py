"""Loopback transport throughput probe (discard sink, no CRC) for tuning."""
import sys, os, time, json, itertools
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import custom_go_client_benchmark_amd as pkg
n = pkg._native
size = int(os.environ.get("SIZE", 256 << 20))
reads = int(os.environ.get("READS", 6))
for zc, ssnd in itertools.product([True, False], [0, 8 << 20]):
    srv = n.Server({"port": 0, "md5": False, "sndbuf": ssnd, "zero_copy": zc})
    srv.start()
    srv.add_synthetic("b", "o", "", 0, 1, size)
    for proto, rcv in itertools.product(["http", "grpc"], [0, 8 << 20]):
        c = n.Client({"protocol": proto, "endpoint": srv.url, "rcvbuf": rcv, "sndbuf": rcv})
        c.read("b", "o0", host_crc=False)
        best = 1e9
        tot = 0
        for _ in range(reads):
            t = time.perf_counter()
            c.read("b", "o0", host_crc=False)
            dt = time.perf_counter() - t
            best = min(best, dt)
            tot += dt
        r = {"proto": proto, "zero_copy": zc, "srv_sndbuf": ssnd, "cli_rcvbuf": rcv, "mean_ms": round(tot / reads * 1e3, 2),
             "best_GiB/s": round(size / best / 2**30, 2), "mean_GiB/s": round(size * reads / tot / 2**30, 2)}
        print(json.dumps(r), flush=True)
    srv.stop()
for f in ["/proc/sys/net/core/rmem_max", "/proc/sys/net/core/wmem_max", "/proc/sys/net/ipv4/tcp_rmem",
          "/proc/sys/net/ipv4/tcp_wmem"]:
    try:
        print(f, open(f).read().strip())
    except Exception as e:
        print(f, e)
print("cpus", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
