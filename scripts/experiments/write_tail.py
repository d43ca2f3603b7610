"""Config-5 upload tail probe: N back-to-back 64 MiB uploads from HBM over the
bench's write-block setup (share-placed endpoint, uploader on the GPU's L3
domains), printing every upload's time in order so a periodic tail (every
k-th upload) can be told from a random one.

  python scripts/experiments/write_tail.py [--n 200] [--protocol grpc] [--size 64MiB]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))

import torch  # noqa: E402

import custom_go_client_benchmark_amd as pkg  # noqa: E402
from custom_go_client_benchmark_amd.parallel import affinity  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--protocol", default="grpc")
    ap.add_argument("--size", type=int, default=64 << 20)
    ap.add_argument("--chunk", type=int, default=16 << 20)
    ap.add_argument("--slot-bytes", type=int, default=2 << 20)
    ap.add_argument("--slots", type=int, default=8)
    ap.add_argument("--label", default="")
    ap.add_argument("--gap", default="none", choices=["none", "sleep", "nccl", "gloo", "sync", "pginit", "devsync"],
                    help="between warm-up and timed uploads: nothing, a 200 ms sleep, or a one-rank "
                         "process-group barrier (all_reduce + synchronize), as bench.py does")
    a = ap.parse_args()
    n = pkg._native
    sh = affinity.plan(0, "share", 0)
    ep = n.Server({"port": 0, "md5": False, "cpus": sh["server"], "retain_uploads": False})
    ep.start()
    if sh["client"]:
        os.sched_setaffinity(0, sh["client"])
    client = n.Client({"protocol": a.protocol, "endpoint": ep.url, "retry_initial_s": 0.05})
    buf = torch.empty(a.size, dtype=torch.uint8, device="cuda:0")
    n.gpu_fill_pattern(0, buf.data_ptr(), a.size, "upload/probe", 0)
    for i in range(a.warmup):
        client.write_from_device("b", f"w/warm{i}", buf.data_ptr(), a.size, 0, True, a.chunk, a.slot_bytes, a.slots)
    if a.gap == "sleep":
        time.sleep(0.2)
    elif a.gap == "sync":
        torch.cuda.synchronize()
    elif a.gap == "devsync":
        n.gpu_device_synchronize(0) if hasattr(n, "gpu_device_synchronize") else torch.cuda.synchronize()
    elif a.gap == "pginit":
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29577")
        dist.init_process_group("gloo", rank=0, world_size=1)
    elif a.gap in ("nccl", "gloo"):
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29577")
        dist.init_process_group(a.gap, rank=0, world_size=1)
        t = torch.ones(1, dtype=torch.int32, device="cuda:0" if a.gap == "nccl" else "cpu")
        dist.all_reduce(t)
        torch.cuda.synchronize()
    lat = []
    inner = []
    crcms = []
    for i in range(a.n):
        t0 = time.perf_counter()
        m = client.write_from_device("b", f"w/up{i}", buf.data_ptr(), a.size, 0, True, a.chunk, a.slot_bytes,
                                     a.slots)
        lat.append((time.perf_counter() - t0) * 1e3)
        inner.append(m.get("upload_ms", 0.0))
        crcms.append(m.get("gpu_crc_ms", 0.0))
        if m["size"] != a.size or m["crc32c"] != m["gpu_crc32c"]:
            print("upload not confirmed", m, file=sys.stderr)
            return 1
    s = sorted(lat)
    q = lambda p: s[min(len(s) - 1, len(s) * p // 100)]
    slow = [(i, round(v, 2), round(crcms[i], 2), round(inner[i], 2)) for i, v in enumerate(lat) if v > 1.5 * q(50)]
    print(json.dumps({"label": a.label, "protocol": a.protocol, "n": a.n, "p50": round(q(50), 3),
                      "p90": round(q(90), 3), "p99": round(q(99), 3), "max": round(s[-1], 3),
                      "mib_s": round(a.size * a.n / (sum(lat) / 1e3) / (1 << 20), 1),
                      "crc_ms_p50": round(sorted(crcms)[len(crcms) // 2], 3),
                      "gap": a.gap, "first_ms": round(lat[0], 3),
                      "slow_uploads (i, ms, gpu_crc_ms, upload_ms)": slow[:40], "n_slow": len(slow),
                      "placement": {k: sh.get(k) for k in ("client", "server")}}))
    ep.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
