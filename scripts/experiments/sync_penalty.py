"""Does torch.cuda.synchronize() (hipDeviceSynchronize) make our next GPU
operation slow?  Times gpu_crc32c of 4 KiB and 64 MiB buffers back to back,
then right after a device synchronize, a stream synchronize and a sleep.
Found by scripts/experiments/write_tail.py --gap sync (first upload after the
bench's barrier + synchronize: GPU CRC 7 ms instead of 0.09 ms)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch  # noqa: E402

import custom_go_client_benchmark_amd as pkg  # noqa: E402

n = pkg._native
buf = torch.empty(64 << 20, dtype=torch.uint8, device="cuda:0")
n.gpu_fill_pattern(0, buf.data_ptr(), 64 << 20, "p", 0)
p = buf.data_ptr()


def t(fn):
    t0 = time.perf_counter()
    fn()
    return round((time.perf_counter() - t0) * 1e3, 3)


small = lambda: n.gpu_crc32c(0, p, 4096)
big = lambda: n.gpu_crc32c(0, p, 64 << 20)
out = {"warm_big": [t(big) for _ in range(3)], "warm_small": [t(small) for _ in range(3)]}
for name, gap in [("devsync", torch.cuda.synchronize), ("streamsync", lambda: torch.cuda.current_stream().synchronize()),
                  ("sleep50", lambda: time.sleep(0.05)), ("devsync_again", torch.cuda.synchronize)]:
    gap()
    out[name] = {"small_then": t(small), "big_then": t(big), "big_again": t(big)}
gap = torch.cuda.synchronize
gap()
out["devsync_big_first"] = t(big)
gap()
x = torch.empty(1024, device="cuda:0")
t0 = time.perf_counter()
x.add_(1)
torch.cuda.current_stream().synchronize()
out["devsync_torch_op_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
out["big_after_torch_op"] = t(big)
print(json.dumps(out))
