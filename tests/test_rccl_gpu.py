"""RCCL (torch.distributed backend "nccl" on ROCm) on a real MI355X.

The control plane (parallel/dist.py: R0 rendezvous, R1/R2 barriers, R3 stat
reductions, R4 all-gather) must run over RCCL on the hardware it targets, not
only over gloo on the CPU.  A 1-GPU box can only host a world-1 communicator
(RCCL refuses two ranks on one GPU), so these tests create the process group
at world 1 (`always_pg`) and drive every collective through it; the bench does
the same in every GPU run.  Each case runs in a child process so the process
group never leaks into the pytest process.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

_CHILD = r"""
import json, sys
sys.path.insert(0, ROOT)
import torch
import torch.distributed as dist
from custom_go_client_benchmark_amd.parallel import dist as gdist

ctx = gdist.init(always_pg=True)
assert ctx.pg and ctx.backend == "nccl" and dist.get_backend() == "nccl", (ctx, dist.get_backend())
assert ctx.device.type == "cuda"
gdist.barrier(ctx, "R1 test barrier")
st = gdist.reduce_stats(ctx, x=3.5, y=-1.0)
g = gdist.gather_floats(ctx, [1.0, 2.0, 3.0])
h = gdist.reduce_histogram(ctx, [0, 5, 7, 1])
# a bigger all_reduce on the rank's stream, checked on the host
t = torch.arange(1 << 20, dtype=torch.float32, device=ctx.device)
dist.all_reduce(t)
torch.cuda.synchronize()
ok_big = bool(torch.equal(t.cpu(), torch.arange(1 << 20, dtype=torch.float32)))
ver = ".".join(str(v) for v in torch.cuda.nccl.version()) if hasattr(torch.cuda, "nccl") else "?"
gdist.shutdown(ctx)
print(json.dumps({"st": st, "g": g, "h": h, "ok_big": ok_big, "rccl": ver}))
"""


def _env():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "GCSB_DIST_BACKEND"):
        env.pop(k, None)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    return env


def test_rccl_world1_collectives(gpu_available):
    r = subprocess.run([sys.executable, "-c", f"ROOT = {ROOT!r}\n" + _CHILD], capture_output=True, text=True,
                       timeout=110, cwd=ROOT, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    st = out["st"]
    assert st["x_sum"] == 3.5 and st["x_max"] == 3.5 and st["y_min"] == -1.0 and st["x_per_rank"] == [3.5]
    assert out["g"] == [[1.0, 2.0, 3.0]]
    assert out["h"] == [0, 5, 7, 1]
    assert out["ok_big"]
    print("RCCL version", out["rccl"])


def _bench(args, extra_env=None, timeout=110):
    env = _env()
    env.update(extra_env or {})
    r = subprocess.run([sys.executable, "bench.py"] + args, capture_output=True, text=True, timeout=timeout,
                       cwd=ROOT, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_one_gpu_rccl_and_blocks(gpu_available):
    """The bench's 1-GPU path: RCCL process group, headline single-stream
    reads with every read CRC-verified, compare/sliced/write side blocks."""
    out = _bench(["--gpus", "1", "--steps", "3", "--warmup", "1", "--object-size", "32MiB", "--side-steps", "2",
                  "--write-size", "16MiB"])
    assert out["n_gpus"] == 1 and out["ranks"] == 1 and out["devices"] == [0]
    assert out["config"]["streams_per_read"] == 1 and out["verified_reads"] == 3
    assert out["value"] > 0 and out["p50_ms"] > 0
    assert out["compare"]["ok"] and out["sliced"]["ok"], out
    assert out["write"]["ok"] and out["write"]["mib_s"] > 0, out


def test_bench_write_headline(gpu_available):
    out = _bench(["--workload", "write", "--steps", "3", "--warmup", "1", "--write-size", "16MiB"])
    assert out["config"]["workload"] == "write" and out["value"] > 0 and out["n_gpus"] == 1


def test_bench_shared_gpu_rehearsal_counts_distinct_devices(gpu_available):
    """Two ranks on one GPU (gloo control plane) report n_gpus = 1, ranks = 2."""
    out = _bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--object-size", "16MiB", "--side-steps", "0"],
                 {"GCSB_DIST_BACKEND": "gloo"})
    assert out["n_gpus"] == 1 and out["ranks"] == 2 and out["devices"] == [0]


def test_bench_fanout_block_shared_gpu(gpu_available):
    """Fan-out block on the GPU path (ranged slice reads into HBM in place,
    GPU CRC of the gathered object); the all-gather goes through host memory
    on this 1-GPU box's gloo control plane."""
    out = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--object-size", "32MiB", "--side-steps", "2",
                  "--sliced-streams", "0"], {"GCSB_DIST_BACKEND": "gloo"})
    f = out["fanout"]
    assert f["ok"] and f["crc_verified_ranks"] == 2, f


def test_bench_refuses_more_ranks_than_gpus(gpu_available):
    import torch

    n = torch.cuda.device_count()
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(n + 1), "--steps", "1", "--warmup", "0",
                        "--object-size", "1MiB", "--side-steps", "0"], capture_output=True, text=True,
                       timeout=110, cwd=ROOT, env=_env())
    assert r.returncode != 0 and "visible GPU" in r.stderr, r.stderr[-2000:]
