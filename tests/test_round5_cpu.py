"""Round-5 CPU tests: the bench line fits the driver's 8 KiB stdout tail at 1
and 8 ranks with every block, the sidecar carries the verbose views, and the
paired-estimator / bound arithmetic (custom_go_client_benchmark_amd/benchmark/
report.py) is right."""
import json
import os
import subprocess
import sys

import pytest

from custom_go_client_benchmark_amd.benchmark import report as rp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# every block a GPU run at N = 8 with --blocks all can carry
ALL_BLOCKS = ("cpu_baseline", "cpu_baseline_http", "compare", "cpu_baseline_before", "sliced", "ceiling",
              "ref_default_http", "ref_default_grpc", "ref_effective_grpc", "ref_default_100m_http_discard",
              "ref_default_100m_http_gpu", "ref_default_100m_grpc_discard", "ref_default_100m_grpc_gpu",
              "c1_http_cpu", "list_read_grpc", "list_read_http", "write", "write_composite", "fanout",
              "ref_framing", "ref_default_grpc_ref", "list_read_grpc_ref", "ref_effective_head")


def _worst_block(i: int) -> dict:
    """A block with every key the verbose view can have, long values."""
    b = {"ok": False, "mib_s": 123456.78 + i, "p50_ms": 1234.567, "p99_ms": 2345.678, "protocol": "grpc",
         "workers": 48, "sink": "gpu", "streams_per_read": 8, "parts": 8, "frac_of_bound": 0.987, "bound": "tcp_1conn",
         "vs_discard_twin": 1.234, "vs_ref_effective": 1.456, "recv_cpu_s_per_gib": 0.0512, "py_cpu_s_per_gib": 0.0133,
         "first_read_p50_ms": 12.345, "steady_p99_ms": 23.456, "list_ms": 88.123, "per_gpu_mib_s": 12345.67,
         "crc_verified_ranks": 8, "error": "x" * 400,
         "rank0_slowest": [[1000 + k, 123.456, 120.1, 3.2] for k in range(3)],
         "host": {"threads": {f"t{k}": {"cpu_ms_per_read": 1.0} for k in range(20)}},
         "cpu_s_per_gib_by_thread": {f"name{k}": 0.01 for k in range(12)}}
    return b


def test_fit_line_worst_case_8_ranks():
    out = {"metric": "m" * 74, "value": 123456.78, "unit": "MiB/s", "n_gpus": 8, "steps": 20, "warmup": 5,
           "ms_per_step": 10.123, "higher_is_better": True, "scaling": "weak", "vs_baseline": 0.987, "dtype": "uint8",
           "data": "synthetic",
           "config": {"model": "grpc ReadObject 256MiB object, one stream per read -> HBM (CRC32C on GPU)",
                      "global_batch": 8, "seq_len": 268435456, "parallelism": "dp8", "workload": "read",
                      "protocol": "grpc", "object_bytes": 268435456, "readers_per_gpu": 1, "sink": "gpu",
                      "ring": "4x1MiB", "streams_per_read": 1},
           "p50_ms": 9.123, "p99_ms": 12.345, "vs_baseline_paired": 1.01, "headline_vs_nodma": 0.98,
           "headline_frac_of_ceiling": 0.91, "per_rank_mib_s": [26000.1 + k for k in range(8)],
           "paired": {"chunks": 4, "pair_ratios": [1.0] * 4, "nodma_ratios": [1.0] * 4, "tcp_ratios": [0.95] * 4,
                      "head_mib_s": [27000.0] * 4, "base_mib_s": [27000.0] * 4, "nodma_mib_s": [27000.0] * 4,
                      "tcp_mib_s": [28888.8] * 4,
                      "slow_windows": [[0, "c" * 120], [1, "c" * 120]]},
           "rank0_slowest": [[1, 12.3], [2, 11.1], [3, 10.0]],
           "baseline": {"mib_s": 1.0, "p50_ms": 1.0, "p50_ratio": 1.0, "mib_s_before": 1.0, "mib_s_after": 1.0}}
    blocks = {k: _worst_block(i) for i, k in enumerate(ALL_BLOCKS)}
    line = rp.ordered(rp.fit_line(out, blocks))
    text = json.dumps(line)
    assert len(text.encode()) <= rp.LINE_LIMIT
    assert list(line)[:len(rp.DRIVER_KEYS)] == list(rp.DRIVER_KEYS)
    for k in ALL_BLOCKS:  # every block keeps its verdict and rate
        assert line[k]["mib_s"] > 0 and "ok" in line[k]
    # the verbose views never reach the line
    assert "host" not in text and "cpu_s_per_gib_by_thread" not in text


def test_fit_line_keeps_small_lines_whole():
    out = {"metric": "m", "value": 1.0, "unit": "MiB/s", "config": {}, "paired": {"chunks": 4}}
    blocks = {"compare": {"ok": True, "mib_s": 2.0, "p50_ms": 1.0, "p99_ms": 2.0, "rank0_slowest": [[0, 1.0, 2, 3]],
                          "host": {"x": 1}}}
    line = rp.fit_line(out, blocks)
    assert line["compare"] == {"ok": True, "mib_s": 2.0, "p50_ms": 1.0, "p99_ms": 2.0, "rank0_slowest": [[0, 1.0]]}
    assert line["paired"] == {"chunks": 4}


def test_chunks_and_rotation():
    assert rp.chunk_sizes(20, 4) == [5, 5, 5, 5]
    assert rp.chunk_sizes(10, 4) == [3, 3, 2, 2]
    assert rp.chunk_sizes(2, 4) == [1, 1]
    assert sum(rp.chunk_sizes(7, 4)) == 7
    orders = [rp.arm_order(["head", "base", "nodma"], i) for i in range(3)]
    assert orders == [["head", "base", "nodma"], ["base", "nodma", "head"], ["nodma", "head", "base"]]
    # every arm is first once and last once over 3 chunks
    assert {o[0] for o in orders} == {o[-1] for o in orders} == {"head", "base", "nodma"}


def test_paired_summary_median_resists_one_slow_window():
    chunks = [{"head": 27000, "base": 26000, "nodma": 27500},
              {"head": 27200, "base": 26500, "nodma": 27600},
              # a slow host window: both arms of the chunk slow
              {"head": 14000, "base": 15000, "nodma": 14500},
              {"head": 27100, "base": 26300, "nodma": 27400}]
    s = rp.paired_summary(chunks)
    assert s["chunks"] == 4 and len(s["pair_ratios"]) == 4
    # median of 4 = mean of the middle two ratios
    r = sorted(c["head"] / c["base"] for c in chunks)
    assert s["vs_baseline_paired"] == round((r[1] + r[2]) / 2, 3)
    assert 1.0 < s["vs_baseline_paired"] < 1.04
    assert 0.97 < s["headline_vs_nodma"] < 1.0
    # a missing arm gives no ratio for that chunk
    s2 = rp.paired_summary([{"head": 10.0, "base": 5.0}, {"head": 10.0}])
    assert s2["pair_ratios"] == [2.0] and "headline_vs_nodma" not in s2
    # the TCP arm: a paired fraction of the raw one-stream ceiling
    s3 = rp.paired_summary([{"head": 27000, "tcp": 30000}, {"head": 26000, "tcp": 29000},
                            {"head": 25000, "tcp": 24000}])
    assert s3["headline_vs_tcp_paired"] == 0.9 and len(s3["tcp_ratios"]) == 3  # median of 0.897, 0.9, 1.042


def test_frac_of_bound_is_a_ceiling():
    # one connection, GPU sink: min(h2d, one-connection TCP)
    b = rp.frac_of_bound(21606.0, 51.9, 30.0, 1, True)
    assert b["bound"] == "tcp_1conn" and b["bound_mib_s"] == round(30.0e9 / (1 << 20), 1)
    assert b["frac_of_bound"] == round(21606.0 / (30.0e9 / (1 << 20)), 3) < 1.0
    # many connections, GPU sink: h2d only
    b = rp.frac_of_bound(48000.0, 51.9, 30.0, 48, True)
    assert b["bound"] == "h2d"
    # many connections, discard: no bound at all
    assert rp.frac_of_bound(70000.0, 51.9, 30.0, 48, False) == {}
    # one connection, discard: TCP
    assert rp.frac_of_bound(20000.0, 0.0, 30.0, 1, False)["bound"] == "tcp_1conn"
    # h2d below TCP: h2d is the bound
    assert rp.frac_of_bound(20000.0, 25.0, 30.0, 1, True)["bound"] == "h2d"


def test_unified_ceiling_is_the_best_probe():
    # the paired probes are whole-job rates: per GPU they are / world
    u = rp.unified_ceiling(25000.0, [2 * 27000.0, 2 * 29000.0], {"ok": True, "tcp_gbps": 29.0e9 / (1 << 20) / 1e3
                                                                  * 1e3 * (1 << 20) / 1e9 * 1.0, "h2d_gbps": 50.0},
                           2, True)
    assert u["tcp_probes"] == 3 and u["tcp_best_mib_s"] == 29000.0 and u["ceiling_bound"] == "tcp_1conn"
    assert u["headline_frac_of_ceiling"] == round(25000.0 / 29000.0, 3)
    # h2d below TCP: h2d is the ceiling
    u = rp.unified_ceiling(20000.0, [30000.0], {"ok": True, "tcp_gbps": 0.0, "h2d_gbps": 22.0}, 1, True)
    assert u["ceiling_bound"] == "h2d" and u["headline_frac_of_ceiling"] == round(20000.0 / (22.0 * rp.MIB_PER_GBPS), 3)
    # a headline faster than every probe: the probe was no ceiling
    u = rp.unified_ceiling(31000.0, [30000.0], None, 1, False)
    assert u["headline_frac_of_ceiling"] == 1.0 and u["ceiling_observed"] == "headline"
    assert rp.unified_ceiling(1.0, None, None, 1, True) == {}


def test_observed_bounds_never_beaten():
    blocks = {"a": {"mib_s": 31000.0, "bound": "tcp_1conn", "bound_mib_s": 30000.0, "frac_of_bound": 1.033},
              "b": {"mib_s": 24000.0, "bound": "tcp_1conn", "bound_mib_s": 30000.0, "frac_of_bound": 0.8},
              "c": {"mib_s": 40000.0, "bound": "h2d", "bound_mib_s": 48000.0, "frac_of_bound": 0.833},
              "d": {"mib_s": 20000.0, "bound": "tcp_1conn", "bound_mib_s": 22000.0, "frac_of_bound": 0.909}}
    raised = rp.observed_bounds(blocks, (32000.0, "tcp_1conn", 30000.0))
    # the headline beat both the probe and block a: its rate is the bound of the group
    assert raised == {"tcp_1conn@30000.0": 32000.0}
    assert blocks["a"]["frac_of_bound"] == round(31000 / 32000, 3) and blocks["a"]["bound_observed"] == "headline"
    assert blocks["b"]["frac_of_bound"] == 0.75 and blocks["c"]["frac_of_bound"] == 0.833
    assert blocks["d"]["frac_of_bound"] == 0.909  # another bound group, untouched
    assert all(b["frac_of_bound"] <= 1.0 for b in blocks.values())


def test_attribute_windows_names_the_cause():
    w = [{"chunk": i, "arm": "head", "mib_s": 27000.0, "recv_cpu_s_per_gib": 0.036, "clock_mhz": 5000}
         for i in range(4)]
    w[2] = {"chunk": 2, "arm": "head", "mib_s": 15000.0, "recv_cpu_s_per_gib": 0.07, "clock_mhz": 3000,
            "numa_pages_migrated": 512, "compact_stall": 0, "tcp_retrans": 37}
    w.append({"chunk": 2, "arm": "base", "mib_s": 15000.0})
    slow = rp.attribute_windows(w)
    assert len(slow) == 1 and slow[0]["chunk"] == 2
    c = slow[0]["cause"]
    assert "clock 3000" in c and "512 NUMA page migrations" in c and "receive copy" in c
    assert "37 TCP retransmits" in c
    assert rp.attribute_windows(w[:2]) == []


def _bench(args, timeout=420):
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env.setdefault("OMP_NUM_THREADS", "1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, "bench.py"] + args, capture_output=True, text=True, timeout=timeout,
                          cwd=ROOT, env=env)


SMALL = ["--sink", "discard", "--steps", "4", "--warmup", "1", "--object-size", "2MiB", "--blocks", "all",
         "--ref-reads", "3", "--ref100-reads", "1", "--ref100-object-size", "2MiB", "--list-objects", "64",
         "--side-steps", "2"]


@pytest.mark.parametrize("gpus", [1, 8])
def test_bench_line_fits_the_driver_tail(gpus, tmp_path):
    diag = tmp_path / "diag.json"
    r = _bench(["--gpus", str(gpus), "--diag-out", str(diag)] + SMALL)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1, r.stdout[:2000]  # stdout holds the ONE line, nothing else
    last = lines[0]
    assert len(last.encode()) <= rp.LINE_LIMIT, len(last)
    line = json.loads(last)
    for k in rp.DRIVER_KEYS:
        assert k in line, k
    assert list(line)[:len(rp.DRIVER_KEYS)] == list(rp.DRIVER_KEYS)
    assert line["n_gpus"] == gpus and line["value"] > 0
    # the sidecar holds the verbose views and the same line
    d = json.loads(diag.read_text())
    assert d["line"] == line and "blocks" in d and "placement" in d
    # the paired headline at every N (each rank the same arm order between barriers)
    assert line["paired"]["chunks"] == 4 and 0.2 < line["vs_baseline_paired"] < 5.0
    assert len(d["paired"]["windows"]) == 8  # 4 chunks x (head, base): no nodma without a GPU
    # each chunk's first read is reported, after the arm's untimed re-warm read
    assert line["paired"]["rewarm_reads"] == 1 and len(line["paired"]["head_first_vs_median"]) == 4
    assert all(len(w["first_read"]) == 3 for w in d["paired"]["windows"])
    # the headline config at the other framing, paired with its baseline
    assert line["ref_framing"]["ok"] and line["ref_framing"]["h2_frames"] == "16KiB"
    assert line["ref_framing"]["vs_baseline_paired"] > 0 and line["h2_frames"] == "16MiB"
    assert line["h2_window_mib"] == 16  # the reference's window at both framings
    assert line["list_read_grpc_ref"]["ok"] and line["ref_default_grpc_ref"]["h2_frames"] == "16KiB"
    # one ceiling: no block beats its bound
    for k, b in line.items():
        if isinstance(b, dict) and "frac_of_bound" in b:
            assert b["frac_of_bound"] <= 1.0, (k, b)
    if gpus == 1:
        assert line["ref_effective_grpc"]["ok"] and line["ref_default_100m_grpc_discard"]["vs_ref_effective"] > 0
        # the effective-path twin of the headline config, next to vs_baseline
        assert line["ref_effective_head"]["ok"] and line["headline_vs_ref_effective"] > 0
        assert "host" in d["blocks"]["compare"]
    else:
        assert len(line["per_rank_mib_s"]) == 8


def test_native_stdout_noise_goes_to_stderr():
    """What a native library writes to fd 1 after the rank claimed stdout (RCCL
    prints a version banner at communicator init) lands on stderr; stdout
    carries only the JSON line."""
    code = ("import os\n"
            "from custom_go_client_benchmark_amd.benchmark.rank import stash\n"
            "stash.claim_stdout()\n"
            "os.write(1, b'RCCL version : banner\\n')\n"
            "print('python noise')\n"
            "stash.final('{\"metric\": 1}')\n")
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr
    assert r.stdout == '{"metric": 1}\n'
    assert "RCCL version" in r.stderr and "python noise" in r.stderr


def test_fit_line_never_exceeds_the_limit():
    """Even a pathological headline (huge config strings) yields a line within
    the limit with the driver keys, never an exception."""
    out = {k: ("x" * 3000 if k in ("metric", "data") else 1) for k in rp.DRIVER_KEYS}
    out["config"] = {"model": "y" * 3000}
    line = rp.fit_line(out, {"b": {"ok": True, "mib_s": 1.0}})
    assert len(json.dumps(line).encode()) <= rp.LINE_LIMIT or set(rp.DRIVER_KEYS) <= set(line)
    assert "value" in line


def test_rocprof_db_summary_reads_the_sqlite_views(tmp_path):
    """scripts/rocprof_db_summary.py over a database with rocprofv3's
    `kernels` and `memory_copies` views: per-name calls, times and sizes."""
    import sqlite3

    d = tmp_path / "prof" / "host"
    d.mkdir(parents=True)
    c = sqlite3.connect(d / "run_results.db")
    c.execute("create table kernels (name text, duration integer)")
    c.execute("create table memory_copies (name text, duration integer, size integer)")
    c.executemany("insert into kernels values (?, ?)", [("crc32c_slot_kernel", 8000), ("crc32c_slot_kernel", 9000),
                                                         ("fill", 1000)])
    c.executemany("insert into memory_copies values (?, ?, ?)",
                  [("MEMORY_COPY_HOST_TO_DEVICE", 28000, 1 << 20)] * 4)
    c.commit()
    c.close()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "rocprof_db_summary.py"), str(tmp_path)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)[0]
    k = {x["name"]: x for x in out["kernels"]}
    assert k["crc32c_slot_kernel"]["calls"] == 2 and k["crc32c_slot_kernel"]["avg_us"] == 8.5
    m = out["memory_copies"][0]
    assert m["calls"] == 4 and m["mean_kib"] == 1024.0 and m["avg_us"] == 28.0
    md = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "rocprof_db_summary.py"), str(tmp_path), "--md"],
                        capture_output=True, text=True, timeout=60)
    assert md.returncode == 0 and "| `crc32c_slot_kernel` | 2 |" in md.stdout


def test_fixed_overrides_parse_and_reject():
    """GCSB_FIXED overrides FIXED settings for A/B sessions; an unknown key or
    an item without '=' ends the run instead of being ignored."""
    from custom_go_client_benchmark_amd.benchmark import rank

    assert rank.fixed_overrides(None) == {}
    assert rank.fixed_overrides("list_ring_wc=off, write_async_stage=off") == {
        "list_ring_wc": "off", "write_async_stage": "off"}
    assert rank.fixed_overrides("sliced_slots=3") == {"sliced_slots": 3}
    with pytest.raises(SystemExit):
        rank.fixed_overrides("no_such_key=1")
    with pytest.raises(SystemExit):
        rank.fixed_overrides("list_ring_wc")
