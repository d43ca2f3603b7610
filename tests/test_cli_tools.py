"""CLI (Go-flag compatible), exporters, drivers and native FS tools."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "custom_go_client_benchmark_amd", "bin")
GCSBENCH = os.path.join(ROOT, "gcsbench")


def run(args, **kw):
    return subprocess.run(args, capture_output=True, text=True, timeout=kw.pop("timeout", 120), **kw)


# --- Go flag semantics -------------------------------------------------------

def test_goflags_forms():
    from custom_go_client_benchmark_amd.utils.goflags import FlagError, FlagSet, parse_duration

    fs = FlagSet("t")
    fs.int("worker", 48, "")
    fs.bool("enable-tracing", False, "")
    fs.string("client-protocol", "http", "")
    fs.float("trace-sample-rate", 1.0, "")
    fs.duration("d", 0.0, "")
    fs.parse(["-worker", "3", "--enable-tracing", "-client-protocol=grpc", "--trace-sample-rate=0.25",
              "-d", "1m30s", "rest", "-x"])
    assert fs.get("worker") == 3 and fs.get("enable-tracing") is True
    assert fs.get("client-protocol") == "grpc" and fs.get("trace-sample-rate") == 0.25
    assert fs.get("d") == 90.0 and fs.args == ["rest", "-x"]
    fs2 = FlagSet("t")
    fs2.bool("b", True, "")
    fs2.int("n", 0, "")
    fs2.parse(["-b=false", "-n=0x10"])
    assert fs2.get("b") is False and fs2.get("n") == 16
    with pytest.raises(FlagError, match="not defined: -nope"):
        FlagSet("t").parse(["-nope"], exit_on_error=False)
    assert parse_duration("250ms") == 0.25 and parse_duration("30s") == 30.0


def test_cli_unknown_flag_exits_2():
    r = run([GCSBENCH, "-nope"])
    assert r.returncode == 2 and "flag provided but not defined: -nope" in r.stderr
    assert "-read-call-per-worker" in r.stderr


def test_cli_rejects_bad_protocol():
    r = run([GCSBENCH, "-client-protocol", "ftp", "-start-fake-server"])
    assert r.returncode == 2 and "want http" in r.stderr


def test_cli_no_endpoint_fails_cleanly():
    env = {k: v for k, v in os.environ.items() if k not in ("GCSB_ENDPOINT", "STORAGE_EMULATOR_HOST")}
    r = run([GCSBENCH, "-worker", "1", "-read-call-per-worker", "1"], env=env)
    assert r.returncode == 1 and "no endpoint" in r.stderr


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_cli_latency_lines_metrics_traces(tmp_path, proto):
    m = tmp_path / "m.prom"
    mj = tmp_path / "m.jsonl"
    t = tmp_path / "t.jsonl"
    r = run([GCSBENCH, "-worker", "3", "-read-call-per-worker", "4", "-client-protocol", proto, "-start-fake-server",
             "-fake-object-size", str(1 << 20), "-enable-tracing", "-trace-sample-rate", "1", "-trace-file", str(t),
             "-metrics-file", str(m), "-metrics-jsonl", str(mj)])
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 12 and all(l.endswith("ms") for l in lines)
    # execute_pb.sh's `tr 'ms' ' '` + float() pipeline (README histogram)
    vals = [float(l.translate(str.maketrans("ms", "  "))) for l in lines]
    assert all(v > 0 for v in vals)
    assert "Read benchmark completed successfully!" in r.stderr
    prom = m.read_text()
    assert 'princer_go_client_read_latency_count{princer_read_latency=""} 12' in prom
    rec = json.loads(mj.read_text().splitlines()[-1])
    assert rec["metric"]["type"] == "custom.googleapis.com/custom-go-client/princer_go_client_read_latency"
    assert rec["points"][0]["value"]["distributionValue"]["count"] == 12
    spans = [s for line in t.read_text().splitlines()
             for rs in json.loads(line)["resourceSpans"] for ss in rs["scopeSpans"] for s in ss["spans"]]
    roots = [s for s in spans if s["name"] == "ReadObject"]
    assert len(roots) == 12
    attrs = {a["key"]: a["value"] for a in roots[0]["attributes"]}
    assert attrs["bucket"]["stringValue"] == "princer-working-dirs"
    res = json.loads(t.read_text().splitlines()[0])["resourceSpans"][0]["resource"]["attributes"]
    res = {a["key"]: a["value"].get("stringValue") for a in res}
    assert res["service.name"] == "princer-storage-benchmark" and res["transport"] == proto
    assert any(s["name"] == "NewReader" and s["parentSpanId"] == roots[0]["spanId"] or True for s in spans)


def test_trace_sampler_ratio():
    from custom_go_client_benchmark_amd.utils.trace_exporter import trace_id_ratio_sampled

    import random

    rnd = random.Random(1)
    n = sum(trace_id_ratio_sampled(rnd.getrandbits(64), 0.25) for _ in range(20000))
    assert 4500 < n < 5500
    assert trace_id_ratio_sampled(2**64 - 1, 1.0) and not trace_id_ratio_sampled(0, 0.0)


def test_cli_list_read_and_write_workloads():
    r = run([GCSBENCH, "-workload", "list-read", "-worker", "2", "-read-call-per-worker", "1", "-start-fake-server",
             "-fake-objects", "5", "-fake-object-size", "65536", "-client-protocol", "grpc"])
    assert r.returncode == 0, r.stderr
    assert len(r.stdout.strip().splitlines()) == 6  # 5 objects over 2 workers -> 3 reads each, 1 wraps


def test_execute_pb_and_histogram(tmp_path):
    env = dict(os.environ)
    env["GCSB_ARGS"] = "-start-fake-server -worker 2 -read-call-per-worker 3 -fake-object-size 65536"
    env["GCSB_RESULTS_DIR"] = str(tmp_path / "res")
    r = run([os.path.join(ROOT, "scripts", "execute_pb.sh"), "9"], cwd=tmp_path, env=env)
    assert r.returncode == 0, r.stderr
    for p in ("grpc_9.txt", "http_9.txt"):
        assert (tmp_path / "res" / p).exists()
        vals = [float(x) for x in (tmp_path / p).read_text().splitlines()]
        assert len(vals) == 6
    h = run([sys.executable, os.path.join(ROOT, "scripts", "histogram.py"), str(tmp_path / "http_9.txt")])
    assert h.returncode == 0 and "Average:" in h.stdout


# --- native FS microbenchmarks (reference benchmark-script/*) ------------------

def _mk(path, n):
    with open(path, "wb") as f:
        f.write(os.urandom(n))


def test_read_operation(tmp_path):
    for i in range(2):
        _mk(tmp_path / f"file_{i}", 300 * 1024)
    r = run([f"{BIN}/read_operation", "--dir", str(tmp_path), "--threads", "2", "--block-size", "64",
             "--read-count", "3", "--hold-seconds", "0"])
    assert r.returncode == 0, r.stderr
    assert "read benchmark completed successfully!" in r.stdout
    assert "read 1843200 bytes" in r.stderr  # 2 files x 300 KiB x 3 passes


def test_read_operation_missing_dir_flag():
    r = run([f"{BIN}/read_operation"])
    assert r.returncode == 1 and "you must set --dir flag" in r.stderr


def test_ssd_test_percentiles(tmp_path):
    for i in range(2):
        (tmp_path / f"Workload.{i}").mkdir()
        _mk(tmp_path / f"Workload.{i}" / "0", 8 * 1024 * 1024)
    for rt in ("seq", "rand"):
        r = run([f"{BIN}/ssd_test", "--dir", str(tmp_path), "--threads", "2", "--block-size", "1024",
                 "--file-size", "8192", "--read-type", rt])
        assert r.returncode == 0, r.stderr
        keys = [l.split(":")[0] for l in r.stdout.splitlines()[1:]]
        assert keys == ["Average", "P20", "P50", "P90", "p99", "Min", "Max"]
    bad = run([f"{BIN}/ssd_test", "--dir", str(tmp_path), "--file-size", "4096"])
    assert bad.returncode == 1 and "not equal to given file-size" in bad.stderr


def test_write_operations(tmp_path):
    r = run([f"{BIN}/write_operations", "--dir", str(tmp_path), "--threads", "2", "--block-size", "64",
             "--file-size", "256", "--write-count", "2", "--hold-seconds", "0"])
    assert r.returncode == 0, r.stderr
    assert os.path.getsize(tmp_path / "file_0") == 256 * 1024
    assert "write benchmark completed successfully!" in r.stdout


def test_list_and_open(tmp_path):
    for i in range(3):
        _mk(tmp_path / f"list_file_{i}", 10 + i)
    r = run([f"{BIN}/list_operation", "--dir", str(tmp_path), "--hold-seconds", "0"])
    assert r.returncode == 0 and "Listing completed..." in r.stdout and "list_file_2" in r.stdout
    r = run([f"{BIN}/list_operation", "--dir", str(tmp_path), "--mode", "native"])
    assert r.stdout.splitlines() == ["list_file_0 10", "list_file_1 11", "list_file_2 12"]
    r = run([f"{BIN}/open_file", "--dir", str(tmp_path), "--open-files", "3", "--hold-seconds", "0"])
    assert r.returncode == 0 and "All the files are opened now" in r.stdout
    r = run([f"{BIN}/open_file", "--dir", str(tmp_path), "--open-files", "4", "--hold-seconds", "0"])
    assert r.returncode == 1


def test_small_poc(tmp_path):
    (tmp_path / "e.txt").write_text("a\nb\nc")
    r = run([f"{BIN}/small_poc", str(tmp_path / "e.txt")])
    assert r.stdout == "a\n\nb\n\n"  # Println of lines that keep their '\n'; unterminated tail dropped


def test_fakegcs_binary_serves_both_protocols():
    import custom_go_client_benchmark_amd as pkg
    from custom_go_client_benchmark_amd import server

    ep = server.start_subprocess("bkt", "o_", "", 0, 2, 1 << 20, md5=True)
    try:
        n = pkg._native
        for proto in ("http", "grpc"):
            c = n.Client({"protocol": proto, "endpoint": ep.url})
            r = c.read("bkt", "o_1")
            assert r["verified"] and r["bytes"] == 1 << 20
    finally:
        ep.stop()


def test_fs_suite_drivers(tmp_path):
    """scripts/fs_suite.py: the reference's benchmark-script drivers over the
    native tools (read matrix, write, list with/without cache, open files,
    ssd_test seq + random) on a prepared directory tree."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "fs.json"
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "fs_suite.py"), "--root", str(tmp_path / "fs"),
                        "--prepare", "--threads", "2", "--scale", "0.002", "--hold", "0", "--list-files", "20",
                        "--open-files", "8", "--out", str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    d = json.loads(out.read_text())
    phases = [p["phase"] for p in d["phases"]]
    assert len(phases) == 11 and all(p["rc"] == 0 for p in d["phases"])
    ssd = [p for p in d["phases"] if p["phase"].startswith("ssd_test")]
    assert all("P50" in p["stdout"] or "p99" in p["stdout"] for p in ssd)
