"""Round-4 host-side features on CPU: the endpoint's listener congestion
control (no inherited BBR pacing), FIFO HTTP/2 frame writes with a quantum,
per-read stall attribution (Runner read_diag), client-side
congestion control, and the sysdiag host view."""
import os
import threading

import pytest

B = "princer-working-dirs"
P = "princer_100M_files/file_"


def _softirqs():
    with open("/proc/softirqs") as f:
        lines = f.read().splitlines()
    for line in lines[1:]:
        head, _, rest = line.partition(":")
        if head.strip() == "HRTIMER":
            return sum(int(x) for x in rest.split())
    return 0


def test_endpoint_connections_are_not_paced(native):
    """The endpoint sets its congestion control on the listening socket, so
    accepted connections never run BBR's init (which marks a socket for
    internal pacing that a later TCP_CONGESTION does not undo): a 256 MiB
    gRPC read arms no per-skb pacing hrtimers."""
    with open("/proc/sys/net/ipv4/tcp_congestion_control") as f:
        host_cc = f.read().strip()
    srv = native.Server({"port": 0})
    srv.start()
    srv.add_synthetic(B, P, "", 0, 1, 256 << 20)
    try:
        c = native.Client({"protocol": "grpc", "endpoint": srv.url})
        c.read(B, P + "0")
        h0 = _softirqs()
        for _ in range(2):
            assert c.read(B, P + "0")["verified"]
        per_read = (_softirqs() - h0) / 2
    finally:
        srv.stop()
    if host_cc != "bbr":
        pytest.skip(f"host congestion control is {host_cc}: nothing to inherit")
    # paced: ~4,000 per 256 MiB read (one per 64 KiB skb); unpaced: timer noise only
    assert per_read < 400, per_read


@pytest.mark.parametrize("quantum", [0, 256 << 10])
def test_multiplexed_streams_byte_exact_with_frame_quantum(native, quantum):
    """16 streams on one gRPC connection with the endpoint's DATA frame
    quantum on / off: every read verified; with the quantum the endpoint
    wrote frames of at most 256 KiB (more frames than 2 MiB messages) and
    reports its per-frame queue wait and request -> HEADERS times."""
    srv = native.Server({"port": 0, "h2_quantum": quantum})
    srv.start()
    srv.add_synthetic(B, P, "", 0, 16, (3 << 20) + 77)
    try:
        r = native.Runner({"protocol": "grpc", "endpoint": srv.url, "bucket": B, "object_prefix": P, "workers": 16,
                           "reads_per_worker": 3, "sink": "discard", "host_crc": True, "grpc_conn_pool_size": 1,
                           "keep_records": False})
        r.start()
        r.wait()
        s = r.summary()
        st = srv.stats()
    finally:
        srv.stop()
    assert s["errors"] == 0 and s["verified"] == 48, s
    msgs = 48 * 2  # two ReadObjectResponse messages (2 MiB + the rest) per read
    if quantum:
        # frames are cut to the quantum only while another stream is active
        # (server_grpc.cc send turn): a stream left alone at the end of the
        # run sends whole messages, so the count depends on how the 16 streams
        # finish; at least half the reads were still cut
        assert st["h2_data_frames"] >= 48 * ((3 << 20) // quantum) // 2, st
    else:
        assert st["h2_data_frames"] >= msgs, st
    assert st["h2_responses"] >= 48 and st["h2_ttfb_us"] > 0 and st["h2_queue_wait_max_us"] >= 0


def test_fifo_frame_writes_serve_streams_in_turn(native):
    """Two streams on one connection: with FIFO frame hand-off neither
    stream's reads finish far behind the other's (the old std::mutex let one
    handler keep the connection)."""
    srv = native.Server({"port": 0})
    srv.start()
    srv.add_synthetic(B, P, "", 0, 2, 32 << 20)
    try:
        r = native.Runner({"protocol": "grpc", "endpoint": srv.url, "bucket": B, "object_prefix": P, "workers": 2,
                           "reads_per_worker": 4, "sink": "discard", "host_crc": False, "grpc_conn_pool_size": 1,
                           "keep_records": True})
        r.start()
        r.wait()
        recs = r.drain()
    finally:
        srv.stop()
    assert len(recs) == 8 and all(x["ok"] for x in recs)
    ends = {}
    for x in recs:
        ends.setdefault(x["worker"], []).append(x["end_ns"])
    a, b = (max(v) for v in ends.values())
    first = min(min(v) for v in ends.values())
    # the two workers' last reads end close together relative to the run
    assert abs(a - b) < 0.6 * (max(a, b) - first), (a, b, first)


def test_runner_read_diag_names_threads(native):
    srv = native.Server({"port": 0})
    srv.start()
    srv.add_synthetic(B, P, "", 0, 1, 16 << 20)
    try:
        r = native.Runner({"protocol": "grpc", "endpoint": srv.url, "bucket": B, "object_prefix": P, "workers": 1,
                           "reads_per_worker": 2, "sink": "discard", "read_diag": True, "keep_records": False})
        r.start()
        r.wait()  # warm: the connection (and its reader thread) exist before the timed reads
        r.reset_stats()
        r.set_reads_per_worker(6)
        r.start()
        r.wait()
        s = r.summary()
    finally:
        srv.stop()
    assert len(s["slowest_diag"]) == len(s["slowest"]) == 3
    d = s["slowest_diag"][0]
    assert "gcsb-h2-reader" in d["threads"] and any(k.startswith("gcsb-srv") for k in d["threads"])
    row = d["threads"]["gcsb-h2-reader"]
    assert row["cpu_ms"] > 0 and row["run_delay_ms"] >= 0 and row["cpus"]
    assert d["wall_ms"] >= s["slowest"][0][1] * 0.5
    # namespace TCP counters over the read (loopback: normally no retransmits)
    assert set(d["tcp"]) >= {"RetransSegs", "TCPTimeouts"} and all(v >= 0 for v in d["tcp"].values())
    assert set(d["softnet"]) == {"dropped", "time_squeeze"}
    from custom_go_client_benchmark_amd.utils import sysdiag

    cause = sysdiag.attribute(d, s["slowest"][0][1], s["p50_ms"])
    assert isinstance(cause, str) and cause


def test_attribute_names_run_queue_delay_and_timer_storms():
    from custom_go_client_benchmark_amd.utils import sysdiag

    d = {"threads": {"gcsb-h2-reader": {"cpu_ms": 9.0, "run_delay_ms": 4.0, "nivcsw": 30},
                     "gcsb-srv-rpc": {"cpu_ms": 6.0, "run_delay_ms": 0.1, "nivcsw": 0}},
         "softirqs": {"HRTIMER": 3000, "NET_RX": 4000}, "wall_ms": 14.0}
    c = sysdiag.attribute(d, 14.0, 10.0)
    assert "receiving thread waited 4.00 ms" in c and "HRTIMER" in c
    d = {"threads": {"gcsb-h2-reader": {"cpu_ms": 13.5, "run_delay_ms": 0.0, "nivcsw": 0}}, "softirqs": {},
         "wall_ms": 14.0}
    assert "receive copy itself" in sysdiag.attribute(d, 14.0, 10.0)
    d["tcp"] = {"RetransSegs": 12, "TCPTimeouts": 1, "TCPLossProbes": 0}
    assert "12 TCP retransmits (1 RTOs" in sysdiag.attribute(d, 14.0, 10.0)


def test_client_congestion_control_option(native, server):
    """tcp_congestion is applied before connect; an unknown algorithm is
    ignored by the kernel (setsockopt fails quietly), not fatal."""
    server.add_synthetic(B, P, "", 0, 1, 1 << 20)
    for cc in ("cubic", "reno", "no-such-cc"):
        c = native.Client({"protocol": "grpc", "endpoint": server.url, "tcp_congestion": cc})
        assert c.read(B, P + "0")["verified"]
        data = os.urandom(3 << 20)
        m = c.write_bytes(B, f"upload/cc_{cc}", data)
        assert m["size"] == len(data)


def test_sysdiag_window_reports_threads():
    from custom_go_client_benchmark_amd.utils import sysdiag

    w = sysdiag.Window()
    stop = threading.Event()

    def spin():
        while not stop.is_set():
            pass
    t = threading.Thread(target=spin, name="spinner")
    t.start()
    import time

    time.sleep(0.2)
    rep = w.report(None, 1)
    stop.set()
    t.join()
    assert rep["threads"] and "softirq_on_placement" in rep and "irq_on_placement" in rep


def test_latency_series_bounded_and_accurate(native):
    """The runner's latency series stay exact up to EXACT_CAP samples, then
    switch to a log histogram: memory bounded over the reference's default
    48 x 1,000,000 reads, percentiles within 0.05% of the exact ones."""
    import numpy as np

    rng = np.random.default_rng(7)
    v = np.concatenate([rng.lognormal(0.0, 0.6, native.LatencySeries.EXACT_CAP + 50_000), [250.0]])
    ls = native.LatencySeries()
    ls.extend(v[:1000].tolist())
    s = np.sort(v[:1000])
    assert ls.exact and all(ls.pct_floor(p) == s[min(len(s) - 1, len(s) * p // 100)] for p in (20, 50, 90, 99))
    ls.extend(v[1000:].tolist())
    assert not ls.exact and len(ls) == len(v)
    s = np.sort(v)
    for p in (20, 50, 90, 99):
        want = s[min(len(s) - 1, len(s) * p // 100)]
        assert abs(ls.pct_floor(p) - want) <= 5e-4 * want, (p, ls.pct_floor(p), want)
    assert ls.max == 250.0 and ls.min == s[0]


def test_sysdiag_tcp_counters():
    """Block host view: namespace TCP counters (retransmits, RTOs, receive
    queue prunes / drops), reported as non-zero increases only."""
    from custom_go_client_benchmark_amd.utils import sysdiag

    a = sysdiag.tcp_snapshot()
    assert "RetransSegs" in a and "TCPTimeouts" in a
    b = dict(a, RetransSegs=a["RetransSegs"] + 5, TCPTimeouts=a["TCPTimeouts"] + 1)
    assert sysdiag.tcp_delta(a, b) == {"RetransSegs": 5, "TCPTimeouts": 1}
    assert "tcp" in sysdiag.Window().report(None, 1)
    d = {"threads": {"gcsb-worker": {"cpu_ms": 16.0, "run_delay_ms": 0.0}}, "softirqs": {},
         "tcp": {"RcvPruned": 2, "TCPRcvQDrop": 1}, "wall_ms": 226.0}
    assert "3 receive-queue prunes / drops" in sysdiag.attribute(d, 226.0, 16.0)
    d["softnet"] = {"dropped": 40, "time_squeeze": 2}
    assert "40 packets dropped at a CPU's input backlog" in sysdiag.attribute(d, 226.0, 16.0)
    sn = sysdiag.softnet_snapshot()
    assert sn and all(len(v) == 2 for v in sn.values())
    assert set(sysdiag.Window().report(None, 1)["softnet_on_placement"]) == {"dropped", "time_squeeze"}


def test_endpoint_sockets_get_loopback_rto_min(native, server):
    """The endpoint sets a loopback-sized minimum RTO (TCP_RTO_MIN_US, Linux
    6.15+) on its LISTENING socket, which accepted sockets inherit (checked
    here on a plain listener: the endpoint's fds are not reachable from
    Python), so one receive-queue drop cannot stall a read for 200 ms.
    Client sockets opt in (loopback_rto_min); older kernels refuse the
    option and nothing changes."""
    import socket

    ls = socket.socket()
    try:
        ls.setsockopt(socket.IPPROTO_TCP, 45, native.LOOPBACK_RTO_MIN_US)
    except OSError:
        pytest.skip("kernel without TCP_RTO_MIN_US")
    ls.bind(("127.0.0.1", 0))
    ls.listen()
    c = socket.create_connection(ls.getsockname())
    a, _ = ls.accept()
    assert a.getsockopt(socket.IPPROTO_TCP, 45) <= 10000 < c.getsockopt(socket.IPPROTO_TCP, 45)
    for s_ in (a, c, ls):
        s_.close()
    server.add_synthetic(B, P, "", 0, 1, 1 << 20)
    cl = native.Client({"protocol": "grpc", "endpoint": server.url, "loopback_rto_min": True})
    assert cl.read(B, P + "0")["verified"]


def test_bench_receiver_interference_flag():
    """benchmark.report.receiver_interference: the headline receiver's CPU-s/GiB against
    the same thread in the bracketing baselines; a >= 2x cost names host
    interference (profiles/r4_dist b_4), a normal run carries only the ratio."""
    from custom_go_client_benchmark_amd.benchmark import report as bench
    base = [{"cpu_s_per_gib_by_name": {"gcsb-h2-reader": 0.042}}, {"cpu_s_per_gib_by_name": {"gcsb-h2-reader": 0.038}}]
    ok = bench.receiver_interference({"cpu_s_per_gib_by_name": {"gcsb-h2-reader": 0.038}}, base)
    assert ok["cost_ratio"] == 0.95 and "note" not in ok
    bad = bench.receiver_interference(
        {"cpu_s_per_gib_by_name": {"gcsb-h2-reader": 0.126}, "host_vmstat": {"pgfault": 2311813},
         "host": {"threads": {"gcsb-h2-reader": {"run_delay_ms_per_read": 0.02}}}}, base)
    assert bad["cost_ratio"] == 3.15 and "host interference" in bad["note"] and "2311813" in bad["note"]
    http = bench.receiver_interference({"cpu_s_per_gib_by_name": {"gcsb-worker (exited)": 0.08}},
                                       [{"cpu_s_per_gib_by_name": {"gcsb-worker (exited)": 0.076}}])
    assert http["cost_ratio"] == 1.05
    assert bench.receiver_interference({}, base) == {}


def test_clock_sampler(tmp_path, monkeypatch):
    """sysdiag.ClockSampler: MHz per CPU from the cpufreq files while the
    window is open; none on a host without cpufreq; Window reports it as
    clock_mhz_on_placement, and bench.receiver_interference picks the
    receiving core's clock."""
    import time
    from custom_go_client_benchmark_amd.utils import sysdiag
    f = tmp_path / "freq"
    f.write_text("4800000\n")
    monkeypatch.setattr(sysdiag, "_freq_file", lambda c: str(f) if c == 7 else None)
    s = sysdiag.ClockSampler([7, 8], period_s=0.005)
    time.sleep(0.05)
    f.write_text("2400000\n")
    time.sleep(0.05)
    r = s.report()
    assert list(r) == ["7"] and r["7"]["max"] == 4800 and r["7"]["min"] == 2400 and r["7"]["n"] >= 4
    assert s._thread is None
    assert sysdiag.ClockSampler([8]).report() == {}
    w = sysdiag.Window(clock_cpus=[7])
    time.sleep(0.05)
    rep = w.report([7], 1)
    assert rep["clock_mhz_on_placement"]["7"]["mean"] == 2400
    from custom_go_client_benchmark_amd.benchmark import report as bench
    head = {"cpu_s_per_gib_by_name": {"gcsb-h2-reader": 0.07},
            "host": {"threads": {"gcsb-h2-reader": {"last_cpus": [7]}}, "clock_mhz_on_placement": rep["clock_mhz_on_placement"]}}
    out = bench.receiver_interference(head, [{"cpu_s_per_gib_by_name": {"gcsb-h2-reader": 0.047}}])
    assert out["clock_mhz"] == 2400 and out["cost_ratio"] == 1.49
