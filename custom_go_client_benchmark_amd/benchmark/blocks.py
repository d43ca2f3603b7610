"""The bench's side blocks and the paired headline, as a mixin of
RankBench (split out of rank.py): the reference-semantics twins, the
reference's default experiment at 1 MiB and 100 MiB, config 3's list-read,
config 5's upload, the fan-out all-gather and the in-run ceilings.  Each
block cites the reference lines it models."""
from __future__ import annotations

import os
import time

from . import report as rp
from .hostio import Meter, parse_size, vmstat


class SideBlocks:
    """Methods of RankBench that build one block each (self is a RankBench)."""

    # ------------------------------------------------------ paired headline
    def paired_headline(self, head_over: dict, base_over: dict, nodma_over: dict | None, steps: int,
                        warmup: int, chunks: int, probe_tcp: bool = True, what: str = "paired") -> tuple[dict, dict]:
        """The headline's `steps` timed reads in `chunks` chunks, each chunk
        followed -- in a rotating order -- by a chunk of the same size of the
        reference-semantics baseline and of the never-DMA-read twin.  Only
        the headline's chunks count toward its value and ms_per_step.

        Every arm's chunk is preceded by --paired-rewarm untimed reads of
        that arm (outside the barriers): the reference reads back to back
        (/root/reference/main.go:127-153), and a chunk's first read otherwise
        paid for the connection, ring and copy engines having idled through
        the other arms' chunks (round 5: the slowest timed reads were the
        chunk-first ones).  Each head / base chunk window
        carries its first read's latency, TTFB and host-landed time and the
        workers' hand-off delay, so that cost stays visible.
        Returns (headline block stats, paired summary + per-chunk windows)."""
        from ..utils import sysdiag

        arms = {"head": head_over, "base": base_over}
        if nodma_over is not None:
            arms["nodma"] = nodma_over
        rewarm = max(0, int(getattr(self.args, "paired_rewarm", 1)))
        runners, errs = {}, {}
        for a, over in arms.items():
            # per-read records of the chunk arms (a few dozen reads): each
            # chunk's first read is reported on its window
            runners[a], errs[a] = self.open_runner({**over, "keep_records": True},
                                                   warmup if a == "head" else self.side_warm)
            if runners[a] is not None:
                runners[a].drain()
        meters = {a: Meter() for a in arms}
        ep_stats = self.srv.stats
        before = self._counters(ep_stats)
        # the transport counters are process-wide: keep only what moved
        # during the headline's chunks (the twins' chunks run in between)
        acc = {"rv": [0, 0], "rd": {k: 0 for k in before["rd"]}, "h2": {k: 0 for k in before["h2"]},
               "sv": {k: 0 for k in before["sv"] if isinstance(before["sv"][k], (int, float))}}
        elapsed = {a: 0.0 for a in arms}
        sizes = rp.chunk_sizes(steps, chunks)
        rates, windows = [], []
        recv_cpus = self.placement.get("client") or []
        # a fourth arm: the raw one-stream TCP ceiling in the headline's
        # placement (core/ceiling.cc: no GPU, no framing), probed between the
        # same chunks, so the headline's fraction of it is paired too (the
        # ceiling block's single probe after the side blocks drifted above
        # the headline in 2 of 3 runs, profiles/r5_window)
        probe_tcp = probe_tcp and self.use_gpu and self.placement.get("client")
        for ci, k in enumerate(sizes):
            row = {}
            for a in rp.arm_order(list(arms) + (["tcp"] if probe_tcp else []), ci):
                if a == "tcp":
                    t, terr = None, ""
                    try:
                        t = self.n.loopback_ceiling({"mode": "tcp", "object_bytes": self.size, "reads": k,
                                                     "ring_bytes": self.args.slots * parse_size(self.args.slot_bytes),
                                                     "rcvbuf": parse_size(self.args.rcvbuf),
                                                     "recv_cpus": self.placement["client"],
                                                     "send_cpus": self.placement["server"], "ring_pages": 1})
                    except Exception as e:  # noqa: BLE001 - the probe is a side measurement
                        terr = str(e)[:200]
                    # whole-job like the arms' rates: every rank probes its own link
                    mine = t["gbps"] * 1e9 / (1 << 20) if t else 0.0
                    red = self.gdist.reduce_stats(self.ctx, tcp=mine, ok=0.0 if terr else 1.0)
                    if red["ok_min"] >= 1.0:
                        row["tcp"] = red["tcp_sum"]
                        windows.append({"chunk": ci, "arm": "tcp", "reads": k, "mib_s": round(row["tcp"], 1),
                                        "recv_cpu_s_per_gib": round(t["recv_cpu_s_per_gib"], 4)})
                    else:
                        windows.append({"chunk": ci, "arm": "tcp", "error": terr or "a peer's probe failed"})
                    continue
                # light window: the receiving core's clock, host vmstat and
                # the receiving thread's schedstat, outside the CPU bracket
                clock = sysdiag.ClockSampler(recv_cpus[:4]) if recv_cpus and not errs[a] else None
                vm0, sch0, tcp0 = vmstat(), sysdiag.thread_sched(), sysdiag.tcp_snapshot()
                m = meters[a]
                m.last = {}
                if rewarm and not errs[a]:
                    self.untimed_reads(runners[a], rewarm)
                c0 = self._counters(ep_stats, reset_hip=False) if a == "head" else None
                e = self.timed_segment(runners[a], k, f"{what} {a} chunk {ci}", errs[a], m)
                sch1, vm1, tcp1 = sysdiag.thread_sched(), vmstat(), sysdiag.tcp_snapshot()
                if c0 is not None:
                    c1 = self._counters(ep_stats, reset_hip=False)
                    acc["rv"] = [acc["rv"][i] + c1["rv"][i] - c0["rv"][i] for i in range(2)]
                    for g in ("rd", "h2", "sv"):
                        for f in acc[g]:
                            acc[g][f] += c1[g][f] - c0[g][f]
                mhz = clock.report() if clock is not None else {}
                elapsed[a] += e
                # whole-job rate of this arm's chunk: all ranks' bytes over the
                # slowest rank (every rank reads k objects of `size` per worker)
                workers = {**self.cfg, **arms[a]}.get("workers", self.args.workers)
                nbytes = float(k * workers * self.size) if not errs[a] else 0.0
                red = self.gdist.reduce_stats(self.ctx, elapsed=e, nbytes=nbytes, ok=0.0 if errs[a] else 1.0)
                if red["ok_min"] >= 1.0:
                    row[a] = rp.mib_s(red)
                gib = max(k * workers * self.size, 1) / (1 << 30)
                # the receiving thread (the connection's h2 reader, else the
                # worker that recv()s) by schedstat: ns, not 10 ms ticks
                def _d(field, prefix):
                    return sum(y[field] - sch0.get(tid, {}).get(field, 0)
                               for tid, y in sch1.items() if y["name"].startswith(prefix))
                recv = (_d("cpu_ns", "gcsb-h2-reader") or _d("cpu_ns", "gcsb-worker")) / 1e9
                rd = _d("run_delay_ns", ("gcsb-h2-reader", "gcsb-worker"))
                w = {"chunk": ci, "arm": a, "reads": k, "mib_s": round(row.get(a, 0.0), 1),
                     "recv_cpu_s_per_gib": round(recv / gib, 4) if recv else None,
                     "run_delay_ms": round(rd / 1e6, 3),
                     # namespace TCP retransmits in the chunk (loopback: spurious
                     # fast retransmits after reordering, README "Known limits")
                     "tcp_retrans": tcp1.get("RetransSegs", 0) - tcp0.get("RetransSegs", 0)}
                if runners[a] is not None and not errs[a]:
                    recs = sorted(runners[a].drain(), key=lambda x: x["start_ns"])
                    if recs:
                        f0 = recs[0]
                        w["first_read"] = rp.read_times(f0)
                        w["reads_ms"] = [round((x["end_ns"] - x["start_ns"]) / 1e6, 3) for x in recs]
                        if self.last_start_ns:
                            # start() -> the first read's start (the parked workers' wake-up)
                            w["start_delay_ms"] = round((f0["start_ns"] - self.last_start_ns) / 1e6, 3)
                if mhz:
                    w["clock_mhz"] = round(sum(v["mean"] for v in mhz.values()) / len(mhz))
                    w["clock_mhz_min"] = min(v["min"] for v in mhz.values())
                for f in ("numa_pages_migrated", "numa_hint_faults", "compact_stall", "pgfault", "thp_fault_alloc"):
                    if f in vm0 and f in vm1:
                        w[f] = vm1[f] - vm0[f]
                windows.append(w)
            rates.append(row)
        # "before" such that now - before = the headline chunks' deltas
        now = self._counters(ep_stats, reset_hip=False)
        before = {"rv": [now["rv"][i] - acc["rv"][i] for i in range(2)],
                  "rd": {f: now["rd"][f] - acc["rd"][f] for f in acc["rd"]},
                  "h2": {f: now["h2"][f] - acc["h2"][f] for f in acc["h2"]},
                  "sv": {**now["sv"], **{f: now["sv"][f] - acc["sv"][f] for f in acc["sv"]}}}
        head = self.finish_block(runners.pop("head"), errs["head"], head_over, steps, elapsed["head"],
                                 meters["head"], before, ep_stats, None, None)
        out = rp.paired_summary(rates)
        out["rewarm_reads"] = rewarm
        out["chunk_first"] = rp.chunk_first_summary(windows)
        out["windows"] = windows
        out["slow_windows"] = rp.attribute_windows(windows)
        for a in list(runners):
            r = runners.pop(a)
            if r is not None and not errs[a]:
                s = r.summary()
                acfg = {**self.cfg, **arms[a]}
                if acfg.get("gpu_stage") == "none":  # nothing reads the ring: nothing verified
                    acfg = {"sink": "discard", "host_crc": False}
                ok, why = self.read_ok(s, steps * {**self.cfg, **arms[a]}.get("workers", self.args.workers), acfg)
                if not ok:
                    out[f"{a}_error"] = why[:200]
                out[f"{a}_p50_ms"] = round(s["p50_ms"], 3)
                out[f"{a}_recv_cpu_s_per_gib"] = rp.recv_cost(
                    {"cpu_s_per_gib_by_name": {t: v / max(float(s["bytes"]), 1.0) * (1 << 30)
                                               for t, v in meters[a].threads.items()}})
            elif errs[a]:
                out[f"{a}_error"] = errs[a][:200]
            del r
        return head, out

    def untimed_reads(self, r1, reads: int) -> None:
        """`reads` reads per worker of an open runner that count nowhere (a
        failure still fails the block)."""
        r1.set_recording(False)
        try:
            r1.set_reads_per_worker(reads)
            r1.start()
            r1.wait()
        finally:
            r1.set_recording(True)
        r1.drain()

    # ------------------------------------------------------------ endpoints
    def share_endpoint(self):
        """An endpoint of its own on the rank's share of L3 domains: the
        sliced block's 8 send threads, and uploads, whose receive + CRC32C
        on the endpoint is as heavy as the client's send."""
        sh = self.affinity.plan(self.gpu, "share", self.slot) if self.use_gpu else {"client": [], "server": []}
        e = self.n.Server({"port": 0, "md5": False, "cpus": sh["server"], "retain_uploads": False})
        e.start()
        e.add_synthetic(self.bucket, self.prefix, "", self.first, self.args.workers, self.size)
        return e, sh

    # ---------------------------------------------------------------- write
    def write_block(self, steps: int, warmup: int, parts: int = 1) -> dict:
        """Config 5: each rank uploads a 64 MiB object from HBM `steps` times
        (HBM -> pinned ring D2H on a side stream -> resumable upload; the
        object CRC32C is computed on the GPU and checked by the endpoint).
        parts > 1 [extension]: parallel composite upload -- `parts` slices
        uploaded on their own connections, composed server-side, the composed
        CRC32C checked against the combine of the parts' GPU CRCs
        (csrc/storage/sliced.h SlicedWriter)."""
        from ..utils import cpuacct

        args, n, torch, gdist = self.args, self.n, self.torch, self.gdist
        err = ""
        lat = []
        phases = []  # per upload: where its time went (the client's UploadPhases)
        wsize = parse_size(args.write_size)
        astage = getattr(args, "write_async_stage", "on") == "on"
        # staging slot = the largest upload message the transport sends from
        # it (messages never cross a slot; gRPC caps them at 2 MiB)
        wslot = parse_size(getattr(args, "write_slot_bytes", args.slot_bytes))
        chunk = parse_size(args.write_chunk)
        client = buf = None
        ep = None
        sh: dict = {}
        saved_aff = os.sched_getaffinity(0)
        gpu, rank = self.gpu, self.rank
        try:
            if parts == 1 and self.use_gpu and args.write_placement == "pair":
                # three quiet cores of one L3 domain: the uploader (this
                # thread) on one, the endpoint's receive and CRC threads on
                # the other two (profiles/r3_write/placement).  Each of the
                # two on a physical core of its own: left to the scheduler
                # over both cores' four hardware threads, the receive thread
                # -- the upload's bound -- often shared its core with the CRC
                # worker, and its cost per GiB swung 0.040 - 0.057 between
                # runs while the raw probe's receiver stayed at 0.037 (r6_t)
                pl = self.affinity.plan(gpu, "pair", self.slot)
                own = getattr(args, "write_crc_core", "own") == "own" and pl.get("aux")
                sh = {"client": pl["client"],
                      "server": pl["server"] if own else sorted(pl["server"] + pl.get("aux", []))}
                ep = n.Server({"port": 0, "md5": False, "cpus": sh["server"], "send_cpus": sh.get("send_cpus"),
                               "crc_cpus": pl["aux"] if own else None, "retain_uploads": False,
                               "write_verify": getattr(args, "write_verify", "on") == "on"})
                ep.start()
            elif parts > 1 and self.use_gpu and getattr(args, "write_composite_placement", "share") != "share":
                sh = self.affinity.plan(gpu, args.write_composite_placement, self.slot)
                ep = n.Server({"port": 0, "md5": False, "cpus": sh["server"], "retain_uploads": False,
                               "write_verify": getattr(args, "write_verify", "on") == "on"})
                ep.start()
            else:
                ep, sh = self.share_endpoint()
            # the upload runs on this (Python main) thread: keep it, its
            # connection reader and the pinned staging ring on the GPU's node
            if sh["client"]:
                os.sched_setaffinity(0, sh["client"])
            client = n.Client({"protocol": self.protocol, "endpoint": ep.url, "retry_initial_s": 0.05,
                               "tcp_congestion": args.client_cc, "loopback_rto_min": True, **self.framing})
            if parts > 1:
                client = n.SlicedWriter({"protocol": self.protocol, "endpoint": ep.url, "retry_initial_s": 0.05,
                                         "tcp_congestion": args.client_cc, "loopback_rto_min": True, **self.framing,
                                         "slices": parts, "slice_min_bytes": 1 << 20, "cpus": sh["client"]})
            buf = torch.empty(wsize, dtype=torch.uint8, device=f"cuda:{gpu}")
            n.gpu_fill_pattern(gpu, buf.data_ptr(), wsize, f"upload/rank{rank}", 0)
            for i in range(warmup):
                client.write_from_device(self.bucket, f"upload/warmup_{rank}_{i}", buf.data_ptr(), wsize, gpu, True,
                                         chunk, wslot, args.slots, astage)
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
        gdist.barrier(self.ctx, "R1 write start barrier")
        self.sync()
        n.reset_slow_hip_calls()
        es0 = ep.stats() if ep is not None and parts == 1 else None
        th0 = cpuacct.thread_cpu()
        t1 = time.perf_counter()
        nbytes = 0
        if not err:
            try:
                for i in range(steps):
                    t0 = time.perf_counter()
                    m = client.write_from_device(self.bucket, f"upload/rank{rank}_{i}", buf.data_ptr(), wsize, gpu,
                                                 True, chunk, wslot, args.slots, astage)
                    lat.append((time.perf_counter() - t0) * 1e3)
                    if m.get("phases"):
                        phases.append(m["phases"])
                    # (SlicedWriter checks the composed CRC32C itself)
                    if m["size"] != wsize or (parts == 1 and m["crc32c"] != m["gpu_crc32c"]):
                        err = f"upload {i} not confirmed: {m}"
                        break
                    nbytes += wsize
            except Exception as e:  # noqa: BLE001
                err = f"{type(e).__name__}: {e}"
        self.sync()
        gdist.barrier(self.ctx, "R2 write stop barrier")
        e1 = time.perf_counter() - t1
        es1 = ep.stats() if es0 is not None else None
        by_name = {k: v - th0.get(k, 0.0) for k, v in cpuacct.thread_cpu().items()}
        cpu_split = {k: round(v / max(nbytes, 1) * (1 << 30), 4) for k, v in sorted(by_name.items())
                     if v > 0.0005 and nbytes}
        # the upload's own bound, outside the timed region: ONE loopback TCP
        # stream in the upload's direction and placement -- the uploader's
        # core sending the upload's own staging pages by reference (a
        # GpuByteSource: this HBM buffer copied D2H into pinned slots, as the
        # transport splices them), the endpoint's cores receiving into a
        # 2 x 2 MiB THP buffer (as its WriteObject receive does); best of 3
        # probes.  The same probe sending the endpoint's THP object (pages no
        # DMA engine wrote) is reported beside it.
        up_tcp = 0.0
        up_probe = {}
        if not err and parts == 1 and sh.get("client") and sh.get("server"):
            try:
                base = {"mode": "tcp", "object_bytes": wsize, "reads": max(3, min(8, steps)),
                        "ring_bytes": 4 << 20, "recv_cpus": sh["server"], "send_cpus": sh["client"], "ring_pages": 1}
                staged = {**base, "gpu_source_ptr": buf.data_ptr(), "gpu_source_device": gpu,
                          "gpu_source_slot_bytes": wslot, "gpu_source_slots": args.slots}
                runs, thp = [], []
                for _ in range(3):
                    runs.append(n.loopback_ceiling(staged))
                    thp.append(n.loopback_ceiling(base))
                best = max(runs, key=lambda r: r["gbps"])
                bthp = max(thp, key=lambda r: r["gbps"])
                up_tcp = best["gbps"] * 1e9 / (1 << 20)
                # the probe's receiver against the endpoint's gcsb-srv-conn
                up_probe = {"source": "gpu_staged",
                            "recv_cpu_s_per_gib": round(best["recv_cpu_s_per_gib"], 4),
                            "send_cpu_s_per_gib": round(best["send_cpu_s_per_gib"], 4),
                            "thp_source_mib_s": round(bthp["gbps"] * 1e9 / (1 << 20), 1),
                            "thp_recv_cpu_s_per_gib": round(bthp["recv_cpu_s_per_gib"], 4)}
            except Exception as e:  # noqa: BLE001 - the probe is a side measurement
                cpu_split["upload_probe_error"] = str(e)[:160]
        s = sorted(lat)
        p50 = s[len(s) * 50 // 100] if s else 0.0
        p99 = s[min(len(s) - 1, len(s) * 99 // 100)] if s else 0.0
        if ep is not None:
            del client
            ep.stop()
        os.sched_setaffinity(0, saved_aff)
        st = gdist.reduce_stats(self.ctx, elapsed=e1, nbytes=float(nbytes), p50=p50, p99=p99, ok=0.0 if err else 1.0,
                                upload_tcp=up_tcp)
        st["error"] = err
        st["slowest"] = [[i, round(v, 2)] for i, v in sorted(enumerate(lat), key=lambda x: -x[1])[:3]]
        st["slow_hip"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in n.slow_hip_calls().items()}
        st["cpu_s_per_gib_by_thread"] = cpu_split
        if up_probe:
            st["upload_probe"] = up_probe
        if es1 is not None and es1.get("write_recvs", 0) > es0.get("write_recvs", 0):
            # the endpoint's WriteObject receive granularity over the timed uploads
            nrecv = es1["write_recvs"] - es0["write_recvs"]
            st.setdefault("upload_probe", {})["endpoint_recv_avg_kib"] = round(
                (es1["write_recv_bytes"] - es0["write_recv_bytes"]) / nrecv / 1024, 1)
        if phases:
            # medians over the timed uploads: the start RPC, the first and
            # last content byte sent, the final response (ms from the start)
            st["phases_ms"] = {k: round(sorted(p[k] for p in phases)[len(phases) // 2], 3) for k in phases[0]}
        return st

    # --------------------------------------------------------------- fanout
    def fanout_block(self, steps: int, warmup: int) -> dict:
        """[extension, N > 1] read once per node, fan out over xGMI: every rank
        reads only its 1/N slice of ONE shared 256 MiB object (ranged gRPC
        read into HBM, per-message CRC32C on the GPU), then an RCCL
        all-gather over the node's GPUs gives every GPU the whole object,
        whose CRC32C each GPU then checks."""
        args, n, torch, gdist, ctx = self.args, self.n, self.torch, self.gdist, self.ctx
        rank, world, size, gpu = self.rank, self.world, self.size, self.gpu
        err = ""
        lat = []
        crc_ok = 0
        part_n = size // world
        name = "fanout/obj_0"
        full = part = sink = client = None
        want = 0
        try:
            if size % world:
                raise ValueError(f"object size {size} not divisible by {world} ranks")
            self.srv.add_synthetic(self.bucket, "fanout/obj_", "", 0, 1, size)
            want = self.srv.object_info(self.bucket, name)["crc32c"]
            client = n.Client({"protocol": self.protocol, "endpoint": self.srv.url, "retry_initial_s": 0.05,
                               "tcp_congestion": args.client_cc, "loopback_rto_min": True,
                               "cpus": self.placement["client"], "rcvbuf": parse_size(args.rcvbuf), **self.framing})
            full = torch.empty(size, dtype=torch.uint8, device=f"cuda:{gpu}" if self.use_gpu else "cpu")
            # this rank's slice lands in place: the all-gather's input is the
            # slice of its output at rank * part_n (in-place all-gather)
            part = full[rank * part_n:(rank + 1) * part_n]
            if self.use_gpu:
                sink = n.GpuSink({"device": gpu, "ring_slot_bytes": parse_size(args.slot_bytes),
                                  "ring_slots": args.slots})
                sink.set_external_destination(part.data_ptr(), size - rank * part_n)
        except Exception as e:  # noqa: BLE001 - reported in the block, collectives still run
            err = f"{type(e).__name__}: {e}"

        for i in range(warmup + steps):
            # every rank makes the same collective calls whatever happened locally
            flags = gdist.reduce_stats(ctx, ok=0.0 if err else 1.0)
            if flags["ok_min"] < 1.0:
                err = err or "a peer rank failed"
                break
            gdist.barrier(ctx, "fan-out start")
            t0 = time.perf_counter()
            local = ""
            try:
                if self.use_gpu:
                    r = client.read_gpu(self.bucket, name, sink, rank * part_n, part_n)
                    if r["bytes"] != part_n or r["crc_mismatch"]:
                        local = f"slice read failed: {r}"
                else:  # CPU rehearsal: the slice through host memory
                    b = client.read_bytes(self.bucket, name, rank * part_n, part_n)
                    part.copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
            except Exception as e:  # noqa: BLE001
                local = f"{type(e).__name__}: {e}"
            try:
                gdist.all_gather_bytes(ctx, full, part, "fan-out all-gather")
                self.sync()
            except Exception as e:  # noqa: BLE001 - the process group is gone: no more collectives
                err = f"all-gather: {type(e).__name__}: {e}"
                return {"ok_min": 0.0, "p50_max": 0.0, "p99_max": 0.0, "crc_ok_sum": 0.0, "nbytes_sum": 0.0,
                        "elapsed_max": 0.0, "error": err}
            gdist.barrier(ctx, "fan-out stop")
            if local:
                err = local
            elif i >= warmup:
                lat.append((time.perf_counter() - t0) * 1e3)
        if not err:
            got = n.gpu_crc32c(gpu, full.data_ptr(), size) if self.use_gpu else n.crc32c(full.numpy().tobytes())
            crc_ok = int(got == want)
            if not crc_ok:
                err = "CRC32C of the gathered object does not match"
        s_ = sorted(lat)
        p50 = s_[len(s_) * 50 // 100] if s_ else 0.0
        p99 = s_[min(len(s_) - 1, len(s_) * 99 // 100)] if s_ else 0.0
        st = gdist.reduce_stats(ctx, elapsed=sum(lat) / 1e3, nbytes=float(size * len(lat)), p50=p50, p99=p99,
                                ok=0.0 if err else 1.0, crc_ok=float(crc_ok))
        st["error"] = err
        del part, full, sink
        return st

    # ------------------------------------------------------------ list-read
    def list_read_block(self, proto: str, warmup_passes: int, extra: dict | None = None) -> dict:
        """Config 3 (BASELINE.json): list `--list-objects` 1 MiB objects, then
        `--list-workers` readers read every listed object once into HBM, GPU
        CRC32C on every read (reference list_operation + read_operation).
        One timed pass after untimed ones; the listing's own time apart."""
        args, n = self.args, self.n
        nobj, workers = args.list_objects, args.list_workers
        # one L3 domain for the readers and the endpoint (profiles/r2_check_s4b, r2_cli_geometry)
        sh = (self.affinity.plan(self.gpu, getattr(args, "list_placement", "same"), self.slot) if self.use_gpu
              else {"client": [], "server": []})
        if self.use_gpu and proto != "http" and args.mux_reader == "isolate":
            sh = self.affinity.isolate_reader(sh)
        if self.use_gpu and proto != "http" and getattr(args, "mux_send", "shared") == "isolate":
            sh = self.affinity.isolate_sender(sh)
        ep = None
        names, list_ms, err = [], 0.0, ""
        rank = self.rank
        try:
            ep = n.Server({"port": 0, "md5": False, "cpus": sh["server"], "send_cpus": sh.get("send_cpus"),
                           "retain_uploads": False})
            ep.start()
            ep.add_synthetic(self.bucket, f"c3_rank{rank}/file_", "", 0, nobj, 1 << 20)
            lister = n.Client({"protocol": proto, "endpoint": ep.url, "retry_initial_s": 0.05, **self.framing})
            t0 = time.perf_counter()
            names = [o["name"] for o in lister.list_all(self.bucket, f"c3_rank{rank}/file_", 1000)]
            list_ms = (time.perf_counter() - t0) * 1e3
            del lister
            if len(names) != nobj:
                err = f"listed {len(names)} of {nobj} objects"
        except Exception as e:  # noqa: BLE001 - reported in the block, collectives still run
            err = f"{type(e).__name__}: {e}"
        per_pass = (nobj + workers - 1) // workers
        lslots, _, lbytes = args.list_ring.partition("x")
        over = {"protocol": proto, "endpoint": ep.url if ep is not None else "", "workers": workers,
                "object_names": names or [f"c3_rank{rank}/file_0"], "cpus": sh["client"], "worker_id_offset": 0,
                "rcvbuf": parse_size(args.list_rcvbuf), "ring_slots": int(lslots), "ring_slot_bytes": parse_size(lbytes),
                "ring_wc": args.list_ring_wc == "on", "reader_cpus": sh.get("reader_cpus"),
                "async_submit": bool(getattr(args, "list_async_submit", 1)),
                "wait_poll_us": int(getattr(args, "list_wait_poll_us", 10))}
        if extra:
            over.update(extra)
        st = self.read_block(over, per_pass, per_pass * warmup_passes, f"{proto} list-read", endpoint=ep)
        if err:
            st["error"] = err
            st["ok_min"] = 0.0
        if ep is not None:
            ep.stop()
        st["list_ms_max"] = self.gdist.reduce_stats(self.ctx, list_ms=list_ms)["list_ms_max"]
        return st

    # -------------------------------------------------------------- ceiling
    def ceiling_block(self, head_mib_s_per_rank: float) -> dict:
        """Same-box bounds: one loopback TCP stream with no GPU and no framing
        (vmsplice/sendfile by a thread on the endpoint's CPUs -> recv() into a
        THP ring by a thread on the client's CPUs, core/ceiling.cc), in the
        headline's placement (tcp_gbps) and in the one-L3-domain placement of
        the multiplexed gRPC blocks (tcp_gbps_same); the client core's memcpy
        rate; pinned -> HBM copies in the sink's pattern (engine.hip
        copy_ceiling)."""
        args, n = self.args, self.n
        err = ""
        r = {"tcp_gbps": 0.0, "tcp_gbps_same": 0.0, "tcp_recv_cpu_s_per_gib": 0.0, "tcp_send_cpu_s_per_gib": 0.0,
             "memcpy_gbps": 0.0, "h2d_gbps": 0.0}
        try:
            ring = args.slots * parse_size(args.slot_bytes)
            reads = max(3, min(10, self.side_steps))

            def tcp(recv_cpus, send_cpus):
                # a ceiling is the best the link did: best of 3 probes (one
                # probe swung +-10% run to run, below the blocks it bounds;
                # best of 2 still sat under the headline in 4 of 20 runs,
                # profiles/r5_window)
                runs = [n.loopback_ceiling({"mode": "tcp", "object_bytes": self.size, "reads": reads,
                                            "ring_bytes": ring, "rcvbuf": parse_size(args.rcvbuf),
                                            "recv_cpus": recv_cpus, "send_cpus": send_cpus, "ring_pages": 1})
                        for _ in range(3)]
                return max(runs, key=lambda x: x["gbps"])
            t = tcp(self.placement["client"], self.placement["server"])
            m = n.loopback_ceiling({"mode": "memcpy", "object_bytes": self.size, "reads": reads, "ring_bytes": ring,
                                    "recv_cpus": self.placement["client"], "ring_pages": 1})
            r.update(tcp_gbps=t["gbps"], tcp_recv_cpu_s_per_gib=t["recv_cpu_s_per_gib"],
                     tcp_send_cpu_s_per_gib=t["send_cpu_s_per_gib"], memcpy_gbps=m["gbps"])
            if self.use_gpu:
                # in the multiplexed blocks' own placement: one L3 domain, the
                # reader and the endpoint's send thread on cores of their own
                # when those blocks isolate them (--mux-reader / --mux-send)
                same = self.affinity.plan(self.gpu, "same", self.slot)
                if args.mux_reader == "isolate":
                    same = self.affinity.isolate_reader(same)
                if getattr(args, "mux_send", "shared") == "isolate":
                    same = self.affinity.isolate_sender(same)
                r["tcp_gbps_same"] = tcp(same.get("reader_cpus") or same["client"][:1],
                                         same.get("send_cpus") or same["server"])["gbps"]
                # pinned -> HBM: the best of the sinks' copy patterns (the
                # headline's 1 MiB x 4 streams, the 48-worker rings' 2 MiB x
                # 8, big copies); the 48-worker HTTP block beat the first alone
                pats = [(parse_size(args.slot_bytes), args.slots, args.slots), (2 << 20, 8, 8), (8 << 20, 8, 8)]
                r["h2d_gbps"] = max(n.copy_ceiling(self.gpu, "h2d", self.size, c, sl, st, 5)["gbps"]
                                    for c, sl, st in pats)
            else:
                r["tcp_gbps_same"] = t["gbps"]
        except Exception as e:  # noqa: BLE001 - reported in the block, collectives still run
            err = f"{type(e).__name__}: {e}"
        st = self.gdist.reduce_stats(self.ctx, ok=0.0 if err else 1.0, **r)
        out = {"ok": st["ok_min"] >= 1.0}
        for k in r:  # the slowest rank's bound (each rank measures its own)
            out[k] = round(st[k + "_min"], 3)
        # (the headline's fraction of the run's ONE ceiling -- the best of
        # these probes and the paired chunks' -- is on the line:
        # report.unified_ceiling)
        head_gbps = head_mib_s_per_rank * (1 << 20) / 1e9
        bounds = [b for b in (out["tcp_gbps"], out["h2d_gbps"] if self.use_gpu else 0.0) if b > 0]
        if bounds:
            out["bound_gbps"] = round(min(bounds), 3)
            out["headline_gbps_per_gpu"] = round(head_gbps, 3)
        if err:
            out["error"] = err[:300]
        return out

    # ---------------------------------------------------------- ref default
    def ref_default_block(self, proto: str, osz: int = 0, reads: int = 0, sink: str = "discard",
                          warmup: int = 2, extra: dict | None = None) -> dict:
        """The reference's only experiment (execute_pb.sh:4,8; main.go:36,
        30,111): -worker 48 readers, each re-reading its own object
        file_<id>, over gRPC with ONE connection (pool 1) or HTTP/1.1
        keep-alive.  sink "discard": io.Discard with the library's host
        CRC32C (reference semantics); "gpu": every read lands in HBM (the
        connection ring for gRPC, a small ring per worker for HTTP) with
        CRC32C on the GPU.  Objects are --ref-object-size or 100 MiB
        (ref_default_100m_*, princer_100M_files, main.go:52)."""
        args, n = self.args, self.n
        workers = args.ref_workers
        osz = osz or parse_size(args.ref_object_size)
        reads = reads or args.ref_reads
        mode = args.ref_grpc_placement if proto != "http" else args.ref_http_placement
        sh = self.affinity.plan(self.gpu, mode, self.slot) if self.use_gpu else {"client": [], "server": []}
        if self.use_gpu and proto != "http" and args.mux_reader == "isolate":
            sh = self.affinity.isolate_reader(sh)
        if self.use_gpu and proto != "http" and getattr(args, "mux_send", "shared") == "isolate":
            sh = self.affinity.isolate_sender(sh)
        ep = None
        err = ""
        prefix = "ref_default/file_" if osz == parse_size(args.ref_object_size) else f"ref_default_{osz >> 20}m/file_"
        try:
            ep = n.Server({"port": 0, "md5": False, "cpus": sh["server"], "send_cpus": sh.get("send_cpus"),
                           "retain_uploads": False})
            ep.start()
            ep.add_synthetic(self.bucket, prefix, "", self.rank * workers, workers, osz)
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
        over = {"protocol": proto, "endpoint": ep.url if ep is not None else "", "workers": workers,
                "object_prefix": prefix, "worker_id_offset": self.rank * workers, "sink": sink,
                "host_crc": sink != "gpu", "cpus": sh["client"],
                # one gRPC connection: the headline's 64 MiB request is one
                # socket's worth; 48 HTTP connections keep autotuning
                "rcvbuf": parse_size(getattr(args, "ref_grpc_rcvbuf", "0")) if proto != "http" else 0,
                "grpc_conn_pool_size": 1,
                "reader_cpus": sh.get("reader_cpus")}
        if sink == "gpu":
            rs, _, rb = args.ref_gpu_ring.partition("x")
            over.update(ring_slots=int(rs), ring_slot_bytes=parse_size(rb), landing="object")
        if extra:
            over.update(extra)
        st = self.read_block(over, reads, warmup, f"{proto} reference default {osz >> 20} MiB {sink}", endpoint=ep)
        if err:
            st["error"] = err
            st["ok_min"] = 0.0
        if ep is not None:
            ep.stop()
        return st

    def baseline_over(self) -> dict:
        # The baseline gets the headline's submitter core too: its host CRC
        # runs on the worker (gRPC: apart from the connection's reader, as
        # the Go library's caller goroutine is apart from grpc-go's transport
        # reader), so both designs get two physical cores.
        over = {"protocol": self.protocol, "sink": "discard", "host_crc": True}
        base_cpus = sorted(set(self.placement.get("client", [])) | set(self.placement.get("aux", [])))
        if base_cpus:
            over["cpus"] = base_cpus
        return over
