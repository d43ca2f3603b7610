"""The bench line and its sidecar: pure functions, no torch, no native code.

The driver reads ONE JSON line from the tail of bench.py's stdout (the last
8 KiB of it), so the line carries the driver keys first and then scalars
only: per side block `ok`, `mib_s`, `p50_ms`, `p99_ms`, its bound / twin
ratios and at most 3 slowest reads.  Everything else the blocks measure --
per-thread CPU tables, IRQ / softirq views, HTTP/2 reader splits, NUMA and
placement, per-chunk windows -- goes to the sidecar file (`--diag-out`).

Reference timed region: /root/reference/main.go:133-146 (request -> last
byte, io.Discard sink); the reference prints no summary line at all.
"""
from __future__ import annotations

import json

# the driver's stdout tail is 8 KiB; the line must fit with room to spare
LINE_LIMIT = 8192
LINE_TARGET = 6144

DRIVER_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
               "scaling", "vs_baseline", "dtype", "data", "config", "p50_ms", "p99_ms")

# per side block, the scalars that go on the line (everything else: sidecar)
BLOCK_KEYS = ("ok", "mib_s", "p50_ms", "p99_ms", "protocol", "workers", "sink", "streams_per_read", "parts",
              "frac_of_bound", "bound", "vs_discard_twin", "vs_ref_effective", "recv_cpu_s_per_gib",
              "py_cpu_s_per_gib", "first_read_p50_ms", "steady_p99_ms", "list_ms", "per_gpu_mib_s",
              "crc_verified_ranks", "tcp_gbps", "tcp_gbps_same", "memcpy_gbps", "h2d_gbps", "bound_gbps", "headline_frac_of_ceiling",
              "h2_frames", "vs_baseline_paired", "partial", "error")

# receiving threads, in order of preference: the HTTP/2 connection reader
# (gRPC) or the worker that recv()s its own HTTP/1.1 stream
RECV_THREADS = ("gcsb-h2-reader", "gcsb-worker", "gcsb-worker (exited)")


def mib_s(st: dict) -> float:
    """Whole-job MiB/s of a reduced block: all ranks' bytes over the slowest
    rank's elapsed time."""
    return st["nbytes_sum"] / max(st["elapsed_max"], 1e-12) / (1 << 20)


def median(xs: list[float]) -> float | None:
    s = sorted(x for x in xs if x is not None)
    if not s:
        return None
    m = len(s) // 2
    return s[m] if len(s) % 2 else 0.5 * (s[m - 1] + s[m])


def chunk_sizes(steps: int, chunks: int) -> list[int]:
    """`steps` reads split into at most `chunks` near-equal chunks (larger
    first): 20 -> [5, 5, 5, 5], 10 -> [3, 3, 2, 2], 2 -> [1, 1]."""
    c = max(1, min(chunks, steps))
    q, r = divmod(steps, c)
    return [q + (1 if i < r else 0) for i in range(c)]


def arm_order(arms: list[str], chunk: int) -> list[str]:
    """Rotation of the arms for chunk i (a Latin square over the chunks), so
    no arm always runs first after the others, or always last."""
    k = chunk % len(arms)
    return arms[k:] + arms[:k]


def paired_summary(chunks: list[dict]) -> dict:
    """Per-chunk rates of the interleaved arms -> the paired estimators.

    chunks: [{"head": mib_s, "base": mib_s, "nodma": mib_s}, ...] (whole-job
    rates of each arm's chunk; an arm may be missing).  vs_baseline_paired is
    the median over chunks of head / base, headline_vs_nodma the median of
    head / nodma: a slow host window hits both arms of its chunk, so it moves
    one pair ratio, not the estimate."""
    def ratios(other: str) -> list[float]:
        return [c["head"] / c[other] for c in chunks if c.get("head") and c.get(other)]
    out = {"chunks": len(chunks)}
    rb, rn = ratios("base"), ratios("nodma")
    if rb:
        out["vs_baseline_paired"] = round(median(rb), 3)
        out["pair_ratios"] = [round(x, 3) for x in rb]
    if rn:
        out["headline_vs_nodma"] = round(median(rn), 3)
        out["nodma_ratios"] = [round(x, 3) for x in rn]
    rt = ratios("tcp")
    if rt:
        # the headline against the raw one-stream TCP probe run between the
        # same chunks (no GPU, no framing), chunk by chunk; the ceiling itself
        # is the best of every probe (unified_ceiling)
        out["headline_vs_tcp_paired"] = round(median(rt), 3)
        out["tcp_ratios"] = [round(x, 3) for x in rt]
    for arm in ("head", "base", "nodma", "tcp"):
        v = [c[arm] for c in chunks if c.get(arm)]
        if v:
            out[f"{arm}_mib_s"] = [round(x, 1) for x in v]
    return out


def read_times(rec: dict) -> list[float]:
    """[ms, TTFB ms, host-landed ms] of one Runner record (drain())."""
    st = rec["start_ns"]
    ms = (rec["end_ns"] - st) / 1e6
    ttfb = (rec["ttfb_ns"] - st) / 1e6 if rec.get("ttfb_ns", 0) > st else 0.0
    host = (rec["host_done_ns"] - st) / 1e6 if rec.get("host_done_ns", 0) > st else ms
    return [round(ms, 3), round(ttfb, 3), round(host, 3)]


def chunk_first_summary(windows: list[dict]) -> dict:
    """Per arm: each chunk's first read against the chunk's median read
    (ms ratios), the first reads' TTFB and host-landed times, and how many
    chunks had their first read as their slowest.  Whether a chunk restart
    costs anything, and where (connection / TTFB, receive / host-landed, or
    the GPU's copy + CRC after the last host byte)."""
    out = {}
    for arm in ("head", "base"):
        ws = [w for w in windows if w.get("arm") == arm and w.get("reads_ms")]
        if not ws:
            continue
        ratios, slowest_first = [], 0
        for w in ws:
            r = w["reads_ms"]
            med = median(r)
            if med:
                ratios.append(round(w["first_read"][0] / med, 3))
            if len(r) > 1 and w["first_read"][0] >= max(r):
                slowest_first += 1
        out[arm] = {"first_vs_median": ratios, "first_is_slowest": slowest_first, "chunks": len(ws),
                    "first_ttfb_ms": [w["first_read"][1] for w in ws],
                    "first_host_ms": [w["first_read"][2] for w in ws],
                    "start_delay_ms": [w.get("start_delay_ms") for w in ws]}
    return out


def frac_of_bound(block_mib_s: float, h2d_gbps: float, tcp_gbps: float, connections: int | None,
                  gpu_sink: bool) -> dict:
    """A GPU-sink block's bound: the pinned -> HBM copy rate, and for blocks
    on ONE connection (one stream, or gRPC pool 1 multiplexing every worker)
    also the in-run one-connection TCP ceiling -- a ceiling, never a twin's
    rate.  Blocks on many connections are bounded by h2d alone (the
    one-stream TCP probe says nothing about 48 sockets).  Discard-sink
    blocks are bounded by TCP alone when on one connection."""
    cands = []
    if gpu_sink and h2d_gbps > 0:
        cands.append(("h2d", h2d_gbps))
    if connections == 1 and tcp_gbps > 0:
        cands.append(("tcp_1conn", tcp_gbps))
    if not cands:
        return {}
    name, gbps = min(cands, key=lambda x: x[1])
    bound_mib_s = gbps * 1e9 / (1 << 20)
    return {"bound": name, "bound_mib_s": round(bound_mib_s, 1),
            "frac_of_bound": round(block_mib_s / max(bound_mib_s, 1e-9), 3)}


MIB_PER_GBPS = 1e9 / (1 << 20)


def unified_ceiling(head_mib_s_per_gpu: float, paired_tcp_mib_s: list[float] | None, ceiling: dict | None,
                    world: int, gpu_sink: bool) -> dict:
    """ONE one-stream TCP ceiling per run: the best of
    every loopback TCP probe the process made in the headline's placement --
    the paired chunks' probes (whole-job rates, so / world) and the ceiling
    block's best of three -- and the pinned -> HBM copy rate for a GPU sink.
    headline_frac_of_ceiling = headline per GPU / the lower of the two."""
    probes = [x / max(1, world) for x in (paired_tcp_mib_s or []) if x]
    if ceiling and ceiling.get("ok") and ceiling.get("tcp_gbps"):
        probes.append(ceiling["tcp_gbps"] * MIB_PER_GBPS)
    if not probes:
        return {}
    tcp = max(probes)
    bounds = [("tcp_1conn", tcp)]
    if gpu_sink and ceiling and ceiling.get("ok") and ceiling.get("h2d_gbps"):
        bounds.append(("h2d", ceiling["h2d_gbps"] * MIB_PER_GBPS))
    name, b = min(bounds, key=lambda x: x[1])
    out = {"tcp_best_mib_s": round(tcp, 1), "tcp_probes": len(probes), "ceiling_bound": name,
           "ceiling_mib_s": round(b, 1)}
    if head_mib_s_per_gpu > b:
        # the headline did what the probe said one stream cannot: the probe
        # was no ceiling; the observed rate is
        out["ceiling_observed"] = "headline"
        b = head_mib_s_per_gpu
    out["headline_frac_of_ceiling"] = round(head_mib_s_per_gpu / max(b, 1e-9), 3)
    return out


def observed_bounds(blocks: dict[str, dict], head: tuple[float, str, float] | None = None) -> dict:
    """A bound no measured rate may beat: per bound (name, rate), if any block
    -- or the headline, head = (MiB/s per GPU, bound name, bound MiB/s) --
    ran faster than the probe, that rate is what one connection / the copy
    engines did in this process, so the bound becomes it and every block of
    that bound is re-divided (`bound_observed` names the block that set it).
    Mutates the blocks' frac_of_bound / bound_mib_s; returns {bound key:
    observed MiB/s} for the raised ones."""
    groups: dict[tuple, list] = {}
    for k, b in blocks.items():
        if b.get("bound") and b.get("bound_mib_s") and b.get("mib_s") is not None:
            groups.setdefault((b["bound"], b["bound_mib_s"]), []).append(k)
    raised = {}
    for (name, bmib), keys in groups.items():
        best_k = max(keys, key=lambda k: blocks[k]["mib_s"])
        best = blocks[best_k]["mib_s"]
        if head and head[1] == name and abs(head[2] - bmib) < 0.5 and head[0] > best:
            best, best_k = head[0], "headline"
        if best <= bmib:
            continue
        raised[f"{name}@{bmib}"] = round(best, 1)
        for k in keys:
            blocks[k]["bound_mib_s"] = round(best, 1)
            blocks[k]["frac_of_bound"] = round(blocks[k]["mib_s"] / best, 3)
            blocks[k]["bound_observed"] = best_k
    return raised


def recv_cost(cpu: dict) -> float | None:
    """The receiving thread's CPU-s per GiB from a block's by-name table."""
    by = cpu.get("cpu_s_per_gib_by_name") or {}
    for name in RECV_THREADS:
        if by.get(name):
            return float(by[name])
    return None


def receiver_interference(head_cpu: dict, base_cpus: list[dict]) -> dict:
    """The receiving thread's CPU-s per GiB in the headline against the same
    thread in the bracketing baseline runs (both copy every byte out of one
    socket on the same core).  Normally 0.9 - 1.0 (profiles/r4_dist); a
    headline whose receiver cost several times its baseline's while it never
    waited for a CPU ran under host interference (profiles/r4_dist b_4: 3.3x,
    host-wide page faults 10x, function-call IPIs 2x on the placement)."""
    h = recv_cost(head_cpu)
    b = [c for c in (recv_cost(x) for x in base_cpus) if c]
    if not h or not b:
        return {}
    ratio = h / (sum(b) / len(b))
    out = {"cpu_s_per_gib": round(h, 4), "baseline_cpu_s_per_gib": round(sum(b) / len(b), 4),
           "cost_ratio": round(ratio, 2)}
    clock = (head_cpu.get("host") or {}).get("clock_mhz_on_placement") or {}
    for k, v in ((head_cpu.get("host") or {}).get("threads") or {}).items():
        if k.startswith(("gcsb-h2-reader", "gcsb-worker")) and v.get("last_cpus"):
            c = clock.get(str(v["last_cpus"][0]))
            if c:
                # the receiving core's clock through the headline
                out["clock_mhz"] = c["mean"]
                out["clock_mhz_min"] = c["min"]
            break
    if ratio >= 2.0:
        th = ((head_cpu.get("host") or {}).get("threads") or {})
        rd = max((v.get("run_delay_ms_per_read", 0.0) for k, v in th.items() if k.startswith("gcsb-h2-reader")
                  or k.startswith("gcsb-worker")), default=0.0)
        out["note"] = ("receive copy ran {:.1f}x its same-run baseline cost per GiB on the same core, run-queue delay "
                       "{:.2f} ms per read, host-wide page faults {} over the headline: host interference, not the "
                       "client path".format(ratio, rd, (head_cpu.get("host_vmstat") or {}).get("pgfault", "n/a")))
    return out


def window_cause(w: dict, typical_recv: float | None) -> str:
    """Names what made one paired chunk slow from its window fields (the
    receiving thread's CPU-s/GiB against the run's median, its core's clock,
    NUMA page migrations, compaction stalls and TCP retransmits during the
    chunk)."""
    causes = []
    mhz, mhz_ref = w.get("clock_mhz"), w.get("clock_mhz_ref")
    if mhz and mhz_ref and mhz < 0.9 * mhz_ref:
        causes.append(f"receiving core clock {mhz} MHz (run median {mhz_ref})")
    if w.get("numa_pages_migrated", 0) > 0:
        causes.append(f"{w['numa_pages_migrated']} NUMA page migrations")
    if w.get("compact_stall", 0) > 0:
        causes.append(f"{w['compact_stall']} compaction stalls")
    rc = w.get("recv_cpu_s_per_gib")
    if rc and typical_recv and rc > 1.25 * typical_recv:
        causes.append(f"receive copy {rc / typical_recv:.2f}x its median CPU per GiB (memory-side contention "
                      f"or co-tenant)")
    if w.get("run_delay_ms", 0) > 1.0:
        causes.append(f"receiving thread waited {w['run_delay_ms']:.1f} ms for a CPU")
    if w.get("tcp_retrans", 0) > 0:
        causes.append(f"{w['tcp_retrans']} TCP retransmits (loopback reordering)")
    return "; ".join(causes) or "none named"


def attribute_windows(windows: list[dict], slow_frac: float = 0.85) -> list[dict]:
    """Marks the chunks whose headline rate is below `slow_frac` of the run's
    median chunk and names their cause (window_cause).  Nothing is dropped or
    re-run: the slow chunk stays in the headline."""
    rates = [w.get("mib_s") for w in windows if w.get("arm") == "head" and w.get("mib_s")]
    med = median(rates)
    recv = median([w.get("recv_cpu_s_per_gib") for w in windows if w.get("recv_cpu_s_per_gib")])
    mhz = median([w.get("clock_mhz") for w in windows if w.get("clock_mhz")])
    out = []
    for w in windows:
        if w.get("arm") != "head" or not med or not w.get("mib_s"):
            continue
        if w["mib_s"] < slow_frac * med:
            out.append({"chunk": w.get("chunk"), "mib_s": w["mib_s"], "median_mib_s": round(med, 1),
                        "cause": window_cause({**w, "clock_mhz_ref": mhz}, recv)})
    return out


def compact_block(full: dict, max_slowest: int = 3) -> dict:
    """The line's view of one side block: BLOCK_KEYS scalars, error trimmed,
    the slowest reads as [index, ms] rows."""
    d = {k: full[k] for k in BLOCK_KEYS if k in full and full[k] is not None}
    if "error" in d:
        d["error"] = str(d["error"])[:160]
    rows = full.get("rank0_slowest") or []
    if rows and max_slowest > 0:
        d["rank0_slowest"] = [[r[0], r[1]] if isinstance(r, (list, tuple)) and len(r) > 1 else r
                              for r in rows[:max_slowest]]
    return d


def _size(obj: dict) -> int:
    return len(json.dumps(obj).encode())


def fit_line(out: dict, blocks: dict[str, dict], target: int = LINE_TARGET, limit: int = LINE_LIMIT) -> dict:
    """out (headline keys) + compact blocks, shrunk until it serializes to
    at most `target` bytes if it can, and never more than `limit`: first the
    blocks' slowest rows go, then their secondary scalars, then the
    headline's optional keys.  The driver keys are never dropped."""
    line = dict(out)
    comp = {k: compact_block(v) for k, v in blocks.items()}
    line.update(comp)
    if _size(line) <= target:
        return line
    for k in comp:  # 1: slowest rows of the side blocks
        comp[k].pop("rank0_slowest", None)
    line.update(comp)
    if _size(line) <= target:
        return line
    core = ("ok", "mib_s", "p50_ms", "p99_ms", "frac_of_bound", "vs_discard_twin", "vs_ref_effective",
            "recv_cpu_s_per_gib", "headline_frac_of_ceiling", "vs_baseline_paired", "h2_frames", "error")
    for k in comp:  # 2: side blocks down to their core scalars
        comp[k] = {f: v for f, v in comp[k].items() if f in core}
    line.update(comp)
    for opt in ("paired", "rank0_slowest", "per_rank_mib_s", "baseline"):  # 3: headline extras
        if _size(line) <= target:
            break
        if opt in line and _size(line) > target:
            if opt == "per_rank_mib_s" and isinstance(line[opt], list) and len(line[opt]) > 2:
                v = line[opt]
                line[opt] = [min(v), max(v)]
            elif opt == "baseline":
                line[opt] = {k: line[opt][k] for k in ("mib_s", "p50_ms") if k in line[opt]}
            else:
                line.pop(opt)
    if _size(line) > limit:  # 4: side blocks down to ok + rate (largest first)
        for k in sorted(comp, key=lambda k: -_size(comp[k])):
            line[k] = {"ok": comp[k].get("ok"), "mib_s": comp[k].get("mib_s")}
            if _size(line) <= limit:
                break
    if _size(line) > limit:  # 5: never an over-long line: the driver keys alone
        line = {k: out[k] for k in DRIVER_KEYS if k in out}
        line["truncated"] = "side blocks dropped to fit the driver's 8 KiB tail (see the sidecar)"
    return line


def ordered(line: dict) -> dict:
    """Driver keys first (the driver and a human reading the tail see them
    first), everything else after in insertion order."""
    out = {k: line[k] for k in DRIVER_KEYS if k in line}
    out.update({k: v for k, v in line.items() if k not in out})
    return out
