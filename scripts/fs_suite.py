#!/usr/bin/env python3
"""Filesystem microbenchmark suite: the reference's benchmark-script drivers
(read_operations.sh, write_operations.sh, list_operations.sh,
open_file_operation.sh; ssd_test had none of its own) as one
driver over the native tools in custom_go_client_benchmark_amd/bin.

The reference mounts gcsfuse over a bucket before every phase and unmounts
after it (e.g. benchmark-script/read_operation/read_operations.sh).  There is
no gcsfuse or network here, so the suite runs on any directory tree: pass
--mount-cmd / --umount-cmd to wrap each phase in a mount (the "{root}"
placeholder is substituted), or leave them empty for a local directory.  The
tree is created on demand (--prepare) with the reference's layout:

    reading/{256KB,1MB,100MB,1GB}/file_<i>      read_operation matrix
    listing/<dir>/...  listing/100K/list_file_<i>  list_operation / open_file
    writing/                                    write_operations
    ssd/Workload.<i>/0                          ssd_test

--scale shrinks every size (CI: --scale 0.01) without changing the shape.
Each phase's stdout is kept; a JSON summary goes to --out.

    python scripts/fs_suite.py --root /tmp/fs --prepare --threads 2 --scale 0.01 --hold 0
"""
from __future__ import annotations

import argparse
import json
import os
import shlex
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "custom_go_client_benchmark_amd", "bin")

# reference read_operations.sh matrix: (dir, read-count, block-size KB, file size)
READ_MATRIX = [("256KB", 1000, 256, 256 << 10), ("1MB", 100, 1024, 1 << 20), ("100MB", 10, 1024, 100 << 20),
               ("1GB", 1, 1024, 1 << 30)]


def scaled(n: int, scale: float, floor: int = 4096) -> int:
    return max(floor, int(n * scale) // 4096 * 4096)


def write_file(path: str, size: int):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    if os.path.exists(path) and os.path.getsize(path) == size:
        return
    chunk = os.urandom(min(size, 4 << 20))
    with open(path, "wb") as f:
        left = size
        while left > 0:
            k = min(left, len(chunk))
            f.write(chunk[:k])
            left -= k


def prepare(root: str, threads: int, scale: float, list_files: int, open_files: int, ssd_size: int,
            list_dir: str = "dir"):
    for d, _, _, size in READ_MATRIX:
        for i in range(threads):
            write_file(os.path.join(root, "reading", d, f"file_{i}"), scaled(size, scale))
    for i in range(list_files):
        write_file(os.path.join(root, "listing", list_dir, f"file_{i}"), 4096)
    for i in range(open_files):
        write_file(os.path.join(root, "listing", "100K", f"list_file_{i}"), 4096)
    os.makedirs(os.path.join(root, "writing"), exist_ok=True)
    for i in range(threads):
        write_file(os.path.join(root, "ssd", f"Workload.{i}", "0"), ssd_size)


class Suite:
    def __init__(self, args):
        self.a = args
        self.results = []

    def mount(self, when: str):
        cmd = self.a.mount_cmd if when == "mount" else self.a.umount_cmd
        if cmd:
            subprocess.run(cmd.format(root=self.a.root), shell=True, check=True)

    def run(self, phase: str, argv: list[str]):
        self.mount("mount")
        t0 = time.perf_counter()
        env = dict(os.environ, GODEBUG="asyncpreemptoff=1")  # as the reference drivers set for Go tools
        r = subprocess.run(argv, capture_output=True, text=True, env=env)
        dt = time.perf_counter() - t0
        self.mount("umount")
        rec = {"phase": phase, "cmd": " ".join(shlex.quote(x) for x in argv), "rc": r.returncode,
               "seconds": round(dt, 3), "stdout": r.stdout[-4000:], "stderr": r.stderr[-2000:]}
        self.results.append(rec)
        print(f"LoggerPrince: {phase}: rc={r.returncode} {dt:.2f}s", flush=True)
        if r.returncode != 0:
            print(r.stdout[-2000:], r.stderr[-2000:], file=sys.stderr)
        return rec


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--root", required=True, help="mount point / directory holding the layout")
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--scale", type=float, default=1.0, help="file-size scale factor (CI: 0.01)")
    ap.add_argument("--prepare", action="store_true", help="create the directory layout first")
    ap.add_argument("--list-files", type=int, default=1000)
    ap.add_argument("--list-dir", default="dir", help="listing/<dir> to list (reference list_operations.sh $1)")
    ap.add_argument("--open-files", type=int, default=100)
    ap.add_argument("--hold", type=float, default=None,
                    help="override every tool's --hold-seconds (reference: 10 s / 3 min pauses)")
    ap.add_argument("--write-block-kb", type=int, default=256)
    ap.add_argument("--write-file-kb", type=int, default=1024)
    ap.add_argument("--write-count", type=int, default=1)
    ap.add_argument("--ssd-block-kb", type=int, default=1024)
    ap.add_argument("--ssd-file-kb", type=int, default=None, help="default: 5 GiB x scale")
    ap.add_argument("--phases", default="read,write,list,open,ssd")
    ap.add_argument("--mount-cmd", default="", help='e.g. "gcsfuse --stat-cache-ttl 10000m bucket {root}"')
    ap.add_argument("--umount-cmd", default="", help='e.g. "umount {root}"')
    ap.add_argument("--out", default="")
    a = ap.parse_args()

    ssd_kb = a.ssd_file_kb or max(a.ssd_block_kb, scaled(5 << 30, a.scale, a.ssd_block_kb << 10) >> 10)
    ssd_kb = ssd_kb // a.ssd_block_kb * a.ssd_block_kb
    if a.prepare:
        prepare(a.root, a.threads, a.scale, a.list_files, a.open_files, ssd_kb << 10, a.list_dir)
    hold = [] if a.hold is None else ["--hold-seconds", str(a.hold)]
    s = Suite(a)
    phases = set(a.phases.split(","))
    if "read" in phases:
        for d, count, bkb, _ in READ_MATRIX:
            s.run(f"read {d} x{count}", [os.path.join(BIN, "read_operation"), "--read-count", str(count), "--threads",
                                         str(a.threads), "--block-size", str(bkb), "--dir",
                                         os.path.join(a.root, "reading", d)] + hold)
    if "write" in phases:
        s.run("write", [os.path.join(BIN, "write_operations"), "--threads", str(a.threads), "--block-size",
                        str(a.write_block_kb), "--file-size", str(a.write_file_kb), "--write-count",
                        str(a.write_count), "--dir", os.path.join(a.root, "writing")] + hold)
    if "list" in phases:
        for label in ("with cache", "without cache"):  # the reference remounts with/without gcsfuse caches
            s.run(f"list ({label})", [os.path.join(BIN, "list_operation"), "--dir",
                                      os.path.join(a.root, "listing", a.list_dir)] + hold)
    if "open" in phases:
        for label in ("with cache", "without cache"):
            s.run(f"open_file ({label})", [os.path.join(BIN, "open_file"), "--open-files", str(a.open_files),
                                           "--dir", os.path.join(a.root, "listing", "100K")] + hold)
    if "ssd" in phases:
        for rt in ("seq", "random"):
            s.run(f"ssd_test {rt}", [os.path.join(BIN, "ssd_test"), "--threads", str(a.threads), "--block-size",
                                     str(a.ssd_block_kb), "--file-size", str(ssd_kb), "--read-type", rt,
                                     "--dir", os.path.join(a.root, "ssd")])
    summary = {"root": a.root, "threads": a.threads, "scale": a.scale, "phases": s.results}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(summary, f, indent=1)
    return 0 if all(r["rc"] == 0 for r in s.results) else 1


if __name__ == "__main__":
    sys.exit(main())
