#!/usr/bin/env python3
"""Summarise rocprofv3 kernel traces / PMC counter CSVs for the CRC kernels.

usage: pmc_summary.py <prof_dir> [<pmc_dir> ...]   -> JSON on stdout
  prof_dir: a --kernel-trace output (…_kernel_trace.csv): per-kernel time and,
            for crc32c_tiles_kernel, the input bytes per dispatch (from the
            bench's known sequence) -> achieved GB/s per dispatch size.
  pmc_dir : --pmc outputs (…_counter_collection.csv): counters summed per
            kernel (rows are per dispatch x counter).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    for k in ("crc32c_tiles_kernel", "crc32c_segments_kernel", "fill_pattern_kernel", "verify_pattern_kernel"):
        if k in name:
            return k
    return name[:60]


def kernel_trace(d):
    out = defaultdict(lambda: {"calls": 0, "ns": 0, "grids": defaultdict(lambda: [0, 0])})
    for p in glob.glob(os.path.join(d, "*_kernel_trace.csv")):
        for r in csv.DictReader(open(p)):
            k = short(r["Kernel_Name"])
            ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            o = out[k]
            o["calls"] += 1
            o["ns"] += ns
            g = o["grids"][r.get("Grid_Size", "?")]
            g[0] += 1
            g[1] += ns
    res = {}
    for k, o in out.items():
        res[k] = {"calls": o["calls"], "total_us": round(o["ns"] / 1e3, 1),
                  "by_grid": {gs: {"calls": c, "avg_us": round(ns / c / 1e3, 2)} for gs, (c, ns) in o["grids"].items()}}
    return res


def counters(d):
    acc = defaultdict(lambda: defaultdict(float))
    meta = {}
    for p in glob.glob(os.path.join(d, "*_counter_collection.csv")):
        for r in csv.DictReader(open(p)):
            k = short(r["Kernel_Name"])
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            meta[k] = {"VGPR": r.get("VGPR_Count"), "AGPR": r.get("Accum_VGPR_Count"), "SGPR": r.get("SGPR_Count"),
                       "LDS_bytes": r.get("LDS_Block_Size"), "workgroup": r.get("Workgroup_Size")}
    res = {}
    for k, c in acc.items():
        c = dict(c)
        if c.get("SQ_INSTS_LDS"):
            c["lds_conflict_cycles_per_lds_instr"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_INSTS_LDS"], 3)
        if c.get("FETCH_SIZE"):
            c["fetch_bytes_x2_note"] = "FETCH_SIZE (KiB) under-reports wide streaming reads by 2x on gfx950"
        res[k] = {"counters": c, "resources": meta.get(k, {})}
    return res


def main():
    out = {}
    for d in sys.argv[1:]:
        if glob.glob(os.path.join(d, "*_kernel_trace.csv")):
            out[os.path.basename(d.rstrip("/")) + ":trace"] = kernel_trace(d)
        if glob.glob(os.path.join(d, "*_counter_collection.csv")):
            out[os.path.basename(d.rstrip("/")) + ":pmc"] = counters(d)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
