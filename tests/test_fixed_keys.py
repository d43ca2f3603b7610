"""Every setting the benchmark reads with getattr(args, "<name>", default) is
either a bench.py flag or a benchmark/rank.py FIXED value: a typo in either
place would otherwise fall back to the default silently (the A/B sessions
override FIXED values through GCSB_FIXED, which rejects unknown keys)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_getattr_settings_exist():
    import importlib.util

    from custom_go_client_benchmark_amd.benchmark.rank import FIXED

    spec = importlib.util.spec_from_file_location("bench_main", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    flags = {a.dest for a in bench.build_parser()._actions}
    bdir = os.path.join(ROOT, "custom_go_client_benchmark_amd", "benchmark")
    used = set()
    for f in os.listdir(bdir):
        if f.endswith(".py"):
            used |= set(re.findall(r'getattr\(args, "([a-z_0-9]+)"', open(os.path.join(bdir, f)).read()))
    assert used, "no getattr(args, ...) settings found"
    missing = sorted(k for k in used if k not in flags and k not in FIXED)
    assert not missing, missing
