#!/usr/bin/env python3
"""Latency histogram of a result file (reference README.md:15-35).

Same contract as the README snippet: one float (milliseconds) per line, prints
the average, histogram bins 20, 25, ..., 95 ms.  Additionally prints
p20/p50/p90/p99 (floor-index, as reference ssd_test/main.go:158-161) and
saves the plot to <file>.png (--show to open a window instead).
"""
import sys


def load(path):
    x = []
    with open(path, "r") as f:
        for line in f:
            line = line.strip()
            if line:
                x.append(float(line))
    return x


def main(argv):
    show = "--show" in argv
    paths = [a for a in argv[1:] if not a.startswith("--")]
    if not paths:
        print("usage: histogram.py <latency_file> [--show]", file=sys.stderr)
        return 2
    print(argv)
    bins = [x for x in range(20, 100, 5)]
    x = load(paths[0])
    if not x:
        print("no samples", file=sys.stderr)
        return 1
    print("Average: ", (sum(x) / len(x)))
    s = sorted(x)
    n = len(s)
    for p in (20, 50, 90, 99):
        print(f"P{p}: {s[min(n - 1, n * p // 100)]:.3f} ms")
    try:
        import matplotlib

        if not show:
            matplotlib.use("Agg")
        from matplotlib import pyplot as plt

        plt.hist(x, bins)
        if show:
            plt.show()
        else:
            out = paths[0] + ".png"
            plt.savefig(out)
            print(f"histogram saved to {out}")
    except ImportError:
        print("matplotlib not available: skipped the plot", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
