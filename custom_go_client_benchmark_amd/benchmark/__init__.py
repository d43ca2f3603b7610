"""bench.py's rank logic (rank.py) and its output line / sidecar (report.py)."""
