"""Go-compatible flags, metric/trace exporters, latency-file helpers."""
