"""GPU ops: CRC32C kernels, synthetic-pattern fill/verify, HBM landing."""
