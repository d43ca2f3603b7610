"""Workloads ("models") the benchmark runs.

  read       reference workload: each worker re-reads its own object
             file_<global id> (reference main.go:119-156, 200-210)
  list-read  list a prefix, then read every listed object (config 3; the
             reference does listing/reading through gcsfuse, C14/C17)
  write      upload objects generated in HBM through the pinned ring with a
             resumable session / WriteObject stream (config 5; reference C16
             writes through gcsfuse)
"""
from .workloads import RunOptions, WorkloadResult, run_list_read, run_read, run_write  # noqa: F401
