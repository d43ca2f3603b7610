#!/bin/bash
# ssd_test seq + random block reads of ssd/Workload.<i>/0 (the reference had no
# driver of its own: SURVEY.md Q18).  usage: ssd_test.sh <threads> [block_kb] [file_kb]
source "$(dirname "$0")/common.sh"
args=(--phases ssd --threads "${1:?threads}")
[ -n "${2:-}" ] && args+=(--ssd-block-kb "$2")
[ -n "${3:-}" ] && args+=(--ssd-file-kb "$3")
fs_suite "${args[@]}"
