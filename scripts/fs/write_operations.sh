#!/bin/bash
# usage: write_operations.sh <threads> <block_size_kb> <file_size_kb> <write_count>
source "$(dirname "$0")/common.sh"
fs_suite --phases write --threads "${1:?threads}" --write-block-kb "${2:?block_size}" \
  --write-file-kb "${3:?file_size}" --write-count "${4:?write_count}"
