#!/bin/bash
# read_operation over reading/{256KB,1MB,100MB,1GB} (1000/100/10/1 reads).  usage: read_operations.sh <threads>
source "$(dirname "$0")/common.sh"
fs_suite --phases read --threads "${1:?threads}"
