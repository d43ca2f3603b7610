#!/bin/bash
# hold N open files of listing/100K.  usage: open_file_operation.sh <file_count>
source "$(dirname "$0")/common.sh"
fs_suite --phases open --open-files "${1:?file_count}"
