#!/bin/bash
# ls of listing/<dir>, with and without the mount's caches.  usage: list_operations.sh <dir>
source "$(dirname "$0")/common.sh"
fs_suite --phases list --list-dir "${1:?dir}"
