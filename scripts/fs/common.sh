# Shared by the FS driver wrappers: the reference's benchmark-script/*.sh
# argument shapes over scripts/fs_suite.py.  Environment:
#   GCSB_FS_ROOT      directory / mount point (default ~/gcs, as the reference)
#   GCSB_MOUNT_CMD    e.g. "gcsfuse --stat-cache-ttl 10000m my-bucket {root}" (empty: plain directory)
#   GCSB_UMOUNT_CMD   e.g. "umount {root}"
#   GCSB_FS_PREPARE=1 create the directory layout first;  GCSB_FS_SCALE (default 1.0)
#   GCSB_FS_HOLD      override the tools' pause (seconds)
set -e
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
FS_ROOT="${GCSB_FS_ROOT:-$HOME/gcs}"
fs_suite() {
  local extra=()
  [ "${GCSB_FS_PREPARE:-0}" = "1" ] && extra+=(--prepare)
  [ -n "${GCSB_FS_HOLD:-}" ] && extra+=(--hold "$GCSB_FS_HOLD")
  python3 "$HERE/../fs_suite.py" --root "$FS_ROOT" --scale "${GCSB_FS_SCALE:-1.0}" \
    --mount-cmd "${GCSB_MOUNT_CMD:-}" --umount-cmd "${GCSB_UMOUNT_CMD:-}" "${extra[@]}" "$@"
}
