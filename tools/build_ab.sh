#!/bin/bash
# Build libdbscan_hip.so variant NAME into dbscan-on-spark_amd/lib_ab/NAME/ for A/B runs on one GPU
# box (tools/ab_bench.sh; DBSCAN_LIB_PATH=dbscan-on-spark_amd/lib_ab/NAME/libdbscan_hip.so).
#   tools/build_ab.sh NAME [REV|WORKTREE]      REV: a git revision (default HEAD); WORKTREE: the
#                                              current csrc, uncommitted edits included
# ABFLAGS passes the compile-time experiment options of fit.hip, e.g.
#   ABFLAGS="-DDBSCAN_AB_UNION_W=5" tools/build_ab.sh w5 HEAD
set -e
NAME=${1:?variant name}
REV=${2:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
if [ "$REV" = WORKTREE ]; then
  mkdir -p "$TMP/dbscan-on-spark_amd" && cp -r "$ROOT/dbscan-on-spark_amd/csrc" "$TMP/dbscan-on-spark_amd/" && cp -r "$ROOT/include" "$TMP/"
else
  git -C "$ROOT" archive "$REV" dbscan-on-spark_amd/csrc include | tar -x -C "$TMP"
fi
OUT="$ROOT/dbscan-on-spark_amd/lib_ab/$NAME"
mkdir -p "$OUT"
make -s -C "$TMP/dbscan-on-spark_amd/csrc" OUT="$OUT" ABFLAGS="$ABFLAGS" -j8
rm -rf "$TMP" "$OUT"/*.o
ls -la "$OUT/libdbscan_hip.so"
