#!/bin/bash
# Build libdbscan_hip.so of git revision $1 into dbscan-on-spark_amd/lib_ab/ for A/B runs on one
# GPU box (DBSCAN_LIB_PATH=dbscan-on-spark_amd/lib_ab/libdbscan_hip.so).  ABFLAGS passes the
# compile-time experiment options of fit.hip, e.g.  ABFLAGS="-DDBSCAN_AB_UNION_W=5" tools/build_ab.sh HEAD
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" dbscan-on-spark_amd/csrc include | tar -x -C "$TMP"
make -s -C "$TMP/dbscan-on-spark_amd/csrc" OUT="$ROOT/dbscan-on-spark_amd/lib_ab" ABFLAGS="$ABFLAGS" -j8
rm -rf "$TMP" "$ROOT"/dbscan-on-spark_amd/lib_ab/*.o
ls -la "$ROOT/dbscan-on-spark_amd/lib_ab/libdbscan_hip.so"
