#!/bin/bash
# rocprofv3 evidence for the bench workload: kernel-trace stats, then one PMC pass per counter
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950: MI355X_MICROARCH.md §PMC slots).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS="--steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
echo "trace ok"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 || { echo "fetch failed"; tail -20 $OUT/fetch.log; exit 1; }
echo "fetch ok"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1 || { echo "write failed"; tail -20 $OUT/write.log; exit 1; }
echo "write ok"
find $OUT -name "*.csv" | head -20
