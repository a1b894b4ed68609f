#!/bin/bash
# Kernel timeline of the node step at N = 1 (bench.py --node): one step from grid_kernel to the next.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/nodetrace
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --node ${BENCH_ARGS:---steps 5 --warmup 2} --no-cpu-baseline --e2e-steps 0 --no-seam > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 tools/trace_fit.py "$f" > $OUT/timeline.txt && tail -80 $OUT/timeline.txt && rm -rf $OUT/trace
