set -o pipefail
BENCH_ARGS="--config 3 --steps 5 --warmup 2" bash tools/node_trace.sh > /dev/null || exit 1
timeout -k 10 200 python tools/node_breakdown.py 12500000 > gpurun_out/nodetrace/breakdown.txt 2>&1; echo "bd rc=$?"
cat gpurun_out/nodetrace/breakdown.txt | tail -2
