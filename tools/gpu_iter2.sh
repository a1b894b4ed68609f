#!/bin/bash
# GPU tests, then the default bench, the node bench at N = 1 and the dense config-4 bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/gpu_tests.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench.log | tail -1 | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --node --steps 20 --warmup 3 > gpurun_out/bench_node.log 2>&1
rc=$?; echo "node rc=$rc"; grep '^{' gpurun_out/bench_node.log | tail -1 | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --points-per-gpu 50000000 --dense 8 --seed 3 > gpurun_out/bench_dense.log 2>&1
rc=$?; echo "dense rc=$rc"; grep '^{' gpurun_out/bench_dense.log | tail -1 | cut -c1-200
exit $rc
