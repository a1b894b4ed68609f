#!/bin/bash
# GPU tests, the default bench, and the skewed config-4 bench (each step under its own limit).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench.log | tail -1
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --points-per-gpu 50000000 --dense 8 --seed 3 > gpurun_out/bench_dense.log 2>&1
rc=$?; echo "dense rc=$rc"; grep '^{' gpurun_out/bench_dense.log | tail -1
exit $rc
