#!/bin/bash
# Node-path iteration: the GPU tests, then the node bench at N = 1 and the default bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/gpu_tests.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --node --steps 20 --warmup 3 > gpurun_out/bench_node.log 2>&1
rc=$?; echo "node rc=$rc"; grep '^{' gpurun_out/bench_node.log | tail -1 | cut -c1-260
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/host_enqueue.py > gpurun_out/he.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/he.log
exit $rc
