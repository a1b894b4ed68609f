#!/bin/bash
# GPU tests, then the default bench under each env setting in AB (space-separated VAR=VAL sets,
# "-" for none).  Each step under its own time limit; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/gpu_tests.log | head -20; exit $rc; }
fi
i=0
for ab in ${AB:--}; do
  i=$((i+1))
  envs=""; [ "$ab" != "-" ] && envs="${ab//,/ }"
  env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab_$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench $ab rc=$rc"; tail -5 gpurun_out/ab_$i.log; exit $rc; }
  echo "[$ab] $(python -c "import json; d=json.loads([l for l in open('gpurun_out/ab_$i.log') if l.startswith('{')][-1]); k=d['kernels_ms_per_step']; print(d['ms_per_step'], sorted(k.items(), key=lambda x:-x[1])[:8])")"
done
