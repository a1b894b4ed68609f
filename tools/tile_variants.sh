#!/bin/bash
# LDS staging capacity sweep of the per-tile kernels (DBSCAN_COUNT_CAP), after a
# parity pass.  Results are identical for every choice; only the stage times move.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q --timeout 600 > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-3072 2048 1024}; do
  DBSCAN_COUNT_CAP=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/tv_$v.log 2>&1 || exit $?
  echo "$v $(python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/tv_$v.log') if l.startswith('{')][-1]); print(d['ms_per_step'], {k: v for k, v in d['stages_ms_per_step'].items() if k in ('count','union_tile','union_edge','union_root','output')})")"
done
