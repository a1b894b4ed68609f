#!/bin/bash
# Count-pass ablations (timing only): DBSCAN_COUNT_ABLATE=0/1/2 x DBSCAN_COUNT_CAP.
set -o pipefail
mkdir -p gpurun_out
for v in ${CASES:-0:2048 1:2048 2:2048 0:1024 1:1024}; do
  a=${v%%:*}; c=${v##*:}
  DBSCAN_COUNT_ABLATE=$a DBSCAN_COUNT_CAP=$c timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ca_$a_$c.log 2>&1 || exit $?
  echo "ablate=$a cap=$c $(python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ca_$a_$c.log') if l.startswith('{')][-1]); print(d['ms_per_step'], {k: v for k, v in d['stages_ms_per_step'].items() if k in ('count','union_tile','union_edge','output')})")"
done
