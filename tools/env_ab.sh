#!/bin/bash
# A/B timing of library environment switches: CASES="VAR=a VAR=b ..." (one bench per case).
set -o pipefail
mkdir -p gpurun_out
for c in $CASES; do
  env $c timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$c.log 2>&1 || exit $?
  echo "$c $(python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_$c.log') if l.startswith('{')][-1]); print(d['ms_per_step'], d['stages_ms_per_step'])")"
done
