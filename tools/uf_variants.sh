#!/bin/bash
# A/B the union-find load/store variants on the bench workload (same box, back to back).
for v in ${VARIANTS:-0 1 4 0 1 4}; do
  DBSCAN_UF_VARIANT=$v timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/uf_$v.log 2>&1 || exit 1
  echo "variant $v: $(python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/uf_$v.log') if l.startswith('{')][-1]); print(d['ms_per_step'], d['stages_ms_per_step'].get('union'), d['stages_ms_per_step'].get('quarter_init'), d['config']['clusters'])") $(grep 'uf stats' gpurun_out/uf_$v.log | tail -1)"
done
