#!/bin/bash
# Attribute quarter_union time: 0 full, 1 no unite, 2 no pair test, 3 metadata loads only.
for a in 0 1 2 3 0; do
  DBSCAN_UF_ABLATE=$a timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/abl_$a.log 2>&1 || exit 1
  echo "ablate $a: $(python -c "import json; d=json.loads([l for l in open('gpurun_out/abl_$a.log') if l.startswith('{')][-1]); print(d['stages_ms_per_step'].get('union'), d['config']['clusters'])")"
done
