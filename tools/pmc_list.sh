#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1; echo rc=$?
grep -oE "^\s*(SQ|TCP|TCC|TA|TD|GRBM|SPI)[A-Za-z0-9_]*" gpurun_out/pmc_list.txt | sort -u | head -5
wc -l gpurun_out/pmc_list.txt
