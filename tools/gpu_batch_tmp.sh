VARIANTS="base main m5 u2 xg" ROUNDS=2 timeout -k 10 500 bash tools/ab_bench.sh > gpurun_out/ab_r4d.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib/f -o run -- python3 tools/pmc_calibrate.py run > gpurun_out/calib_f.log 2>&1 && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/calib/w -o run -- python3 tools/pmc_calibrate.py run > gpurun_out/calib_w.log 2>&1 && python3 tools/pmc_calibrate.py report gpurun_out/calib > gpurun_out/calib_report.txt 2>&1
DBSCAN_NODE_TRACE=1 timeout -k 10 300 python tools/train_node_probe.py > gpurun_out/train_node_probe.log 2>&1
