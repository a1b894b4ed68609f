timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_structure.py tests/test_gpu_small.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r4c.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 600 --timeout-method thread > gpurun_out/gputest_r4c_cfg.log 2>&1
DBSCAN_LIB_PATH=dbscan-on-spark_amd/lib_ab/stamps/libdbscan_hip.so timeout -k 10 120 python tools/stamps_probe.py > gpurun_out/stamps_r4c.log 2>&1 && VARIANTS="base main xg xgl" ROUNDS=2 timeout -k 10 300 bash tools/ab_bench.sh > gpurun_out/ab_r4c.log 2>&1
timeout -k 10 120 python tools/node_e2e_probe.py > gpurun_out/node_e2e.log 2>&1
