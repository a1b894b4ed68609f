VARIANTS="base main sgn xg xgl" ROUNDS=2 timeout -k 10 500 bash tools/ab_bench.sh > gpurun_out/ab_r4f.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_structure.py tests/test_gpu_small.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r4f.log 2>&1
for v in sgn xgl; do DBSCAN_LIB_PATH=dbscan-on-spark_amd/lib_ab/$v/libdbscan_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_structure.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r4f_$v.log 2>&1; done
