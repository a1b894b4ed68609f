set -o pipefail
mkdir -p gpurun_out/y
timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_batch.py tests/test_gpu_parity.py tests/test_gpu_train.py tests/test_gpu_structure.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/y/test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/y/test.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in sk0 sk1; do
DBSCAN_LIB_PATH=dbscan-on-spark_amd/lib_ab/$v/libdbscan_hip.so timeout -k 10 120 python tools/small_stamps.py > gpurun_out/y/$v.$r.txt 2>&1 || exit 1; echo "$v"; grep "^m=" gpurun_out/y/$v.$r.txt
done; done
for v in noskip main; do
lib=""; [ $v != main ] && lib=dbscan-on-spark_amd/lib_ab/$v/libdbscan_hip.so
DBSCAN_LIB_PATH=$lib timeout -k 10 200 python bench.py --seam-only > gpurun_out/y/seam_$v.log 2>&1 || exit 1
echo $v; python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/y/seam_$v.log') if l.startswith('{')][-1])['seam']
print(d['per_call']); print(d['train']['per_partition_calls'], d['train']['batch_device'])"
done
