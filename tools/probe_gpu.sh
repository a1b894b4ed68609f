python -c "import torch; print('torch first:', torch.cuda.is_available(), torch.cuda.device_count())" 2>&1 | grep -v amdgpu.ids
python -c "
import sys; sys.path.insert(0,'dbscan-on-spark_amd')
import dbscan_amd; L=dbscan_amd.load(); print('lib count', L.dbscan_device_count()); h=dbscan_amd.Handle(0)
import torch; print('torch after lib:', torch.cuda.is_available())
" 2>&1 | grep -v amdgpu.ids
env | grep -iE "HIP|ROCR|CUDA|GPU" 
rocm-smi --showuse 2>&1 | head -20
