mkdir -p gpurun_out/r05dc3
for t in "8,16,4 8,8,4" "8,8,4 8,8,8" "8,16,8 8,8,4"; do
  set -- $t
  FCE_DCLS_TILE_64=$1 FCE_DCLS_TILE_128=$2 FCE_FUSE_DCLS=1 FCE_DCLS_DIAG=1 timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'.'); import fce_pkg; fce_pkg.load()
import torch
from fce_yolo_amd.engine import Engine
from fce_yolo_amd.parser import DetectionModel
from fce_yolo_amd.weights import seeded_state_dict
m=DetectionModel('yolo11n-fce.yaml'); m.load_state_dict(seeded_state_dict([(k,v.shape) for k,v in m.state_dict().items()],0)); m.eval().cuda()
x=torch.rand(32,3,640,640).half().cuda()
e=Engine(m,32,640,torch.device('cuda:0'))
e(x,graph=False); torch.cuda.synchronize()
print('tiles $1 $2', flush=True)
" 2>&1 | grep -v amdgpu.ids || exit 1
done
