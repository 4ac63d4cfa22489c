set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06as
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu.py -m gpu -k "detect_cls" > $O/tests.txt 2>&1 || exit $?
for r in 1 2; do
  for d in 0 1; do
    echo "== FCE_DCLS_DWRUN=$d round $r" >> $O/probe.txt
    FCE_DCLS_DWRUN=$d timeout -k 10 200 python -u scripts/dcls_probe.py --tiles "8,16,8/8,8,8" >> $O/probe.txt 2>&1 || exit $?
  done
done
for d in 0 1; do
  echo "== diag FCE_DCLS_DWRUN=$d" >> $O/diag.txt
  FCE_DCLS_DWRUN=$d FCE_FUSE_DCLS=1 FCE_DCLS_DIAG=1 timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'.'); import fce_pkg; fce_pkg.load()
import torch
from fce_yolo_amd.engine import Engine
from fce_yolo_amd.parser import DetectionModel
from fce_yolo_amd.weights import seeded_state_dict
m=DetectionModel('yolo11n-fce.yaml'); m.load_state_dict(seeded_state_dict([(k,v.shape) for k,v in m.state_dict().items()],0)); m.eval().cuda()
x=torch.rand(32,3,640,640).half().cuda()
e=Engine(m,32,640,torch.device('cuda:0'))
e(x,graph=False); torch.cuda.synchronize()
" >> $O/diag.txt 2>&1 || exit $?
done
