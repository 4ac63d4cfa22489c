set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06ay
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu.py -m gpu -k "every_variant or rings_on_channel_slice or detect_cls" > $O/tests.txt 2>&1 || exit $?
timeout -k 10 200 python -u scripts/dcls_probe.py --tiles "8,16,8/8,8,8" > $O/dcls.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --hw 80 --batch 32 --codes 0xd41,0xd41,0xd29,0xd21,0xd41,0xd29 --reps 5 > $O/s1_64_80.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 32 --cout 32 --k 3 --hw 160 --batch 32 --codes 0xd45,0xd45,0xd49,0xd41 --reps 5 > $O/s1_32_160.txt 2>&1 || exit $?
FCE_DRING_TIMING=1 timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --hw 80 --batch 32 --codes 0xd41 --reps 2 > $O/t_s1_64_80.txt 2>&1 || exit $?
FCE_FUSE_DCLS=1 FCE_DCLS_DIAG=1 timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'.'); import fce_pkg; fce_pkg.load()
import torch
from fce_yolo_amd.engine import Engine
from fce_yolo_amd.parser import DetectionModel
from fce_yolo_amd.weights import seeded_state_dict
m=DetectionModel('yolo11n-fce.yaml'); m.load_state_dict(seeded_state_dict([(k,v.shape) for k,v in m.state_dict().items()],0)); m.eval().cuda()
x=torch.rand(32,3,640,640).half().cuda()
e=Engine(m,32,640,torch.device('cuda:0'))
e(x,graph=False); torch.cuda.synchronize()
" > $O/dcls_diag.txt 2>&1 || exit $?
