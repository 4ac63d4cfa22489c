"""Run the bench engine's forward a few times (for rocprofv3 --pmc passes on individual kernels)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import fce_pkg  # noqa: E402

fce_pkg.load()
from fce_yolo_amd.engine import Engine  # noqa: E402
from fce_yolo_amd.parser import DetectionModel  # noqa: E402
from fce_yolo_amd.weights import seeded_state_dict  # noqa: E402

dev = torch.device("cuda:0")
model = DetectionModel("yolo11n-fce.yaml")
model.load_state_dict(seeded_state_dict([(k, v.shape) for k, v in model.state_dict().items()], 0))
model.eval().to(dev)
x = torch.rand(32, 3, 640, 640, generator=torch.Generator().manual_seed(1000)).half().to(dev)
eng = Engine(model, 32, 640, dev)
print("launches per forward", sum(q[4] for q in eng.profile(x, launches=True)), flush=True)
for _ in range(3):
    eng(x)
torch.cuda.synchronize()
print("ok")
