import sys, torch
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import cases
from fce_yolo_amd.engine import Engine
import numpy as np
z = np.load("tests/golden/e2e.npz")
fx = {k.split("/",1)[1]: z[k] for k in z.files if k.startswith("yolo11n-fce_160_b2/")}
dev = torch.device("cuda:0")
model = cases.seeded_model("yolo11n-fce.yaml", 0).to(dev)
x = cases.e2e_input("yolo11n-fce_160_b2", fx).to(dev).half()
eng = Engine(model, 2, 160, dev)
yg = eng(x).clone()
ym, maps = model(x)
torch.cuda.synchronize()
d = (yg - ym).abs()
print("max diff", d.max().item(), "rows with diff:", (d.amax(dim=(0,2)) > 0).nonzero().flatten().tolist()[:20])
print("box diff", d[:, :4].max().item(), "cls diff", d[:, 4:].max().item())
a = (d.amax(dim=(0,1)) > 0).nonzero().flatten()
print("anchors differing", a.numel(), a[:10].tolist())
