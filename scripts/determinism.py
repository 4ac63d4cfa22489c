"""Run-to-run determinism of the forward: one engine, N forwards of one input, every output against the
first; then two engines on two streams with their forwards in flight together.  Prints mismatch counts
and, for the first mismatch, where it is."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import fce_pkg  # noqa: E402

fce_pkg.load()
from fce_yolo_amd.engine import Engine  # noqa: E402
from fce_yolo_amd.parser import DetectionModel  # noqa: E402
from fce_yolo_amd.weights import seeded_state_dict  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "yolo11n-fce.yaml"
R = int(sys.argv[2]) if len(sys.argv) > 2 else 100
dev = torch.device("cuda:0")
model = DetectionModel(cfg)
model.load_state_dict(seeded_state_dict([(k, v.shape) for k, v in model.state_dict().items()], 0))
model.eval().to(dev)
x = torch.rand(32, 3, 640, 640, generator=torch.Generator().manual_seed(5)).half().to(dev)
e0 = Engine(model, 32, 640, dev)
ref = e0(x).clone()
torch.cuda.synchronize()


def report(tag, y):
    d = (y - ref).abs()
    idx = (d > 0).nonzero()
    print(f"  {tag}: max diff {d.max().item():.3e}, {idx.shape[0]} differ, rows {sorted(set(idx[:, 1].tolist()))[:10]},"
          f" anchors {idx[:, 2].min().item()}..{idx[:, 2].max().item()}, images {sorted(set(idx[:, 0].tolist()))[:8]}",
          flush=True)


bad = 0
for i in range(R):
    y = e0(x)
    if not torch.equal(y, ref):
        if bad == 0:
            report(f"single {i}", y)
        bad += 1
print(f"single engine: {bad} / {R} forwards differ from the first", flush=True)
e1 = Engine(model, 32, 640, dev)
s = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
engs = [e0, e1]
outs = [torch.empty_like(ref) for _ in range(2)]
bad = 0
for i in range(R):
    for k in range(2):
        with torch.cuda.stream(s[k]):
            engs[k](x)
            outs[k].copy_(engs[k].pred)
    torch.cuda.synchronize()
    for k in range(2):
        if not torch.equal(outs[k], ref):
            if bad == 0:
                report(f"dual {i} engine {k}", outs[k])
            bad += 1
print(f"two engines in flight: {bad} / {2 * R} forwards differ", flush=True)
