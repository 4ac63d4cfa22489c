"""Convert a reference (Ultralytics / FCE-YOLO) .pt checkpoint to the tensors-only safetensors format that
fce_yolo_amd.weights.load_model reads.  Run ONCE in an environment where the reference package is
importable (it must unpickle the checkpoint's modules — only ever do that for checkpoints you trust):

    python scripts/convert_checkpoint.py best.pt best.safetensors

What it stores (reference nn/tasks.py:1371-1486 attempt_load_one_weight semantics): the EMA model if
present, else 'model', cast to fp32; its YAML dict (model.yaml) and class names as metadata.  Keys are
unchanged (model.N.<...>), so the MI355X DetectionModel of the same YAML loads them as they are.
"""
import json
import sys

import torch
from safetensors.torch import save_file


def main(src, dst):
    ckpt = torch.load(src, map_location="cpu", weights_only=False)  # trusted user checkpoint only
    if isinstance(ckpt, dict):
        model = ckpt.get("ema") if ckpt.get("ema") is not None else ckpt["model"]
    else:
        model = ckpt
    model = model.float()
    sd = {k: v.detach().contiguous() for k, v in model.state_dict().items()}
    yaml_d = {k: v for k, v in dict(model.yaml).items() if k != "yaml_file"}
    names = getattr(model, "names", None) or {i: str(i) for i in range(yaml_d.get("nc", 80))}
    meta = {"fce_yolo.yaml": json.dumps(yaml_d), "fce_yolo.names": json.dumps({str(k): v for k, v in names.items()})}
    save_file(sd, dst, metadata=meta)
    print(f"{src} -> {dst}: {len(sd)} tensors")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
