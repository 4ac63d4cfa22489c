"""fce_yolo_amd — MI355X-native FCE-YOLOv11 detection inference.

Package directory is ``fce-yolo_amd/``; it is importable as ``fce_yolo_amd`` after
``import fce_pkg; fce_pkg.load()`` (repo root) which registers it under that name.

Layout:
  csrc/       HIP kernels for gfx950 + the C-ABI (include/fce_yolo.h) + the native executor
  _native.py  ctypes binding of libfceyolo.so (fails loudly if it is missing)
  modules.py  drop-in nn.Modules named and shaped like the reference's
  parser.py   the reference YAML parser restated (builds our modules)
  engine.py   whole-graph lowering to the native executor (hipGraph replay) + NMS
  weights.py  portable seeded weights
"""

__version__ = "0.1.0"
