"""CPU oracle for the FCE-YOLOv11 inference hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the shipped package (`fce-yolo_amd/`)
imports this directory; only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` use it, and only as the checker / the timed
CPU baseline.  It is a from-scratch functional restatement of the reference
(ShioMisaka/fce-yolo, Ultralytics 8.3.242 fork) in PyTorch-CPU ops (conv via
ATen/oneDNN, fp32 or fp64) plus a numpy restatement of the NMS.

Parity pinning: the restatement is checked against golden vectors produced by
running the reference itself in the build container (`tests/golden/make_golden.py`,
fixtures in `tests/golden/*.npz`): per-op outputs, parser layer tables and
state_dict key/shape lists, end-to-end detection outputs and NMS keep indices.
"""
