#!/bin/bash
# PMC passes (hbm/alg, MFMA rate) of the final tree: n32, l32, m16-h8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_pmc.sh n32f && bash scripts/gpu_pmc.sh l32f --model yolo11l-fce.yaml --batch 32 --imgsz 640 &&
bash scripts/gpu_pmc.sh m16f --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280
