#!/bin/bash
# Round-2 final measurement, part 2: PMC passes (HBM traffic, MFMA counters) for the n32, l32 and m16 configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_pmc.sh n32 &&
bash scripts/gpu_pmc.sh l32 --model yolo11l-fce.yaml --batch 32 --imgsz 640 &&
bash scripts/gpu_pmc.sh m16 --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280
