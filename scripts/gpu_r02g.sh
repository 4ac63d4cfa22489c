#!/bin/bash
# Round-2 closing measurement: GPU suite + smoke + bench (gpu_check), rocprof trace/stats of the n32 bench,
# PMC passes for l32 and m16 with the final build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh && bash scripts/gpu_prof.sh r02g &&
bash scripts/gpu_pmc.sh l32 --model yolo11l-fce.yaml --batch 32 --imgsz 640 &&
bash scripts/gpu_pmc.sh m16 --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280
