#!/bin/bash
# Bench lines for the other BASELINE.json configs (parity cases; not the headline line).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cfg
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 "$@" > gpurun_out/cfg/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -c 600 gpurun_out/cfg/$tag.log; echo
  return $rc
}
run s32 --model yolo11s-bifpn.yaml --batch 32 --imgsz 640 &&
run m16 --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280 &&
run l32 --model yolo11l-fce.yaml --batch 32 --imgsz 640
