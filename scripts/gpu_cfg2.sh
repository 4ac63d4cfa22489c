#!/bin/bash
# Variant parity tests + per-config bench lines (m16, l32, s32, n32) with per-op profiles.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/cfg; export TMPDIR=/tmp
TAG=${1:-x}
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -q -k "variant" --timeout 200 --timeout-method thread -rf > gpurun_out/cfg/${TAG}_pt_var.log 2>&1; rc=$?; tail -3 gpurun_out/cfg/${TAG}_pt_var.log; [ $rc -eq 0 ] || exit $rc
run() {
  local tag=$1; shift
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --predict-steps 0 --profile-passes 3 --profile-json gpurun_out/cfg/${TAG}_${tag}_profile.json "$@" > gpurun_out/cfg/${TAG}_$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/cfg/${TAG}_$tag.log | tr '\n' ' ')"
  python -c "import json;d=json.loads(open('gpurun_out/cfg/${TAG}_$tag.log').read().strip().splitlines()[-1]);print({k:(v['ms'],v['TFLOP/s']) for k,v in list(d['kernels'].items())[:4]})" 2>/dev/null
  return $rc
}
run m16 --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280 && run l32 --model yolo11l-fce.yaml --batch 32 --imgsz 640 && run s32 --model yolo11s-bifpn.yaml --batch 32 --imgsz 640 && run n32
