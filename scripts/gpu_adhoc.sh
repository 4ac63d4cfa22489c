cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/cfg; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -q -x -k "variant" --timeout 120 --timeout-method thread > gpurun_out/pt_var.log 2>&1; rc=$?; tail -3 gpurun_out/pt_var.log; grep -E "Error|assert" gpurun_out/pt_var.log | head -5; [ $rc -eq 0 ] || exit $rc
for cfg in "l32 --model yolo11l-fce.yaml --batch 32 --imgsz 640" "m16 --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280" "n32"; do
  set -- $cfg; tag=$1; shift
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 "$@" > gpurun_out/cfg/$tag.log 2>&1; rc=$?
  echo "$tag rc=$rc"; grep -o '"value": [0-9.]*\|"forward_ms_per_batch": [0-9.]*\|"conv1x1_mfma": {[^}]*}' gpurun_out/cfg/$tag.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u scripts/tune_report.py --model yolo11l-fce.yaml > gpurun_out/cfg/l32_tune.txt 2>&1; echo tune rc=$?
