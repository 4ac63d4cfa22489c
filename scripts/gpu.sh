#!/bin/bash
# GPU run-tooling in one place (run on the box through gpurun, from the repo root).  Every GPU step runs
# under its own time limit and the first failure (test failures aside) ends the call.
#
#   gpu.sh check TAG                  full -m gpu suite + smoke + the driver's plain `python bench.py`
#   gpu.sh quick TAG "<pytest -k>"    a -k selection of the GPU tests, then a 30-step bench
#   gpu.sh bench TAG [bench args]     one bench line (no CPU baseline, no predict leg)
#   gpu.sh env TAG "A=1 B=2" "A=0" .. one bench line per environment setting, interleaved twice (A/B runs)
#   gpu.sh tune TAG [bench args]      the per-op candidate timings of the planned net (scripts/tune_report.py)
#   gpu.sh configs TAG                bench lines for s32, m16-h8, l32 (BASELINE configs 3-5 on one GPU)
#   gpu.sh prof TAG [bench args]      rocprofv3 kernel trace + stats of the bench (scripts/gpu_prof.sh)
#   gpu.sh pmc TAG [bench args]       FETCH / WRITE / MFMA counter passes (scripts/gpu_pmc.sh)
#
# Output goes to gpurun_out/TAG/; copy the summaries worth keeping into profiles/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CMD=$1
TAG=${2:-run}
shift 2 2>/dev/null || shift $#
OUT=gpurun_out/$TAG
mkdir -p "$OUT"

pytest_gpu() {  # $1 log, rest: pytest args
  local log=$1
  shift
  timeout -k 10 900 python -u -m pytest tests -v -m gpu -rf --timeout 120 --timeout-method thread "$@" > "$log" 2>&1
  local rc=$?
  echo "pytest rc=$rc $(tail -1 "$log")"
  return $rc
}

bench_line() {  # $1 log, rest: bench args
  local log=$1
  shift
  timeout -k 10 400 python bench.py "$@" > "$log" 2>&1
  local rc=$?
  echo "bench rc=$rc $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"forward_ms_per_batch": [0-9.]*\|"frac": [0-9.]*' "$log" | tr '\n' ' ')"
  return $rc
}

case "$CMD" in
  check)
    pytest_gpu "$OUT/pytest_gpu.log" || exit $?
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
    rc=$?; echo "smoke rc=$rc $(tail -1 "$OUT/smoke.log")"; [ $rc -eq 0 ] || exit $rc
    t0=$(date +%s.%N)
    bench_line "$OUT/bench_default_cmd.log" || exit $?
    echo "bench wall $(python -c "import time; print(round(time.time() - $t0, 1))") s"
    ;;
  quick)
    K=${1:-nms}
    shift
    pytest_gpu "$OUT/pytest.log" -k "$K"
    rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
    bench_line "$OUT/bench.log" --steps 30 --warmup 5 --cpu-seconds 0 --predict-steps 0 --dist-config-steps 0 --profile-json "$OUT/profile.json" "$@"
    ;;
  bench)
    bench_line "$OUT/bench.log" --cpu-seconds 0 --predict-steps 0 --dist-config-steps 0 --profile-json "$OUT/profile.json" "$@"
    ;;
  env)
    i=0
    for rep in 1 2; do
      for setting in "$@"; do
        i=$((i + 1))
        echo -n "[$setting] "
        env $setting timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 --predict-steps 0 --dist-config-steps 0 \
          --profile-passes 3 $BARGS > "$OUT/env$i.log" 2>&1
        rc=$?
        echo "rc=$rc $(grep -o '"value": [0-9.]*\|"forward_ms_per_batch": [0-9.]*\|"value_1lane": [0-9.]*' "$OUT/env$i.log" | tr '\n' ' ')"
        [ $rc -eq 0 ] || exit $rc
      done
    done
    ;;
  tune)
    timeout -k 10 400 python -u scripts/tune_report.py "$@" > "$OUT/tune.txt" 2>&1
    rc=$?; echo "tune rc=$rc"; exit $rc
    ;;
  configs)
    for cfg in "s32 --model yolo11s-bifpn.yaml" "m16 --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280" \
               "l32 --model yolo11l-fce.yaml"; do
      set -- $cfg
      t=$1
      shift
      echo -n "$t "
      bench_line "$OUT/$t.log" --steps 30 --warmup 5 --cpu-seconds 0 --predict-steps 0 --dist-config-steps 0 "$@" || exit $?
    done
    ;;
  prof)
    bash scripts/gpu_prof.sh "$TAG" "$@"
    ;;
  pmc)
    bash scripts/gpu_pmc.sh "$TAG" "$@"
    ;;
  *)
    sed -n '2,13p' "$0"
    exit 2
    ;;
esac
