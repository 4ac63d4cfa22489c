set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06aa
mkdir -p $O
for rep in 1 2; do
for cfg in "n32 --steps 100" "l32 --model yolo11l-fce.yaml --steps 30"; do
  set -- $cfg; t=$1; shift
  for v in 1 0; do
    echo -n "$t FCE_NO_DRING=$v "
    FCE_NO_DRING=$v timeout -k 10 300 python bench.py --warmup 10 --cpu-seconds 0 --predict-steps 0 --dist-config-steps 0 --profile-passes 2 "$@" > $O/${t}_${v}_$rep.log 2>&1 || exit $?
    grep -o '"value": [0-9.]*\|"forward_ms_per_batch": [0-9.]*' $O/${t}_${v}_$rep.log | tr '\n' ' '; echo
  done
done
done
timeout -k 10 400 python -u scripts/tune_report.py > $O/tune_n32.txt 2>&1; echo tune rc=$?
