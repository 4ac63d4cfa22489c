set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06x
mkdir -p $O
for rep in 1 2; do
for cfg in "l32 --model yolo11l-fce.yaml" "s32 --model yolo11s-bifpn.yaml" "n32"; do
  set -- $cfg; t=$1; shift
  for v in 1 0; do
    echo -n "$t FCE_NO_DRING=$v "
    FCE_NO_DRING=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-seconds 0 --predict-steps 0 --dist-config-steps 0 --profile-passes 2 "$@" > $O/${t}_${v}_$rep.log 2>&1 || exit $?
    grep -o '"value": [0-9.]*\|"forward_ms_per_batch": [0-9.]*' $O/${t}_${v}_$rep.log | tr '\n' ' '; echo
  done
done
done
