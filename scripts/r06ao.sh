set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu.sh prof r06ao || exit $?
bash scripts/gpu.sh pmc r06ao_n || exit $?
bash scripts/gpu.sh pmc r06ao_l --model yolo11l-fce.yaml || exit $?
bash scripts/gpu.sh pmc r06ao_m --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280 || exit $?
