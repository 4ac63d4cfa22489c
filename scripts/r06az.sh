set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu.sh prof r06az || exit $?
bash scripts/gpu.sh pmc r06az_n || exit $?
bash scripts/gpu.sh pmc r06az_l --model yolo11l-fce.yaml || exit $?
bash scripts/gpu.sh pmc r06az_m --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280 || exit $?
