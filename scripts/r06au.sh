set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu.sh check r06au || exit $?
bash scripts/gpu.sh prof r06au || exit $?
bash scripts/gpu.sh pmc r06au_n || exit $?
bash scripts/gpu.sh pmc r06au_l --model yolo11l-fce.yaml || exit $?
bash scripts/gpu.sh pmc r06au_m --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280 || exit $?
bash scripts/gpu.sh configs r06au || exit $?
