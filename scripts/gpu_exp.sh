cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/exp; export TMPDIR=/tmp
run() { tag=$1; shift; env "$@" timeout -k 10 200 python bench.py --steps 30 --warmup 5 --cpu-seconds 0 --predict-steps 0 ${BARGS} > gpurun_out/exp/$tag.log 2>&1; rc=$?; echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"forward_ms_per_batch": [0-9.]*' gpurun_out/exp/$tag.log | tr '\n' ' ')"; return $rc; }
run base FCE_X=0 && run noring FCE_NO_RING=1 && BARGS=--no-nms run nonms FCE_X=0 && BARGS=--no-nms run nonms_noring FCE_NO_RING=1 && BARGS=--sequential run seq FCE_X=0
