cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/variant_check.py --batch 32 > gpurun_out/vc32.log 2>&1; echo rc=$?; tail -5 gpurun_out/vc32.log
timeout -k 10 500 python -u scripts/variant_check.py --batch 1 > gpurun_out/vc1.log 2>&1; echo rc=$?; tail -5 gpurun_out/vc1.log
timeout -k 10 500 python -u scripts/variant_check.py --batch 2 --imgsz 320 --model yolo11s-bifpn.yaml > gpurun_out/vcs.log 2>&1; echo rc=$?; tail -5 gpurun_out/vcs.log
