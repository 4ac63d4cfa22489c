#!/bin/bash
# multi-rank rehearsals of the default bench path (4 lanes x 8 queues): the self-launching `bench.py --gpus 2` over gloo
# with both ranks on the one GPU, and the RCCL path with one rank (FCE_DIST_FORCE=1: process group, weight broadcast,
# per-batch all-gather on the side stream)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03ac; export TMPDIR=/tmp
FCE_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --cpu-seconds 0 \
  --predict-steps 0 --profile-passes 2 > gpurun_out/r03ac/bench_gloo2.log 2>&1
rc=$?; echo "gloo2 rc=$rc"; tail -1 gpurun_out/r03ac/bench_gloo2.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
FCE_DIST_FORCE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --steps 30 --warmup 5 --cpu-seconds 0 --predict-steps 0 --profile-passes 2 > gpurun_out/r03ac/bench_rccl1.log 2>&1
rc=$?; echo "rccl1 rc=$rc"; tail -1 gpurun_out/r03ac/bench_rccl1.log | cut -c1-300; python - <<'PY'
import json
d = json.loads(open('gpurun_out/r03ac/bench_rccl1.log').read().strip().splitlines()[-1])
print(d["n_gpus"], d["value"], d["config"], d["process_group"])
PY
exit $rc
