#!/bin/bash
# round-3 checkpoint: full GPU suite + smoke + bench (4 lanes x 8 queues default), then the rocprof trace/stats pass
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh || exit $?
bash scripts/gpu_prof.sh ${1:-r03x}
