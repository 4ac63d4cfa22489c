#!/bin/bash
# round-3 checkpoint: full GPU suite + smoke + bench, then the rocprof trace/stats pass of the bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh || exit $?
bash scripts/gpu_prof.sh r03k
