#!/bin/bash
# Round-2 final tree: GPU suite + smoke + bench, rocprof trace/stats of the n32 bench, n32 PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh && bash scripts/gpu_prof.sh r02i && bash scripts/gpu_pmc.sh n32
