#!/bin/bash
# Round-2 final measurement, part 1: GPU suite, smoke, bench, rocprof trace + stats of the n32 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh && bash scripts/gpu_prof.sh r02f
