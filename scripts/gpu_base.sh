#!/bin/bash
# Baseline pass for a round: parity tests + smoke + bench (gpu_check.sh), then a rocprofv3 kernel
# trace of the bench (gpu_prof.sh).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r02a}
bash scripts/gpu_check.sh && bash scripts/gpu_prof.sh $TAG
