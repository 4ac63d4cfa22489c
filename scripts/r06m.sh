set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06m
timeout -k 10 300 python -u scripts/pw2_probe.py > gpurun_out/r06m/probe.txt 2>&1; echo probe rc=$?
