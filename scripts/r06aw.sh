set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu.sh bench r06aw || exit $?
bash scripts/gpu.sh configs r06aw || exit $?
