set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu.sh check r06an || exit $?
bash scripts/gpu.sh configs r06an || exit $?
