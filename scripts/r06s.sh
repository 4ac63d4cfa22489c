set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06s
mkdir -p $O
for occ in 0 1 2 3 4; do echo "occ $occ"; FCE_PERSIST_OCC=$occ timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --hw 80 --batch 32 --codes 0x640,0x641,0x620,0x621 2>&1 | grep -v amdgpu || exit $?; done > $O/occ.txt
