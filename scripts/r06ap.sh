set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06ap
mkdir -p $O
export FCE_DRING_TIMING=1
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --hw 80 --batch 32 --codes 0xd41,0xd21 --reps 2 > $O/t_s1_64_80.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --stride 2 --hw 160 --batch 32 --codes 0xd21 --reps 2 > $O/t_s2_64_160.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 32 --cout 32 --k 3 --hw 160 --batch 32 --codes 0xd49,0xd41 --reps 2 > $O/t_s1_32_160.txt 2>&1 || exit $?
