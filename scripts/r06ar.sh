set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06ar
mkdir -p $O
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --hw 80 --batch 32 --codes 0xd21,0xd41,0xd45,0xd25,0xd26,0xd21,0xd41,0xd45,0xd25 --reps 5 > $O/s1_64_80.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 32 --cout 32 --k 3 --hw 160 --batch 32 --codes 0xd41,0xd49,0xd4d,0xd41,0xd45,0xd25,0xd49,0xd4d,0xd41,0xd45 --reps 5 > $O/s1_32_160.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 32 --cout 32 --k 3 --stride 2 --hw 160 --batch 32 --codes 0xd41,0xd21,0xd25,0xd26,0xd41,0xd21,0xd25,0xd41 --reps 5 > $O/s2_32_160.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --stride 2 --hw 160 --batch 32 --codes 0xd21,0xd21,0xd41,0xd25 --reps 5 > $O/s2_64_160.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 32 --cout 32 --k 3 --hw 80 --batch 32 --codes 0xd41,0xd49,0xd4d,0xd41,0xd45,0xd25,0xd21 --reps 5 > $O/s1_32_80.txt 2>&1 || exit $?
