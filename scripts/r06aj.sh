set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06aj
mkdir -p $O
C=0x640,0xd21,0xd22,0xd41,0xd42,0xd29,0xd49,0xd81
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --hw 80 --batch 32 --codes $C > $O/p_s1_64_80.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 32 --cout 32 --k 3 --hw 160 --batch 32 --codes $C > $O/p_s1_32_160.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --stride 2 --hw 160 --batch 32 --codes 0x620,0xd21 > $O/p_s2_64_160.txt 2>&1 || exit $?
