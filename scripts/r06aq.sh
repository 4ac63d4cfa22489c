set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06aq
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu.py -m gpu -k "every_variant or rings_on_channel_slice" > $O/tests.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --hw 80 --batch 32 --codes 0xd41,0xd45,0xd25,0xd26,0xd21 --reps 5 > $O/s1_64_80.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 32 --cout 32 --k 3 --hw 160 --batch 32 --codes 0xd49,0xd4d,0xd41,0xd45,0xd25,0xd26 --reps 5 > $O/s1_32_160.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 32 --cout 32 --k 3 --stride 2 --hw 160 --batch 32 --codes 0xd21,0xd25,0xd26,0xd41 --reps 5 > $O/s2_32_160.txt 2>&1 || exit $?
export FCE_DRING_TIMING=1
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --hw 80 --batch 32 --codes 0xd41,0xd45 --reps 2 > $O/t_s1_64_80.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 32 --cout 32 --k 3 --hw 160 --batch 32 --codes 0xd49,0xd4d,0xd45 --reps 2 > $O/t_s1_32_160.txt 2>&1 || exit $?
