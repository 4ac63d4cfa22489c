set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06at
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu.py -m gpu -k "every_variant or rings_on_channel_slice" > $O/tests.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --hw 80 --batch 32 --codes 0xd41,0xd41,0x1d41,0xd21,0x1d21,0xd41,0x1d41,0xd21,0x1d21 --reps 5 > $O/s1_64_80.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --hw 40 --batch 32 --codes 0xd41,0xd41,0x1d41,0xd21,0x1d21,0xd41,0x1d41 --reps 5 > $O/s1_64_40.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 32 --cout 32 --k 3 --hw 160 --batch 32 --codes 0xd45,0xd45,0x1d41,0xd41,0x1d21,0xd45,0x1d41,0x1d29,0xd49 --reps 5 > $O/s1_32_160.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --stride 2 --hw 160 --batch 32 --codes 0xd21,0xd21,0x1d21,0xd21,0x1d21 --reps 5 > $O/s2_64_160.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 128 --cout 128 --k 3 --stride 2 --hw 80 --batch 32 --codes 0xd10,0xd10,0x1d10,0xd10,0x1d10 --reps 5 > $O/s2_128_80.txt 2>&1 || exit $?
export FCE_DRING_TIMING=1
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --hw 80 --batch 32 --codes 0xd41,0x1d41 --reps 2 > $O/t_s1_64_80.txt 2>&1 || exit $?
