set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06av
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu.py -m gpu -k "every_variant or rings_on_channel_slice" > $O/tests.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --hw 80 --batch 32 --codes 0xd41,0xd41,0xd29,0xd19,0xd21,0x640,0xd41,0xd29,0xd19 --reps 5 > $O/s1_64_80.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --hw 40 --batch 32 --codes 0xd41,0xd41,0xd29,0xd19,0xd21,0xd41,0xd29,0xd19 --reps 5 > $O/s1_64_40.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 128 --k 3 --hw 80 --batch 32 --codes 0xd41,0xd41,0xd29,0xd19,0xd41,0xd29,0xd19 --reps 5 > $O/s1_64_128_80.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --stride 2 --hw 160 --batch 32 --codes 0xd21,0xd21,0xd19,0xd21,0xd19 --reps 5 > $O/s2_64_160.txt 2>&1 || exit $?
export FCE_DRING_TIMING=1
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --hw 80 --batch 32 --codes 0xd41,0xd29,0xd19 --reps 2 > $O/t_s1_64_80.txt 2>&1 || exit $?
