set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06al
mkdir -p $O
timeout -k 10 120 python -u scripts/conv_probe.py --cin 128 --cout 128 --k 3 --hw 40 --batch 32 --codes 0x2182,0x2142,0xcd0,0xd21,0xd22,0xd40 > $O/p_s1_128_40.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 128 --cout 128 --k 3 --stride 2 --hw 80 --batch 32 --codes 0xcd0,0x2141,0xd10 > $O/p_s2_128_80.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 128 --cout 128 --k 3 --stride 2 --hw 40 --batch 32 --codes 0x2141,0xcd0,0xd10 > $O/p_s2_128_40.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 128 --cout 256 --k 3 --stride 2 --hw 40 --batch 32 --codes 0xcd0,0x6142,0xd10 > $O/p_s2_128_256_40.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -v -m gpu -k "every_variant or channel_slice_views" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc $(tail -1 $O/pytest.log)
