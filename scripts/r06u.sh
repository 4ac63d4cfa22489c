set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
C=0x620,0x640,0x621,0xd21,0xd22,0xd41,0xd42
timeout -k 10 120 python -u scripts/conv_probe.py --cin 64 --cout 64 --k 3 --hw 80 --batch 32 --codes $C > $O/p_s1_64_80.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 32 --cout 32 --k 3 --hw 160 --batch 32 --codes $C > $O/p_s1_32_160.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py --cin 32 --cout 64 --k 3 --stride 2 --hw 320 --batch 32 --codes $C > $O/p_s2_32_320.txt 2>&1 || exit $?
for rep in 1 2; do for v in 1 0; do echo -n "FCE_NO_DRING=$v "; FCE_NO_DRING=$v timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 --predict-steps 0 --dist-config-steps 0 --profile-passes 3 > $O/b_${v}_$rep.log 2>&1 || exit $?; grep -o '"value": [0-9.]*\|"forward_ms_per_batch": [0-9.]*\|"frac": [0-9.]*' $O/b_${v}_$rep.log | tr '\n' ' '; echo; done; done
timeout -k 10 400 python -u scripts/tune_report.py > $O/tune_n32.txt 2>&1; echo tune rc=$?
