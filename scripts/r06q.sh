set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
P1="--cin 64 --cout 64 --k 3 --hw 80 --batch 32"
P2="--cin 128 --cout 128 --k 3 --hw 40 --batch 32"
timeout -k 10 120 python -u scripts/conv_probe.py $P1 > $O/probe64.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/conv_probe.py $P2 > $O/probe128.txt 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/pmc1 -o run -- python3 scripts/conv_probe.py $P1 --codes 0x640,0x620,0x2141 > $O/pmc1.log 2>&1; echo pmc1 rc=$?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_LDS SQ_INSTS_VALU --kernel-trace --output-format csv -d $O/pmc2 -o run -- python3 scripts/conv_probe.py $P1 --codes 0x640,0x620,0x2141 > $O/pmc2.log 2>&1; echo pmc2 rc=$?
