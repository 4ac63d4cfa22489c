set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06y
mkdir -p $O
P="--cin 64 --cout 64 --k 3 --hw 80 --batch 32 --codes 0x640,0xd41 --reps 10"
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS --kernel-trace --output-format csv -d $O/pmc1 -o run -- python3 scripts/conv_probe.py $P > $O/pmc1.log 2>&1; echo pmc1 rc=$?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d $O/pmc2 -o run -- python3 scripts/conv_probe.py $P > $O/pmc2.log 2>&1; echo pmc2 rc=$?
