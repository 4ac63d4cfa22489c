set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06ae
mkdir -p $O
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/pmc1 -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --predict-steps 0 --dist-config-steps 0 --profile-passes 1 --no-nms > $O/pmc1.log 2>&1; echo pmc1 rc=$?
python3 scripts/pmc_kernels.py $O/pmc1/run_counter_collection.csv > $O/pmc1_kernels.txt 2>&1
rm -rf $O/pmc1
