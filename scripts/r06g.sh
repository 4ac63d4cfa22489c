set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06g
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d gpurun_out/r06g/lds -o run -- python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --predict-steps 0 --dist-config-steps 0 --profile-passes 1 --no-nms > gpurun_out/r06g/lds.log 2>&1
echo rc=$?
python scripts/pmc_kernels.py gpurun_out/r06g/lds/run_counter_collection.csv > gpurun_out/r06g/lds_summary.txt
rm -f gpurun_out/r06g/lds/run_counter_collection.csv
