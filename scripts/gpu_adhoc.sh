cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pk3; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY --kernel-trace --output-format csv -d gpurun_out/pk3/a -o run -- python scripts/pmc_kernel.py > gpurun_out/pk3/a.log 2>&1; echo rc=$?; tail -3 gpurun_out/pk3/a.log
