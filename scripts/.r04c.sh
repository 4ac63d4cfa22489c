bash scripts/gpu.sh quick r04c "fused_c3k2"; rc=$?; [ $rc -le 1 ] || exit $rc
FCE_C3K2_DIAG=1 timeout -k 10 400 python scripts/fused_probe.py > gpurun_out/r04c/probe.txt 2>&1; rc=$?; grep -v "^c3k2 fused diag" gpurun_out/r04c/probe.txt; grep "^c3k2 fused diag" gpurun_out/r04c/probe.txt | sort | uniq -c | sort -rn | head -12; exit $rc
