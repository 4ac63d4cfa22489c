set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06h
for th in std alt std alt; do FCE_BNECK_TH=$th timeout -k 10 120 python -u scripts/bneck_probe.py >> gpurun_out/r06h/probe.txt 2>&1 || exit $?; done
for rep in 1 2; do for l in 3 4 5; do echo -n "lanes $l: "; timeout -k 10 300 python bench.py --lanes $l --steps 100 --warmup 10 --cpu-seconds 0 --predict-steps 0 --dist-config-steps 0 --profile-passes 1 > gpurun_out/r06h/lanes_${l}_$rep.log 2>&1 || exit $?; grep -o '"value": [0-9.]*' gpurun_out/r06h/lanes_${l}_$rep.log; done; done
