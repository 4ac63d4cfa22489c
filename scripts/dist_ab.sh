#!/bin/bash
# Multi-GPU path A/B runs on the one-GPU box (a one-rank RCCL group, FCE_DIST_FORCE=1 under torch.distributed.run).
#   dist_ab.sh poster TAG   resident 4-lane bench and host-image path: the per-batch gather issued by the host-thread
#                           poster (default) / the device-side side-stream wait (FCE_POST_DEVICE_WAIT=1) / host gather
#                           (FCE_HOST_GATHER=1, host path) / no process group; 8 hardware queues in all
#   dist_ab.sh cost TAG     torchrun alone / the group without the per-batch gather (FCE_DIST_NO_GATHER=1) / with it
#   dist_ab.sh queues TAG   the group with the device-side wait by GPU_MAX_HW_QUEUES (8 .. 24)
#   dist_ab.sh host TAG     the host-image path with the poster's per-batch gather against no group, 3 rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
MODE=$1
OUT=gpurun_out/${2:-dist_ab}
mkdir -p "$OUT"
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-8}
A="--steps 100 --warmup 10 --cpu-seconds 0 --predict-steps 0 --dist-config-steps 0 --lanes 4"
H="--source host --steps 60 --warmup 5"
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1"
i=0
run() {  # $1 log name, rest: env assignments then bench args (group runs go through torchrun with FCE_DIST_FORCE=1)
  local name=$1
  shift
  i=$((i + 1))
  timeout -k 10 200 env "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' "$OUT/$name.log")"
  return $rc
}
case "$MODE" in
  poster)
    for rep in 1 2; do
      run res_poster_$rep FCE_DIST_FORCE=1 $R --master-port $((29800 + i)) bench.py $A || exit $?
      run res_devwait_$rep FCE_POST_DEVICE_WAIT=1 FCE_DIST_FORCE=1 $R --master-port $((29800 + i)) bench.py $A || exit $?
      run res_plain_$rep X=0 python bench.py $A || exit $?
      run host_poster_$rep FCE_DIST_FORCE=1 $R --master-port $((29800 + i)) bench.py $H || exit $?
      run host_hostgather_$rep FCE_HOST_GATHER=1 FCE_DIST_FORCE=1 $R --master-port $((29800 + i)) bench.py $H || exit $?
      run host_plain_$rep X=0 python bench.py $H || exit $?
    done
    ;;
  cost)
    for rep in 1 2; do
      run torchrun_only_$rep X=0 $R --master-port $((29800 + i)) bench.py $A || exit $?
      run group_nogather_$rep FCE_DIST_NO_GATHER=1 FCE_DIST_FORCE=1 $R --master-port $((29800 + i)) bench.py $A || exit $?
      run group_gather_$rep FCE_DIST_FORCE=1 $R --master-port $((29800 + i)) bench.py $A || exit $?
      run plain_$rep X=0 python bench.py $A || exit $?
    done
    ;;
  host)  # the host-image path only: the poster's per-batch device gather / no process group, 3 interleaved rounds
    for rep in 1 2 3; do
      run host_poster_$rep FCE_DIST_FORCE=1 $R --master-port $((29800 + i)) bench.py --source host --steps 100 --warmup 10 || exit $?
      run host_plain_$rep X=0 python bench.py --source host --steps 100 --warmup 10 || exit $?
    done
    ;;
  every)  # diagnostics: the poster issuing the gather only every n-th batch (results meaningless)
    for rep in 1 2; do
      for n in 1 2 4 8; do
        run every${n}_$rep FCE_POST_EVERY_DIAG=$n FCE_DIST_FORCE=1 $R --master-port $((29800 + i)) bench.py $A || exit $?
      done
    done
    ;;
  queues)
    for q in 8 10 12 16 24; do
      run q$q GPU_MAX_HW_QUEUES=$q FCE_POST_DEVICE_WAIT=1 FCE_DIST_FORCE=1 $R --master-port $((29800 + i)) bench.py $A || exit $?
    done
    ;;
  *)
    sed -n '2,8p' "$0"
    exit 2
    ;;
esac
