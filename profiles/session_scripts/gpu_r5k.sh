#!/bin/bash
# Round 5, session k: order control for session j -- the 512 shard (L = 128) and c3 run the same
# kernel code in the old and the new library; alternate which runs first.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5k}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-120; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="--steps 50 --warmup 5 --no-cpu --no-ipm"
declare -A ARGS=([c3]="" [s1024]="--global-batch 1024" [s512]="--global-batch 512")
for i in 1 2 3 4; do
  for c in s512 c3 s1024; do
    if [ $((i % 2)) -eq 1 ]; then
      run 200 new_${c}_$i.log python bench.py $B ${ARGS[$c]}
      NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 old_${c}_$i.log python bench.py $B ${ARGS[$c]}
    else
      NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 old_${c}_$i.log python bench.py $B ${ARGS[$c]}
      run 200 new_${c}_$i.log python bench.py $B ${ARGS[$c]}
    fi
  done
done
