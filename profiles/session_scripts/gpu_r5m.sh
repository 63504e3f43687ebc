#!/bin/bash
# Round 5, session m: the 512 shard after moving the new KKTArgs fields into padding (kernel
# byte-identical incl. the kernarg size): old vs new, alternating, plus the 1024 shard.

R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5m}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-120; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="--steps 50 --warmup 5 --no-cpu --no-ipm --global-batch 512"
for i in 1 2 3; do
  for v in old new; do
    case $v in new) lib=libnoc_hip.so ;; *) lib=libnoc_hip_$v.so ;; esac
    NOC_HIP_LIB=$L/$lib run 200 ${v}_s512_$i.log python bench.py $B
  done
done
for i in 1 2; do
  NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 old_s1024_$i.log python bench.py --steps 50 --warmup 5 --no-cpu --no-ipm --global-batch 1024
  run 200 new_s1024_$i.log python bench.py --steps 50 --warmup 5 --no-cpu --no-ipm --global-batch 1024
done
