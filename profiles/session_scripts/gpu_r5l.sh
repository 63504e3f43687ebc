#!/bin/bash
# Round 5, session l: the 512 shard's +3.5 % in the new library (byte-identical kernel) -- same
# binary under another name (copy), the new host objects with the round-4 (4, 1) scan object
# (hyb), old, new; alternating order.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5l}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-120; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="--steps 50 --warmup 5 --no-cpu --no-ipm --global-batch 512"
for i in 1 2 3; do
  for v in old new copy hyb; do
    case $v in new) lib=libnoc_hip.so ;; *) lib=libnoc_hip_$v.so ;; esac
    NOC_HIP_LIB=$L/$lib run 200 ${v}_s512_$i.log python bench.py $B
  done
done
