#!/bin/bash
# c3 kernel time under three LLVM scheduling strategies of the scan unit (default lib,
# libnoc_hip_ilp.so = max-ilp, libnoc_hip_mc.so = max-memory-clause), interleaved.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/ab_sched; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="--steps 50 --warmup 5 --no-cpu --no-ipm"
for i in 1 2; do
  run 200 def_$i.log python bench.py $B
  NOC_HIP_LIB=$L/libnoc_hip_ilp.so run 200 ilp_$i.log python bench.py $B
  NOC_HIP_LIB=$L/libnoc_hip_mc.so run 200 mc_$i.log python bench.py $B
done
