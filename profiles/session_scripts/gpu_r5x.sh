#!/bin/bash
# Round 5: the phase-3 cache policy as committed (kkt_nt3: non-temporal for batches beyond
# 1.5x the memory-side cache and for the SIMD-owning instances) vs the previous scan
# (libnoc_hip_old.so), interleaved bench lines; c3 ipm_solve A/B; KKT / golden / IPM GPU tests.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=r5x ROUNDS=2 bash tools/gpu_ab.sh c3 c5 n300 s2048 s1024 s512 || exit $?
O=gpurun_out/r5x
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for i in 1 2; do
  NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 ipm_old_$i.log python tools/ipm_bench.py cartpole 200 4096 persistent
  run 200 ipm_new_$i.log python tools/ipm_bench.py cartpole 200 4096 persistent
done
