#!/bin/bash
# Round 5: phase 3's last reads of Q, R, M, r, q non-temporal (new) vs the committed scan (old,
# libnoc_hip_old.so): interleaved KKT bench lines, c3 persistent ipm_solve A/B, KKT/IPM GPU tests.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=r5v ROUNDS=2 bash tools/gpu_ab.sh c3 c5 n300 s2048 s1024 s512 || exit $?
O=gpurun_out/r5v
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
for i in 1 2; do
  NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 ipm_old_$i.log python tools/ipm_bench.py cartpole 200 4096 persistent
  run 200 ipm_new_$i.log python tools/ipm_bench.py cartpole 200 4096 persistent
done
