#!/bin/bash
# Round 6, session g: the persistent scan's combines masked (no identity partner, no selects) at
# one wave per SIMD (default build, NOC_PERSIST_MASKED=1) vs never (masked0) vs always (masked2),
# interleaved: c3, the 512-trajectory slice and B = 1 (u sha1 compared across builds).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r6g; mkdir -p $O
export TMPDIR=/tmp
L=$R/ip-parallel-optimal-control_amd/noc/_lib
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-120; if [ $rc -ne 0 ]; then exit $rc; fi; }
V="NOC_ALLOW_STALE_LIB=1"
for rnd in 1 2; do
  env $V NOC_HIP_LIB=$L/libnoc_hip_masked0.so NOC_PERSIST_WIDE=0 timeout -k 10 120 python tools/ipm_bench.py cartpole 200 512 persistent > $O/m0_512_$rnd.log 2>&1 || exit 1
  NOC_PERSIST_WIDE=0 run 120 m1_512_$rnd.log python tools/ipm_bench.py cartpole 200 512 persistent
  env $V NOC_HIP_LIB=$L/libnoc_hip_masked0.so timeout -k 10 120 python tools/ipm_bench.py cartpole 200 4096 persistent > $O/m0_c3_$rnd.log 2>&1 || exit 1
  run 120 m1_c3_$rnd.log python tools/ipm_bench.py cartpole 200 4096 persistent
  env $V NOC_HIP_LIB=$L/libnoc_hip_masked2.so timeout -k 10 120 python tools/ipm_bench.py cartpole 200 4096 persistent > $O/m2_c3_$rnd.log 2>&1 || exit 1
done
env $V NOC_HIP_LIB=$L/libnoc_hip_masked0.so NOC_PERSIST_WIDE=0 timeout -k 10 120 python tools/ipm_bench.py cartpole 200 1 persistent > $O/m0_1.log 2>&1 || exit 1
NOC_PERSIST_WIDE=0 run 120 m1_1.log python tools/ipm_bench.py cartpole 200 1 persistent
run 120 m1_1024.log python tools/ipm_bench.py cartpole 200 1024 persistent
env $V NOC_HIP_LIB=$L/libnoc_hip_masked0.so timeout -k 10 120 python tools/ipm_bench.py cartpole 200 1024 persistent > $O/m0_1024.log 2>&1 || exit 1
echo done
