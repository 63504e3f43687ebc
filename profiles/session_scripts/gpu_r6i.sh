#!/bin/bash
# Round 6, session i: the one-wave-per-SIMD instance's per-stage loops (linearise, costates +
# blocks, trial) in groups of 4 stages (libnoc_hip_g4.so, -DNOC_PERSIST_GROUP=4) against the pairs
# of the default build, interleaved: 512 / 1024 / 1 cart-poles N = 200, 1024 pendulums N = 100.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r6i; mkdir -p $O
export TMPDIR=/tmp
L=$R/ip-parallel-optimal-control_amd/noc/_lib
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-120; if [ $rc -ne 0 ]; then exit $rc; fi; }
export NOC_PERSIST_WIDE=0
for rnd in 1 2 3; do
  for B in 512 1024; do
    env NOC_ALLOW_STALE_LIB=1 NOC_HIP_LIB=$L/libnoc_hip_g4.so timeout -k 10 120 python tools/ipm_bench.py cartpole 200 $B persistent > $O/g4_$B_$rnd.log 2>&1 || exit 1
    mv $O/g4_$B_$rnd.log $O/g4_${B}_$rnd.log
    run 120 g2_${B}_$rnd.log python tools/ipm_bench.py cartpole 200 $B persistent
  done
done
env NOC_ALLOW_STALE_LIB=1 NOC_HIP_LIB=$L/libnoc_hip_g4.so timeout -k 10 120 python tools/ipm_bench.py cartpole 200 1 persistent > $O/g4_1.log 2>&1 || exit 1
run 120 g2_1.log python tools/ipm_bench.py cartpole 200 1 persistent
env NOC_ALLOW_STALE_LIB=1 NOC_HIP_LIB=$L/libnoc_hip_g4.so timeout -k 10 120 python tools/ipm_bench.py pendulum 100 1024 persistent > $O/g4_pend.log 2>&1 || exit 1
run 120 g2_pend.log python tools/ipm_bench.py pendulum 100 1024 persistent
echo done
