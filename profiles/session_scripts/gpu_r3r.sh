#!/bin/bash
# Round 3, session r: stage pairs (two stages per pass through linearise / costate + blocks /
# trial, their transcendental chains interleaved) also at two waves per SIMD (libnoc_hip_pairs.so)
# against the current library (pairs only at one wave per SIMD), interleaved; u_sha1 must agree.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3r}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-160; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
for i in 1 2; do
  run 0 200 c3_base_$i.txt python tools/ipm_bench.py cartpole 200 4096 persistent
  run 0 200 c3_pairs_$i.txt env NOC_HIP_LIB=$L/libnoc_hip_pairs.so python tools/ipm_bench.py cartpole 200 4096 persistent
  run 0 200 c2_base_$i.txt python tools/ipm_bench.py pendulum 100 1024 persistent
  run 0 200 c2_pairs_$i.txt env NOC_HIP_LIB=$L/libnoc_hip_pairs.so python tools/ipm_bench.py pendulum 100 1024 persistent
  run 0 200 p4096_base_$i.txt python tools/ipm_bench.py pendulum 100 4096 persistent
  run 0 200 p4096_pairs_$i.txt env NOC_HIP_LIB=$L/libnoc_hip_pairs.so python tools/ipm_bench.py pendulum 100 4096 persistent
done
