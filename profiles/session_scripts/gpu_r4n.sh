#!/bin/bash
# Round 4, session n: issue priority (s_setprio) for the persistent solver's waves past 256 / 512
# KKT solves -- the few long trajectories that end a c3 launch.  Interleaved A/B against the
# committed build (libnoc_hip_old.so) on whole solves: c3 (cart-pole N=200 B=4096, two waves per
# SIMD), c2 (pendulum N=100 B=1024), cart-pole N=200 B=1024 (one wave per SIMD), with the u hash
# (results must be identical); then the IPM / API / golden tests.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r4n}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
for i in 1 2 3; do
  NOC_HIP_LIB=$L/libnoc_hip_old.so run 0 200 old_c3_$i.txt python tools/ipm_bench.py cartpole 200 4096 persistent
  run 0 200 new_c3_$i.txt python tools/ipm_bench.py cartpole 200 4096 persistent
  NOC_HIP_LIB=$L/libnoc_hip_old.so run 0 200 old_c2_$i.txt python tools/ipm_bench.py pendulum 100 1024 persistent
  run 0 200 new_c2_$i.txt python tools/ipm_bench.py pendulum 100 1024 persistent
  NOC_HIP_LIB=$L/libnoc_hip_old.so run 0 200 old_b1024_$i.txt python tools/ipm_bench.py cartpole 200 1024 persistent
  run 0 200 new_b1024_$i.txt python tools/ipm_bench.py cartpole 200 1024 persistent
done
run 1 900 pytest.txt python -u -m pytest tests/test_ipm_gpu.py tests/test_api_gpu.py tests/test_golden_gpu.py -m gpu -q --timeout 300 --timeout-method thread -rf
