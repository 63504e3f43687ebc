#!/bin/bash
# Round 3, session c: per-phase stamps of the current scan (c2, the cart-pole shards 512 / 1024 and
# c3) and the wide-vs-one-wave test with its decision-trace proof.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3c}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -3 "$O/$log" | cut -c1-400; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 400 pytest_wide.txt python -u -m pytest tests/test_ipm_gpu.py -m gpu -q --timeout 300 --timeout-method thread -k wide_solve_matches
run 0 120 stamps_c2.txt env NOC_HIP_LIB=$L/libnoc_hip_stamps2.so python tools/scan_stamps.py pendulum 100 1024
run 0 120 stamps_s512.txt env NOC_HIP_LIB=$L/libnoc_hip_stamps.so python tools/scan_stamps.py cartpole 200 512
run 0 120 stamps_s1024.txt env NOC_HIP_LIB=$L/libnoc_hip_stamps.so python tools/scan_stamps.py cartpole 200 1024
run 0 120 stamps_c3.txt env NOC_HIP_LIB=$L/libnoc_hip_stamps.so python tools/scan_stamps.py cartpole 200 4096
