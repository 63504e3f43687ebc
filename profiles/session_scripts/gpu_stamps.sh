#!/bin/bash
# Phase stamps of the c2 (pendulum N=100 B=1024, 2x1 unit) and c3 (cart-pole N=200 B=4096, 4x1 unit)
# scans under full load, plus the wide-vs-one-wave persistent-solver test.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/stamps; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 300 pytest_wide.log python -u -m pytest tests/test_ipm_gpu.py -m gpu -x -q -k wide_solve --timeout 120 --timeout-method thread
NOC_HIP_LIB=$L/libnoc_hip_stamps2.so run 200 stamps_c2.json python tools/scan_stamps.py pendulum 100 1024
NOC_HIP_LIB=$L/libnoc_hip_stamps.so run 200 stamps_c3.json python tools/scan_stamps.py cartpole 200 4096
