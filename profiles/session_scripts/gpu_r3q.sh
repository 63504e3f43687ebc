#!/bin/bash
# Round 3, session q: the persistent solver without the Q/R/M/r-in-LDS measurement instance, the
# XLDS switch read per launch, and the new XLDS == workspace test: every GPU test, then the c3
# ipm_solve line (must match the final run's 37.9 ms within noise).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3q}; mkdir -p $O
export TMPDIR=/tmp
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-250; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
run 0 200 c3_ipm_1.txt python tools/ipm_bench.py cartpole 200 4096 persistent
run 0 200 c3_ipm_2.txt python tools/ipm_bench.py cartpole 200 4096 persistent
