#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r15; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -3 "$O/$log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 300 pytest_ipm.log python -u -m pytest tests/test_ipm_gpu.py -x -q --timeout 120 --timeout-method thread
run 200 ipm_c3.log python tools/ipm_bench.py cartpole 200 4096 persistent
run 200 ipm_c2.log python tools/ipm_bench.py pendulum 100 1024 persistent
run 200 ipm_c1.log python tools/ipm_bench.py pendulum 50 1 persistent
run 200 ipm_cart1000.log python tools/ipm_bench.py cartpole 1000 1 persistent
