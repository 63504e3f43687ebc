#!/bin/bash
# Retry fixed point (par_retry_repeats): IPM GPU tests, the c3 persistent solve with / without
# the shortcut, and the default bench line (its ipm_solve part times both).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/repeats; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 600 pytest_ipm.log python -u -m pytest tests/test_ipm_gpu.py tests/test_api_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
NOC_NO_REPEAT_SKIP=1 run 300 c3_ipm_all.log python tools/ipm_bench.py cartpole 200 4096 persistent
run 300 c3_ipm_skip.log python tools/ipm_bench.py cartpole 200 4096 persistent
NOC_NO_REPEAT_SKIP=1 run 300 c2_ipm_all.log python tools/ipm_bench.py pendulum 100 1024 persistent
run 300 c2_ipm_skip.log python tools/ipm_bench.py pendulum 100 1024 persistent
run 300 bench_c3.log python bench.py
