#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -3 "gpurun_out/$log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run 600 ipm_tests.log python -m pytest tests/test_ipm_gpu.py -q -x
run 600 ipm_bench_c3.log python tools/ipm_bench.py cartpole 200 4096
run 300 ipm_bench_c2.log python tools/ipm_bench.py pendulum 100 1024
run 600 prof_ipm.log rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof/ipm" -o run -- python "$R/tools/ipm_bench.py" cartpole 200 4096
