#!/bin/bash
# GPU session: stop at the first fault/abort/timeout (exit codes other than 0/1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -3 "gpurun_out/$log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
rocminfo 2>/dev/null | grep -m2 -E "gfx950|Marketing" > gpurun_out/gpuinfo.txt
run 400 kkt_tests.log python -m pytest tests/test_kkt_gpu.py -x -q
run 400 ipm_tests.log python -m pytest tests/test_ipm_gpu.py -x -q
run 300 bench.log python bench.py --steps 20 --warmup 3 --cpu-seconds 5
