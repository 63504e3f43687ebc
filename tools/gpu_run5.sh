#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -3 "gpurun_out/$log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run 600 kkt_tests.log python -m pytest tests/test_kkt_gpu.py -q -x
run 600 ipm_tests.log python -m pytest tests/test_ipm_gpu.py -q -x
run 400 sweep.log python tools/kkt_sweep.py --configs c3,c2 --lanes 64,32,16 --layouts tiled
run 200 ablate32.log python tools/kkt_ablate.py cartpole 200 4096 32
