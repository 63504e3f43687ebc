#!/bin/bash
# GPU tests (parity) + KKT lanes sweep + bench line after staging K, d in LDS.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -3 "gpurun_out/$log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 600 r8_pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run 300 r8_sweep.log python tools/kkt_sweep.py --configs c3,c2 --lanes 64,32,16 --layouts tiled
run 300 r8_bench.log python bench.py --steps 50 --warmup 5 --cpu-seconds 5
