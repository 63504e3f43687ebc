#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r20; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -4 "$O/$log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 200 dbg_stage0.log python tools/debug_persist.py 1
run 600 pytest_all.log python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
run 300 sweep.log python tools/kkt_sweep.py --configs c3,c2 --lanes 64,32 --layouts tiled
run 200 ipm_c3.log python tools/ipm_bench.py cartpole 200 4096 persistent
