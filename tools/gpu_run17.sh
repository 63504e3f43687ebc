#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r17; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -3 "$O/$log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 300 pytest_kkt.log python -u -m pytest tests/test_kkt_gpu.py -x -q --timeout 120 --timeout-method thread
run 300 sweep_c4.log python tools/kkt_sweep.py --configs c4 --lanes 1 --layouts tiled,natural --rounds 3 --reps 3
