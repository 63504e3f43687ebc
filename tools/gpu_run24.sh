#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r24; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -2 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 600 pytest_all.log python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
run 200 sweep.log python tools/kkt_sweep.py --configs c3 --lanes 32 --layouts tiled --rounds 7
