#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r19; mkdir -p $O
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -6 "$O/$log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 200 dbg_stage0.log python tools/debug_persist.py 1
run 200 dbg_final.log python tools/debug_persist.py 0
