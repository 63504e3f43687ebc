#!/bin/bash
# GPU parity incl. the lanes=1 group solve, then c4 sweep (group vs scan) and c3/c2 with lanes=1.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -4 "gpurun_out/$log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 600 r9_pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run 400 r9_sweep_c4.log python tools/kkt_sweep.py --configs c4 --lanes 1,16,8 --layouts natural --rounds 3 --reps 3
run 300 r9_sweep_c3.log python tools/kkt_sweep.py --configs c3,c2 --lanes 1,32 --layouts natural
