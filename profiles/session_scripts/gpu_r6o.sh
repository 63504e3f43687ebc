#!/bin/bash
# Round 6, session o: the tail schedule (capped launches, stragglers gathered and resumed with
# speculative candidates).  Parity tests, then cap ladders at 1024 / 2048 / 4096 cart-poles.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r6o; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-250; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 500 pytest_tail.log python -u -m pytest tests/test_ipm_gpu.py -x -v --timeout 200 --timeout-method thread -k "tail_schedule or speculative or structured or capped or retry"
run 600 tail_caps.log python tools/tail_caps.py
