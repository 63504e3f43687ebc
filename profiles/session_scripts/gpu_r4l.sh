#!/bin/bash
# Round 4, session l: noc_total_cost (ABI 5), the nx = 8 interior-point DDP over the device
# building blocks, ddp() below the schedule floor; DDP / ABI / family / API GPU tests.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r4l}; mkdir -p $O
export TMPDIR=/tmp
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 900 pytest_ddp.txt python -u -m pytest tests/test_ddp.py -m gpu -q --timeout 300 --timeout-method thread -rf
