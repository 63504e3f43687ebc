#!/bin/bash
# Round 4, session t: the derandomized hypothesis DDP-parity test (random pendulum / cart-pole
# interior-point DDP solves against the oracle).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r4t}; mkdir -p $O
export TMPDIR=/tmp
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 600 pytest_random.txt python -u -m pytest tests/test_ddp.py -m gpu -q -k random_ddp --timeout 500 --timeout-method thread -rf --durations=3
