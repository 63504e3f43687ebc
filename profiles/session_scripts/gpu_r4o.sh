#!/bin/bash
# Round 4, session o: the derandomized hypothesis KKT parity test (random shapes / horizons /
# batches / lanes against the oracle) with the rest of the KKT GPU tests.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r4o}; mkdir -p $O
export TMPDIR=/tmp
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 600 pytest_kkt.txt python -u -m pytest tests/test_kkt_gpu.py -m gpu -q --timeout 300 --timeout-method thread -rf --durations=5
