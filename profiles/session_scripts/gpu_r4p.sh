#!/bin/bash
# Round 4, session p: every GPU test (incl. the 100-case derandomized KKT property test and the
# nx = 8 DDP loop), smoke and the default bench line on the round's final tree.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r4p}; mkdir -p $O
export TMPDIR=/tmp
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf --durations=10
run 0 200 smoke.txt python -c "import __graft_entry__ as g; g.smoke()"
run 0 300 bench_c3.txt python bench.py
