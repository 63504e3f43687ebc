#!/bin/bash
# Round 3, session h: validation of HEAD after the container was re-created (traced user costs /
# constraints, round-3 scan): every GPU test, smoke, the default bench line and its kernel trace.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3h}; mkdir -p $O
export TMPDIR=/tmp
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -3 "$O/$log" | cut -c1-400; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
run 0 300 smoke.txt python -c "import __graft_entry__ as g; g.smoke()"
run 0 300 bench_c3.txt python bench.py
run 0 300 trace_c3.txt rocprofv3 --kernel-trace --stats -d $O/trace_c3 -o c3 -- python bench.py --steps 20 --warmup 2 --no-cpu
