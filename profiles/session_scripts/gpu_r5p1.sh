#!/bin/bash
# Probe-ordered persistent solve: parity tests, interleaved A/B against the initial-cost order
# (c3 and c2 sized batches, two seeds), and the default bench line.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5p1}; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 600 pytest_ipm.txt python -u -m pytest tests/test_ipm_gpu.py -x -q --timeout 300 --timeout-method thread -k "probe or cost_ordered or resume or capped or cap"
for r in 1 2 3; do
  for s in cost probe; do
    NOC_SCHEDULE=$s run 120 ipm_${s}_$r.json python tools/ipm_bench.py cartpole 200 4096 persistent
  done
done
run 300 bench_c3.txt python bench.py
