#!/bin/bash
# Round 6, session q: c3 with the heavy-first split (the costliest trajectories of the probe order
# on their own launch) running those with two speculative candidates each.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r6q; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-250; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 300 pytest_heavy.log python -u -m pytest tests/test_ipm_gpu.py -x -v --timeout 200 --timeout-method thread -k "heavy"
for rep in 1 2; do
  run 120 base_$rep.log python tools/ipm_bench.py cartpole 200 4096 persistent
  for h in 64 128 256 512; do
    run 120 h${h}_spec_$rep.log env NOC_PERSIST_HEAVY=$h NOC_PERSIST_HEAVY_SPEC=2 python tools/ipm_bench.py cartpole 200 4096 persistent
  done
  run 120 h128_one_$rep.log env NOC_PERSIST_HEAVY=128 python tools/ipm_bench.py cartpole 200 4096 persistent
done
