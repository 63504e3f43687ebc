#!/bin/bash
# Round 5, session r: c3 ipm_solve with the one-wave (512-register) persistent instance forced
# (NOC_PERSIST_WAVES=1) against the default two-wave instance, interleaved.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5r}; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-250; if [ $rc -ne 0 ]; then exit $rc; fi; }
for i in 1 2; do
  run 200 w2_$i.log python tools/ipm_bench.py cartpole 200 4096 persistent
  NOC_PERSIST_WAVES=1 run 200 w1_$i.log python tools/ipm_bench.py cartpole 200 4096 persistent
done
