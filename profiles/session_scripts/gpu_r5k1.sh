#!/bin/bash
# Probe length of the probe-ordered persistent launch: interleaved A/B of PROBE_SOLVES
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5k1}; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
for r in 1 2 3; do
  for k in ${KS:-6 10 16 24}; do
    PROBE_SOLVES=$k run 120 ipm_k${k}_$r.json python tools/ipm_bench.py cartpole 200 4096 persistent
  done
done
