#!/bin/bash
# The probe-ordered launch (schedule auto) against the initial-cost order on other batches beyond
# the resident waves: pendulum N=100 B=4096, cart-pole N=100 B=4096, cart-pole N=200 B=8192.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5k4}; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
for cfg in "pendulum 100 4096" "cartpole 100 4096" "cartpole 200 8192"; do
  set -- $cfg
  for r in 1 2; do
    for s in cost auto; do
      NOC_SCHEDULE=$s run 150 ${1}_${2}_${3}_${s}_$r.json python tools/ipm_bench.py $1 $2 $3 persistent
    done
  done
done
