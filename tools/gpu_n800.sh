#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/n800; mkdir -p $O
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 120 w_auto.log python tools/ipm_bench.py cartpole 800 1 persistent
NOC_PERSIST_WAVES=2 run 120 w2.log python tools/ipm_bench.py cartpole 800 1 persistent
NOC_PERSIST_WAVES=1 run 120 w1.log python tools/ipm_bench.py cartpole 1000 1 persistent
NOC_PERSIST_WAVES=2 run 120 w2_1000.log python tools/ipm_bench.py cartpole 1000 1 persistent
run 120 pend100.log python tools/ipm_bench.py pendulum 100 1 persistent
