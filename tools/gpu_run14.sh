#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r14; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -3 "$O/$log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 300 pytest_mpc.log python -u -m pytest tests/test_kkt_gpu.py -k mpc -x -v --timeout 120 --timeout-method thread
run 300 runtime_pend.log python tools/runtime_sweep.py --problem pendulum --out $O/runtime
run 300 runtime_cart.log python tools/runtime_sweep.py --problem cartpole --out $O/runtime
