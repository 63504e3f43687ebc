#!/bin/bash
# GPU tests, then the multi-launch interior-point loop at the old default lanes (64) vs the
# batch-aware policy (cart-pole N=100, B=4096 -> 16), with the persistent solve beside them.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/ipm_lanes; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run 300 multi_l64.log python tools/ipm_bench.py cartpole 100 4096 multi 64
run 300 multi_policy.log python tools/ipm_bench.py cartpole 100 4096 multi 0
run 300 persistent.log python tools/ipm_bench.py cartpole 100 4096 persistent
