#!/bin/bash
# DDP retry fixed point: DDP GPU tests and the B=1 runtime sweeps with / without the shortcut.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/ddp_repeats; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 600 pytest_ddp.log python -u -m pytest tests/test_ddp.py -m gpu -x -q --timeout 300 --timeout-method thread
NOC_DDP_NO_REPEAT_SKIP=1 run 400 cart_all.log python tools/runtime_sweep.py --problem cartpole --out $O/cart_all --max-n 400
run 400 cart_skip.log python tools/runtime_sweep.py --problem cartpole --out $O/cart_skip
run 400 pend_skip.log python tools/runtime_sweep.py --problem pendulum --out $O/pend_skip
