#!/bin/bash
# Interior-point DDP: GPU parity vs the oracle, ABI tests, and the B=1 runtime sweeps (par/seq/ddp).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/ddp; mkdir -p $O
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -3 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 400 pytest_ddp.log python -u -m pytest tests/test_ddp.py tests/test_abi.py -x -v --timeout 300 --timeout-method thread
run 400 runtime_pend.log python tools/runtime_sweep.py --problem pendulum --out $O/runtime
run 500 runtime_cart.log python tools/runtime_sweep.py --problem cartpole --out $O/runtime
