#!/bin/bash
# Persistent-solver iteration: IPM parity tests, B=1 runtime sweeps, c3-batch solve at 1 and 2
# waves per SIMD.  Usage (repo root, via gpurun): gpurun --timeout 900 -- bash tools/gpu_persist.sh
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/persist; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-500; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 400 pytest_ipm.log python -u -m pytest tests/test_ipm_gpu.py -x -q --timeout 120 --timeout-method thread
run 300 runtime_pend.log python tools/runtime_sweep.py --problem pendulum --out $O/runtime
run 300 runtime_cart.log python tools/runtime_sweep.py --problem cartpole --out $O/runtime
run 200 ipm_c3_w2.log python tools/ipm_bench.py cartpole 200 4096 persistent
NOC_PERSIST_WAVES=1 run 200 ipm_c3_w1.log python tools/ipm_bench.py cartpole 200 4096 persistent
run 200 ipm_c2.log python tools/ipm_bench.py pendulum 100 1024 persistent
