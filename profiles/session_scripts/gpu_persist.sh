#!/bin/bash
# Persistent-solver ILP iteration: IPM parity tests, phase cycles (instrumented library), B=1
# runtime sweeps and the c2/c3 batch solves.  Usage: gpurun --timeout 900 -- bash tools/gpu_persist.sh
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/persist; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 400 pytest_ipm.log python -u -m pytest tests/test_ipm_gpu.py -x -q --timeout 120 --timeout-method thread
NOC_HIP_LIB="$R/ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_prof.so" run 300 phases.log python tools/persist_phases.py
run 300 runtime_pend.log python tools/runtime_sweep.py --problem pendulum --out $O/runtime
run 300 runtime_cart.log python tools/runtime_sweep.py --problem cartpole --out $O/runtime
run 200 ipm_c3.log python tools/ipm_bench.py cartpole 200 4096 persistent
run 200 ipm_c2.log python tools/ipm_bench.py pendulum 100 1024 persistent
