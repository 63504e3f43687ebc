#!/bin/bash
# Pendulum persistent-solver timing: parity tests, phase cycles, B=1 sweep, c2 batch.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/pend; mkdir -p $O
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; grep '^{' "$O/$log" | cut -c1-330 | tail -3; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 400 pytest_ipm.log python -u -m pytest tests/test_ipm_gpu.py -x -q --timeout 120 --timeout-method thread
NOC_HIP_LIB="$R/ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_prof.so" run 300 phases.log python tools/persist_phases.py
run 300 runtime_pend.log python tools/runtime_sweep.py --problem pendulum --out $O/runtime
run 200 ipm_c2.log python tools/ipm_bench.py pendulum 100 1024 persistent
