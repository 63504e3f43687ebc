#!/bin/bash
# Costate fold inside the linearisation (no separate pass over A, cx): GPU tests of the persistent
# solver against the oracle / the multi-launch driver, then interleaved ipm_solve A/B (old library
# via NOC_HIP_LIB) with the u hash.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5f1}; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
OLD=$R/ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_abold.so
run 600 pytest_ipm.txt python -u -m pytest tests/test_ipm_gpu.py tests/test_api_gpu.py -x -q --timeout 300 --timeout-method thread
for r in ${ROUNDS:-1 2 3}; do
  NOC_HIP_LIB=$OLD run 120 ipm_old_$r.json python tools/ipm_bench.py cartpole 200 4096 persistent
  run 120 ipm_new_$r.json python tools/ipm_bench.py cartpole 200 4096 persistent
done
for r in ${C2ROUNDS:-1 2}; do
  NOC_HIP_LIB=$OLD run 120 c2_old_$r.json python tools/ipm_bench.py pendulum 100 1024 persistent
  run 120 c2_new_$r.json python tools/ipm_bench.py pendulum 100 1024 persistent
done
