#!/bin/bash
# Round 3, session m: wave reductions of the persistent solver (trial cost, stage-cost sum,
# ||cu||, max |Hu|) as VALU butterflies instead of ds_bpermute shuffles (bit-identical): A = HEAD's
# library (libnoc_hip_A.so), B = the working tree; interleaved; u_sha1 must agree.  Then the GPU
# tests that pin persistent == multi-launch and the oracle counts, and the loaded phases.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3m}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
for i in 1 2; do
  run 0 200 c3_A_$i.txt env NOC_HIP_LIB=$L/libnoc_hip_A.so python tools/ipm_bench.py cartpole 200 4096 persistent
  run 0 200 c3_B_$i.txt python tools/ipm_bench.py cartpole 200 4096 persistent
  run 0 200 c2_A_$i.txt env NOC_HIP_LIB=$L/libnoc_hip_A.so python tools/ipm_bench.py pendulum 100 1024 persistent
  run 0 200 c2_B_$i.txt python tools/ipm_bench.py pendulum 100 1024 persistent
done
run 0 300 phases.txt env NOC_HIP_LIB=$L/libnoc_hip_prof.so python tools/persist_phases.py
run 1 600 pytest_ipm.txt python -u -m pytest tests/test_ipm_gpu.py tests/test_ddp.py tests/test_api_gpu.py -m gpu -q --timeout 300 --timeout-method thread -rf
