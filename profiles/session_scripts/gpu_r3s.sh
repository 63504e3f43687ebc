#!/bin/bash
# Round 3, session s: the persistent solver reuses the taken trial's stage costs in the next
# linearisation (the trial wrote them to w.lc; bit-identical) -- every GPU test first, then the
# interleaved A/B against HEAD (libnoc_hip_A.so); u_sha1 must agree.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3s}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
for i in 1 2 3; do
  run 0 200 c3_A_$i.txt env NOC_HIP_LIB=$L/libnoc_hip_A.so python tools/ipm_bench.py cartpole 200 4096 persistent
  run 0 200 c3_B_$i.txt python tools/ipm_bench.py cartpole 200 4096 persistent
  run 0 200 c2_A_$i.txt env NOC_HIP_LIB=$L/libnoc_hip_A.so python tools/ipm_bench.py pendulum 100 1024 persistent
  run 0 200 c2_B_$i.txt python tools/ipm_bench.py pendulum 100 1024 persistent
done
run 0 300 phases.txt env NOC_HIP_LIB=$L/libnoc_hip_prof.so python tools/persist_phases.py
