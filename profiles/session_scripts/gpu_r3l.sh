#!/bin/bash
# Round 3, session l: states / controls in LDS for the whole persistent solve (XLDS, the default
# where the residency allows) against the workspace copies (NOC_PERSIST_XLDS=0), interleaved;
# results must be bit-identical (u_sha1).  Then every GPU test and the phase attribution.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3l}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-330; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
for i in 1 2; do
  run 0 200 c3_xlds_$i.txt python tools/ipm_bench.py cartpole 200 4096 persistent
  run 0 200 c3_ws_$i.txt env NOC_PERSIST_XLDS=0 python tools/ipm_bench.py cartpole 200 4096 persistent
  run 0 200 b1024_xlds_$i.txt python tools/ipm_bench.py cartpole 200 1024 persistent
  run 0 200 b1024_ws_$i.txt env NOC_PERSIST_XLDS=0 python tools/ipm_bench.py cartpole 200 1024 persistent
  run 0 200 c2_xlds_$i.txt python tools/ipm_bench.py pendulum 100 1024 persistent
  run 0 200 c2_ws_$i.txt env NOC_PERSIST_XLDS=0 python tools/ipm_bench.py pendulum 100 1024 persistent
  run 0 200 b1_n100_xlds_$i.txt python tools/ipm_bench.py cartpole 100 1 persistent
  run 0 200 b1_n100_ws_$i.txt env NOC_PERSIST_XLDS=0 python tools/ipm_bench.py cartpole 100 1 persistent
done
run 0 300 phases.txt env NOC_HIP_LIB=$L/libnoc_hip_prof.so python tools/persist_phases.py
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
