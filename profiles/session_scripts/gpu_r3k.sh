#!/bin/bash
# Round 3, session k: SURVEY §8(f)1 at batch scale -- the persistent one-wave solver with Q, R, M, r
# kept in LDS for the scan (NOC_PERSIST_QLDS=1, one wave per SIMD) against the same instance
# reading them from the workspace and against the default (2 waves per SIMD at c3); results must
# be bit-identical (u_sha1).  Then the loaded per-phase attribution of one c3 solve (profile build)
# and the c3 tail timeline.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3k}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-400; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
for i in 1 2; do
  run 0 200 c3_default_$i.txt python tools/ipm_bench.py cartpole 200 4096 persistent
  run 0 200 c3_w1_$i.txt env NOC_PERSIST_WAVES=1 python tools/ipm_bench.py cartpole 200 4096 persistent
  run 0 200 c3_w1_qlds_$i.txt env NOC_PERSIST_WAVES=1 NOC_PERSIST_QLDS=1 python tools/ipm_bench.py cartpole 200 4096 persistent
  run 0 200 b1024_default_$i.txt python tools/ipm_bench.py cartpole 200 1024 persistent
  run 0 200 b1024_qlds_$i.txt env NOC_PERSIST_QLDS=1 python tools/ipm_bench.py cartpole 200 1024 persistent
  run 0 200 b1_n100_default_$i.txt python tools/ipm_bench.py cartpole 100 1 persistent
  run 0 200 b1_n100_qlds_$i.txt env NOC_PERSIST_QLDS=1 python tools/ipm_bench.py cartpole 100 1 persistent
done
run 0 300 phases.txt env NOC_HIP_LIB=$L/libnoc_hip_prof.so python tools/persist_phases.py
