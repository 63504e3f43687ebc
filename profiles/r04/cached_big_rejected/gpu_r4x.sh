#!/bin/bash
# Round 4, session x: the 512-register scan instances with the chunk cached in registers (L = 64
# one wave per SIMD: chunks <= 4 stages; L = 128 two-wave segments: <= 2), interleaved against the
# committed build (libnoc_hip_old.so) on the 1024 and 512 shards and c3 (unaffected); then the
# KKT / golden tests.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r4x}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-120; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
B="--steps 50 --warmup 5 --no-cpu --no-ipm"
run 1 600 pytest_kkt.txt python -u -m pytest tests/test_kkt_gpu.py tests/test_golden_gpu.py -m gpu -q --timeout 300 --timeout-method thread -rf
for i in 1 2 3; do
  for g in 1024 512; do
    NOC_HIP_LIB=$L/libnoc_hip_old.so run 0 200 old_s${g}_$i.txt python bench.py $B --global-batch $g
    run 0 200 new_s${g}_$i.txt python bench.py $B --global-batch $g
  done
done
