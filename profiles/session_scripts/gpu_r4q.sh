#!/bin/bash
# Round 4, session q: c3 at L = 16 (4 trajectories per wave, 1024 waves = one per SIMD) with the
# 512-register instance, against L = 16 without it (NOC_KKT_BIG=0) and the default L = 32;
# interleaved, three rounds; then the KKT tests on this build.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r4q}; mkdir -p $O
export TMPDIR=/tmp
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
B="--steps 50 --warmup 5 --no-cpu --no-ipm"
for i in 1 2 3; do
  run 0 200 l32_c3_$i.txt python bench.py $B
  run 0 200 l16big_c3_$i.txt python bench.py $B --lanes 16
  NOC_KKT_BIG=0 run 0 200 l16_c3_$i.txt python bench.py $B --lanes 16
done
run 1 600 pytest_kkt.txt python -u -m pytest tests/test_kkt_gpu.py -m gpu -q --timeout 300 --timeout-method thread -rf
