#!/bin/bash
# Round 4, session i: the L = 32 one-wave-per-SIMD instance (BIG) on the 2048-per-GPU shard,
# interleaved against the committed build without it (libnoc_hip_old.so), plus the same shard at
# L = 64 (2048 waves, two per SIMD) for the lanes policy; then the KKT / golden / IPM tests.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r4i}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
B="--steps 50 --warmup 5 --no-cpu --no-ipm --global-batch 2048"
for i in 1 2 3; do
  NOC_HIP_LIB=$L/libnoc_hip_old.so run 0 200 old_s2048_$i.txt python bench.py $B
  run 0 200 new_s2048_$i.txt python bench.py $B
  run 0 200 l64_s2048_$i.txt python bench.py $B --lanes 64
done
run 1 900 pytest_kkt.txt python -u -m pytest tests/test_kkt_gpu.py tests/test_golden_gpu.py tests/test_ipm_gpu.py -m gpu -q --timeout 300 --timeout-method thread -rf
# phase attribution (timing-only ablations) of c2 and the 1024 shard
run 0 200 ablate_c2.txt python tools/kkt_ablate.py pendulum 100 1024 64
run 0 200 ablate_s1024.txt python tools/kkt_ablate.py cartpole 200 1024 64
