#!/bin/bash
# Round 3, session w: the waves-per-workgroup policy of the L <= 64 scan (4 while the batch's waves
# fit one per SIMD, 2 beyond; noc_internal.h kkt_waves_per_block).  Every GPU test, the interleaved
# bench lines against HEAD (libnoc_hip_A.so: one wave per workgroup), then the same-build rocprof
# traces + FETCH / WRITE passes of the scan configurations (the KKT source hash changed).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3w}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
S="--steps 200 --warmup 20 --no-cpu --no-ipm"
for i in 1 2; do
  for cfg in "c2:--problem pendulum --horizon 100 --global-batch 1024" "c3:" "s512:--batch 512" "s1024:--batch 1024" "s2048:--batch 2048"; do
    n=${cfg%%:*}; a=${cfg#*:}
    run 0 200 ${n}_A_$i.txt env NOC_HIP_LIB=$L/libnoc_hip_A.so python bench.py $a $S
    run 0 200 ${n}_B_$i.txt python bench.py $a $S
  done
done
OUT=r3w/final CONFIGS="c3 c2 s2048 s1024 s512" bash tools/gpu_final_r3.sh
