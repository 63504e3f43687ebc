#!/bin/bash
# Round 3, session v: several independent waves per workgroup for the L <= 64 scan (NOC_KKT_WPB =
# 1 | 2 | 4) -- fewer workgroups for the dispatcher to place (c2 stamps: waves start over 1.1 us of
# a 7.2 us span).  The scan tests under WPB = 4 first, then interleaved bench lines against HEAD
# (libnoc_hip_A.so, one wave per workgroup, 64-thread launch bounds).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3v}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 600 pytest_wpb4.txt env NOC_KKT_WPB=4 python -u -m pytest tests/test_kkt_gpu.py tests/test_golden_gpu.py -m gpu -q --timeout 300 --timeout-method thread -rf
S="--steps 200 --warmup 20 --no-cpu --no-ipm"
for i in 1 2; do
  for cfg in "c2:--problem pendulum --horizon 100 --global-batch 1024" "c3:" "s1024:--batch 1024" "s2048:--batch 2048"; do
    n=${cfg%%:*}; a=${cfg#*:}
    run 0 200 ${n}_A_$i.txt env NOC_HIP_LIB=$L/libnoc_hip_A.so python bench.py $a $S
    run 0 200 ${n}_w1_$i.txt env NOC_KKT_WPB=1 python bench.py $a $S
    run 0 200 ${n}_w2_$i.txt env NOC_KKT_WPB=2 python bench.py $a $S
    run 0 200 ${n}_w4_$i.txt env NOC_KKT_WPB=4 python bench.py $a $S
  done
done
