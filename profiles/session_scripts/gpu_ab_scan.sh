#!/bin/bash
# A/B of two builds of the KKT scan (default lib vs libnoc_hip_old.so), interleaved bench lines.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/ab_scan; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="--steps 50 --warmup 5 --no-cpu --no-ipm"
run 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
for i in 1 2; do
  NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 old_c3_$i.log python bench.py $B
  run 200 new_c3_$i.log python bench.py $B
done
NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 old_c5.log python bench.py $B --batch 8192
run 200 new_c5.log python bench.py $B --batch 8192
NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 old_n300.log python bench.py $B --horizon 300
run 200 new_n300.log python bench.py $B --horizon 300
NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 old_c2.log python bench.py $B --problem pendulum --horizon 100 --batch 1024
run 200 new_c2.log python bench.py $B --problem pendulum --horizon 100 --batch 1024
