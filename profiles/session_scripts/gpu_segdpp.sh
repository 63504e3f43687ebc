#!/bin/bash
# VALU butterfly for the scan's pred / feasibility reductions: all GPU tests (results must be
# bit-identical, incl. persistent == multi-launch), interleaved c2 / c3 A/B against
# libnoc_hip_old.so.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/segdpp; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="--steps 100 --warmup 10 --no-cpu --no-ipm"
run 700 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for i in 1 2 3; do
  NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 old_c2_$i.log python bench.py $B --problem pendulum --horizon 100 --batch 1024
  run 200 new_c2_$i.log python bench.py $B --problem pendulum --horizon 100 --batch 1024
done
NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 old_c3.log python bench.py $B
run 200 new_c3.log python bench.py $B
