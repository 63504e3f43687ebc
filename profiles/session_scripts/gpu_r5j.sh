#!/bin/bash
# Round 5, session j: A, B slots in the 512-register instances only (BIG), split loops: interleaved
# old / this build with NOC_KKT_AB=0 / AB on the shards and c3; then every GPU test and smoke.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5j}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="--steps 50 --warmup 5 --no-cpu --no-ipm"
declare -A ARGS=([c3]="" [s2048]="--global-batch 2048" [s1024]="--global-batch 1024" [s512]="--global-batch 512")
for i in 1 2 3; do
  for c in s1024 s2048 s512 c3; do
    NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 old_${c}_$i.log python bench.py $B ${ARGS[$c]}
    NOC_KKT_AB=0 run 200 noab_${c}_$i.log python bench.py $B ${ARGS[$c]}
    run 200 new_${c}_$i.log python bench.py $B ${ARGS[$c]}
  done
done
run 1100 pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
run 200 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
