#!/bin/bash
# Round 5, session g: the SIMD-owning scan instances with (1) phase 2's partner elements through
# LDS (LDSB) and (2) A, B of the first chunk slots parked in LDS (AB): three-way interleaved bench
# lines -- old (round-4 scan, libnoc_hip_old.so), LDSB only (NOC_KKT_AB=0), LDSB + AB (default) --
# on the strong-scaling shards and c3 (control); then the KKT / golden tests, the DDP probe and
# the DDP tests.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5g}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="--steps 50 --warmup 5 --no-cpu --no-ipm"
declare -A ARGS=([c3]="" [s2048]="--global-batch 2048" [s1024]="--global-batch 1024" [s512]="--global-batch 512")
for i in 1 2 3; do
  for c in s1024 s512 s2048 c3; do
    NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 old_${c}_$i.log python bench.py $B ${ARGS[$c]}
    NOC_KKT_AB=0 run 200 ldsb_${c}_$i.log python bench.py $B ${ARGS[$c]}
    run 200 new_${c}_$i.log python bench.py $B ${ARGS[$c]}
  done
done
run 900 pytest_kkt.log python -u -m pytest tests/test_kkt_gpu.py tests/test_golden_gpu.py -m gpu -q --timeout 300 --timeout-method thread -rf
run 300 ddp_probe.log python tools/ddp_flip_probe.py
run 600 pytest_ddp.log python -u -m pytest tests/test_ddp.py -m gpu -q --timeout 300 --timeout-method thread -rf
