#!/bin/bash
# A/B of two builds of libnoc_hip.so: ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_old.so
# (old) vs the default library (new), interleaved bench lines per config (ROUNDS rounds, default 2);
# then the KKT / golden / IPM GPU tests on the new build.  Usage: OUT=dir tools/gpu_ab.sh [configs...]
# (c2 c3 c4 c5 n300 s2048 s1024 s512)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-ab}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="--steps 50 --warmup 5 --no-cpu --no-ipm"
declare -A ARGS=([c2]="--problem pendulum --horizon 100 --batch 1024" [c3]="" [c5]="--batch 8192" [n300]="--horizon 300" [c4]="--problem linear8 --horizon 512 --batch 16384" [s2048]="--global-batch 2048" [s1024]="--global-batch 1024" [s512]="--global-batch 512")
CFGS="${@:-c3 c2}"
for i in $(seq 1 ${ROUNDS:-2}); do
  for c in $CFGS; do
    NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 old_${c}_$i.log python bench.py $B ${ARGS[$c]}
    run 200 new_${c}_$i.log python bench.py $B ${ARGS[$c]}
  done
done
run 900 pytest_kkt.log python -u -m pytest tests/test_kkt_gpu.py tests/test_golden_gpu.py tests/test_ipm_gpu.py -m gpu -q --timeout 300 --timeout-method thread -rf
