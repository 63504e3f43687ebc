#!/bin/bash
# c4 forward-sweep prefetch ring: group-solve tests, ablation split, interleaved bench A/B
# against libnoc_hip_old.so.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/c4_fwd; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 600 pytest_kkt.log python -u -m pytest tests/test_kkt_gpu.py tests/test_golden_gpu.py tests/test_ipm_gpu.py tests/test_api_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread
run 300 c4_ablate.log python tools/kkt_ablate.py linear8 512 16384 1
B="--problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 10 --warmup 2 --no-cpu --no-ipm"
for i in 1 2 3; do
  NOC_HIP_LIB=$L/libnoc_hip_old.so run 300 old_c4_$i.log python bench.py $B
  run 300 new_c4_$i.log python bench.py $B
done
