#!/bin/bash
# Round 6, session m: speculative retries (NOC_PERSIST_SPEC=2|4: SPEC waves per trajectory, one
# regularisation candidate each).  Parity tests first; then B = 1 and 512-cart-pole timings, the
# c3 8- and 4-GPU slices with two candidates, and c3 / c4 bench lines of this build against the
# previous one (libnoc_hip_old.so: the round-6 final build's kernels) for the SPEC = 1 path.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r6m; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-250; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 400 pytest_spec.log python -u -m pytest tests/test_ipm_gpu.py -x -v --timeout 200 --timeout-method thread -k speculative
for rep in 1 2; do
  for sp in 1 2 4; do NOC_PERSIST_WIDE=0 NOC_PERSIST_SPEC=$sp run 120 b1_spec${sp}_$rep.log python tools/ipm_bench.py cartpole 200 1 persistent; done
  run 120 b1_wide_$rep.log python tools/ipm_bench.py cartpole 200 1 persistent
  for sp in 1 2; do NOC_PERSIST_WIDE=0 NOC_PERSIST_SPEC=$sp run 120 b512_spec${sp}_$rep.log python tools/ipm_bench.py cartpole 200 512 persistent; done
done
NOC_PERSIST_SPEC=2 run 300 slices8_spec2.log python tools/slice_curve.py --ws 8 --out $O/slices8_spec2.json
NOC_PERSIST_SPEC=2 run 300 slices4_spec2.log python tools/slice_curve.py --ws 4 --out $O/slices4_spec2.json
run 300 bench_c3_new.log python bench.py --no-cpu
NOC_ALLOW_STALE_LIB=1 NOC_HIP_LIB=$R/ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_old.so run 300 bench_c3_old.log python bench.py --no-cpu
run 300 bench_c4_new.log python bench.py --problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 10 --warmup 2 --no-cpu
NOC_ALLOW_STALE_LIB=1 NOC_HIP_LIB=$R/ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_old.so run 300 bench_c4_old.log python bench.py --problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 10 --warmup 2 --no-cpu
