#!/bin/bash
# A/B of the reverse-Sklansky phase 2 (default lib) against libnoc_hip_old.so (Hillis-Steele
# ds_bpermute phase 2): KKT/IPM GPU tests, interleaved c2 / c3 / N=300 bench lines, the c3
# persistent solve and the B=1 cart-pole runtime sweep.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/ab_revsk; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="--steps 50 --warmup 5 --no-cpu --no-ipm"
for i in 1 2; do
  NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 old_c3_$i.log python bench.py $B
  run 200 new_c3_$i.log python bench.py $B
  NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 old_c2_$i.log python bench.py $B --problem pendulum --horizon 100 --batch 1024
  run 200 new_c2_$i.log python bench.py $B --problem pendulum --horizon 100 --batch 1024
done
NOC_HIP_LIB=$L/libnoc_hip_old.so run 200 old_n300.log python bench.py $B --horizon 300
run 200 new_n300.log python bench.py $B --horizon 300
NOC_HIP_LIB=$L/libnoc_hip_old.so run 300 old_c3_ipm.log python tools/ipm_bench.py cartpole 200 4096 persistent
run 300 new_c3_ipm.log python tools/ipm_bench.py cartpole 200 4096 persistent
NOC_HIP_LIB=$L/libnoc_hip_old.so run 300 old_cart.log python tools/runtime_sweep.py --problem cartpole --out $O/old --max-n 400
run 300 new_cart.log python tools/runtime_sweep.py --problem cartpole --out $O/new --max-n 400
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -3 $O/pytest_gpu.log
