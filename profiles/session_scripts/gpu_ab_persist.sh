#!/bin/bash
# A/B of the persistent solver (default lib vs libnoc_hip_old.so) on the B=1 runtime sweeps, interleaved.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/ab_persist; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for i in 1 2; do
  NOC_HIP_LIB=$L/libnoc_hip_old.so run 300 old_cart_$i.log python tools/runtime_sweep.py --problem cartpole --out $O/old$i --max-n 400
  run 300 new_cart_$i.log python tools/runtime_sweep.py --problem cartpole --out $O/new$i --max-n 400
done
run 300 new_pend.log python tools/runtime_sweep.py --problem pendulum --out $O/newp
run 300 new_cart_full.log python tools/runtime_sweep.py --problem cartpole --out $O/newc
run 300 c3_ipm.log python tools/ipm_bench.py cartpole 200 4096 persistent
