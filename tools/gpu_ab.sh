#!/bin/bash
# A/B of two library builds on one box: B=1 pendulum and cart-pole runtime sweeps.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/ab; mkdir -p $O
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
NOC_HIP_LIB=$L/libnoc_hip_old.so run 300 old_pend.log python tools/runtime_sweep.py --problem pendulum --out $O/old
run 300 new_pend.log python tools/runtime_sweep.py --problem pendulum --out $O/new
NOC_HIP_LIB=$L/libnoc_hip_old.so run 300 old_pend2.log python tools/runtime_sweep.py --problem pendulum --out $O/old2
run 300 new_pend2.log python tools/runtime_sweep.py --problem pendulum --out $O/new2
NOC_HIP_LIB=$L/libnoc_hip_old.so run 300 old_cart.log python tools/runtime_sweep.py --problem cartpole --out $O/old --max-n 400
run 300 new_cart.log python tools/runtime_sweep.py --problem cartpole --out $O/new --max-n 400
