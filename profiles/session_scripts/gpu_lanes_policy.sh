#!/bin/bash
# Lane-count sweep of the KKT scan over horizon and batch (input to the lane policy).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/lanes_policy; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for n in 50 100 150 200 300 400; do
  run 200 cart_n${n}_b4096.log python tools/batch_probe.py --problem cartpole --horizon $n --batch 4096 --splits 1 --lanes 64,32,16,8 --reps 10 --rounds 3
done
for b in 1024 4096 16384; do
  run 200 pend_n100_b${b}.log python tools/batch_probe.py --problem pendulum --horizon 100 --batch $b --splits 1 --lanes 64,32,16,8 --reps 10 --rounds 3
done
run 200 cart_n200_b1024.log python tools/batch_probe.py --problem cartpole --horizon 200 --batch 1024 --splits 1 --lanes 64,32,16,8 --reps 10 --rounds 3
run 200 cart_n200_b16384.log python tools/batch_probe.py --problem cartpole --horizon 200 --batch 16384 --splits 1 --lanes 64,32,16,8 --reps 10 --rounds 3
