#!/bin/bash
# Round 6, session k: the wide kernel's wave count.  B = 1 (the reference's runtime sweep) one-wave
# vs two-wave vs four-wave wide kernel over N, and the c3 8-GPU slices (512 cart-poles each) on
# the one-wave vs the two-wave wide kernel: times, KKT-solve counts, iterations, u_sha1.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r6k; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
for pn in pendulum:100 pendulum:200 pendulum:400 pendulum:800 cartpole:128 cartpole:200 cartpole:300; do
  p=${pn%%:*}; n=${pn##*:}
  NOC_PERSIST_WIDE=0 run 120 b1_${p}_${n}_one.log python tools/ipm_bench.py $p $n 1 persistent
  NOC_PERSIST_WIDE=1 NOC_WIDE_WAVES=2 run 120 b1_${p}_${n}_w2.log python tools/ipm_bench.py $p $n 1 persistent
  NOC_PERSIST_WIDE=1 NOC_WIDE_WAVES=4 run 120 b1_${p}_${n}_w4.log python tools/ipm_bench.py $p $n 1 persistent
done
for rep in 1 2; do
  NOC_PERSIST_WIDE=0 run 300 slices8_one_$rep.log python tools/slice_curve.py --ws 8 --out $O/slices8_one_$rep.json
  NOC_PERSIST_WIDE=1 NOC_WIDE_WAVES=2 run 300 slices8_w2_$rep.log python tools/slice_curve.py --ws 8 --out $O/slices8_w2_$rep.json
done
