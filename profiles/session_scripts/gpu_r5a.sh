#!/bin/bash
# Round 5, session a: baseline bench lines of this round's box (c3, c2 and the strong-scaling
# shards), kernel-only (no CPU leg, no ipm_solve), before any round-5 change.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5a}; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="--steps 50 --warmup 5 --no-cpu --no-ipm"
run 300 c3.log python bench.py $B
run 200 c2.log python bench.py $B --problem pendulum --horizon 100 --batch 1024
run 200 s1024.log python bench.py $B --global-batch 1024
run 200 s512.log python bench.py $B --global-batch 512
