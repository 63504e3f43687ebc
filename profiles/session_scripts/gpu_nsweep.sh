#!/bin/bash
# c3 horizon sweep at B=4096 (does the per-stage cost change as the block set crosses the
# 256 MB memory-side cache?) and the c5 per-GPU shard (B=8192) bench line.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/nsweep; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
for n in 50 100 150 200 250 300 400; do
  run 200 n$n.log python bench.py --horizon $n --steps 30 --warmup 3 --no-cpu --no-ipm
done
run 300 c5_shard.log python bench.py --batch 8192 --steps 30 --warmup 3 --cpu-seconds 5
