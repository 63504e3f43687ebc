#!/bin/bash
# Round 4, session u: staggered start of the c3 scan (experiment): half of the waves sleep for a
# fixed time at the start (NOC_KKT_STAGGER=<mode>:<us>; mode 1 = odd pairs of workgroups, 2 = the
# second wave of each workgroup, 3 = odd workgroups) so that their phase 1 (memory) overlaps the
# other half's phases 2-4 (VALU / re-read latency).  Same build throughout; c3 and the 2048 shard.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r4u}; mkdir -p $O
export TMPDIR=/tmp
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-120; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
B="--steps 50 --warmup 5 --no-cpu --no-ipm"
for i in 1 2; do
  run 0 200 base_c3_$i.txt python bench.py $B
  for m in 1 2 3; do
    for us in 8 16 24; do
      NOC_KKT_STAGGER=$m:$us run 0 200 m${m}_u${us}_c3_$i.txt python bench.py $B
    done
  done
done
