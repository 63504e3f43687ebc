#!/bin/bash
# Round 3, session n: lanes for the 2-GPU shard (2048 cart-poles per GPU: the policy's 32 lanes,
# one wave per SIMD, vs 64 lanes, two waves per SIMD -- the round-1 policy sweep had no 2048
# point), interleaved; the wide / one-wave cut-over at cart-pole N = 400 (advisor's question).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3n}; mkdir -p $O
export TMPDIR=/tmp
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
S="--steps 50 --warmup 5 --no-cpu --no-ipm"
for i in 1 2; do
  run 0 200 s2048_L32_$i.txt python bench.py --batch 2048 --lanes 32 $S
  run 0 200 s2048_L64_$i.txt python bench.py --batch 2048 --lanes 64 $S
  run 0 200 s1024_L64_$i.txt python bench.py --batch 1024 --lanes 64 $S
  run 0 200 s1024_L32_$i.txt python bench.py --batch 1024 --lanes 32 $S
done
run 0 300 wide_n400.txt python tools/wide_probe.py cartpole:400 pendulum:400
