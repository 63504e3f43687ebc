#!/bin/bash
# Round 6, session n: speculative candidates against the wide kernel where both apply (B <= CUs):
# cart-pole over N at B = 1 and over B at N = 200; c4 with the group solves' P load no longer
# opaque (against the round-6 final build's library).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r6n; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
for nb in 128:1 200:1 300:1 400:1 200:16 200:64 200:128 200:256; do
  n=${nb%%:*}; b=${nb##*:}
  run 120 one_${n}_${b}.log env NOC_PERSIST_WIDE=0 NOC_PERSIST_SPEC=1 python tools/ipm_bench.py cartpole $n $b persistent
  run 120 spec2_${n}_${b}.log env NOC_PERSIST_WIDE=0 NOC_PERSIST_SPEC=2 python tools/ipm_bench.py cartpole $n $b persistent
  run 120 spec4_${n}_${b}.log env NOC_PERSIST_WIDE=0 NOC_PERSIST_SPEC=4 python tools/ipm_bench.py cartpole $n $b persistent
  run 120 wide_${n}_${b}.log env NOC_PERSIST_WIDE=1 python tools/ipm_bench.py cartpole $n $b persistent
done
run 300 bench_c4_new.log python bench.py --problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 10 --warmup 2 --no-cpu
run 300 bench_c4_old.log env NOC_ALLOW_STALE_LIB=1 NOC_HIP_LIB=$R/ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_old.so python bench.py --problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 10 --warmup 2 --no-cpu
run 300 bench_c4_new2.log python bench.py --problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 10 --warmup 2 --no-cpu
