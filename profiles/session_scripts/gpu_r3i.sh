#!/bin/bash
# Round 3, session i: two-wave segments (L = 128) with one wave per SIMD (the whole register file
# claimed, so the two waves of a block sit on two SIMDs) for the 8-GPU shard (512 cart-poles per
# GPU): every GPU test, shard A/B (policy = 128 vs forced 64, interleaved), stamps, c3 line.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3i}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -2 "$O/$log" | cut -c1-400; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
S="--steps 50 --warmup 5 --no-cpu --no-ipm"
for i in 1 2; do
  run 0 200 shard_512_L128_$i.txt python bench.py --batch 512 $S
  run 0 200 shard_512_L64_$i.txt python bench.py --batch 512 --lanes 64 $S
done
run 0 120 stamps_s512_L128.txt env NOC_HIP_LIB=$L/libnoc_hip_stamps.so python tools/scan_stamps.py cartpole 200 512
run 0 200 shard_1024.txt python bench.py --batch 1024 $S
run 0 200 bench_c3.txt python bench.py --steps 20 --warmup 2 --no-cpu
