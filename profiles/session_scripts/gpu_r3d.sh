#!/bin/bash
# Round 3, session d: two-wave segments (lanes 128) for small batches -- every GPU test, the
# cart-pole shards at 128 vs 64 lanes, c2 / c3 bench lines.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3d}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -2 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
B="--steps 50 --warmup 5 --no-cpu --no-ipm"
for rep in 1 2; do
for b in 256 512 1024; do
  run 0 200 shard_${b}_L128_$rep.txt python bench.py --batch $b --lanes 128 $B
  run 0 200 shard_${b}_L64_$rep.txt python bench.py --batch $b --lanes 64 $B
done
done
run 0 200 bench_c2.txt python bench.py --problem pendulum --horizon 100 --batch 1024 --steps 100 --warmup 10 --no-cpu --no-ipm
run 0 200 bench_c3.txt python bench.py --steps 20 --warmup 2 --no-cpu --no-ipm
run 0 120 stamps_s512_L128.txt env NOC_HIP_LIB=$L/libnoc_hip_stamps.so python tools/scan_stamps.py cartpole 200 512 128
