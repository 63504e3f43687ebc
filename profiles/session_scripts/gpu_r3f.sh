#!/bin/bash
# Round 3, session f: the one-wave-per-SIMD instance with whole-chunk loads (RELOAD) for the
# small cart-pole batches -- every GPU test, the shards 256 / 512 / 1024 (A/B against the plain
# streamed chunks by ablation bit 3), stamps at 512, c3.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3f}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
B="--steps 50 --warmup 5 --no-cpu --no-ipm"
for rep in 1 2; do
for b in 256 512 1024; do
  run 0 200 shard_${b}_$rep.txt python bench.py --batch $b $B
  run 0 200 shard_${b}_ablate_$rep.txt python tools/kkt_ablate.py cartpole 200 $b 64
done
done
run 0 200 bench_c3.txt python bench.py --steps 20 --warmup 2 --no-cpu --no-ipm
run 0 120 stamps_s512.txt env NOC_HIP_LIB=$L/libnoc_hip_stamps.so python tools/scan_stamps.py cartpole 200 512
