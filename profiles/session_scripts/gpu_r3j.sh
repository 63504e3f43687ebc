#!/bin/bash
# Round 3, session j: interleaved A/B of HEAD's library (A: libnoc_hip_A.so) against the working
# tree's (B): masked nx = 4 combines in the one-wave-per-SIMD instances, two-wave segments for the
# 512-per-GPU shard, the wide persistent solver at one wave per SIMD.  Then every GPU test on B.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3j}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
S="--steps 50 --warmup 5 --no-cpu --no-ipm"
for i in 1 2; do
  run 0 200 shard512_A_$i.txt env NOC_HIP_LIB=$L/libnoc_hip_A.so python bench.py --batch 512 $S
  run 0 200 shard512_B_$i.txt python bench.py --batch 512 $S
  run 0 300 wide_A_$i.txt env NOC_HIP_LIB=$L/libnoc_hip_A.so python tools/wide_probe.py pendulum:200 pendulum:800 cartpole:200 cartpole:300
  run 0 300 wide_B_$i.txt python tools/wide_probe.py pendulum:200 pendulum:800 cartpole:200 cartpole:300
done
run 0 120 stamps_s512_B.txt env NOC_HIP_LIB=$L/libnoc_hip_stamps.so python tools/scan_stamps.py cartpole 200 512
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
