#!/bin/bash
# Round 3, session p: the standalone scan with EXEC-masked nx = 4 combines at two waves per SIMD
# (libnoc_hip_m4.so: no identity selects, 92 vs 56 B/lane of scratch at c3) against the current
# library, interleaved: c3 and the 2048 / 1024 shards.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3p}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-160; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
S="--steps 50 --warmup 5 --no-cpu --no-ipm"
for i in 1 2 3; do
  run 0 200 c3_base_$i.txt python bench.py $S
  run 0 200 c3_m4_$i.txt env NOC_HIP_LIB=$L/libnoc_hip_m4.so python bench.py $S
done
for i in 1 2; do
  for b in 2048 1024; do
    run 0 200 s${b}_base_$i.txt python bench.py --batch $b $S
    run 0 200 s${b}_m4_$i.txt env NOC_HIP_LIB=$L/libnoc_hip_m4.so python bench.py --batch $b $S
  done
done
