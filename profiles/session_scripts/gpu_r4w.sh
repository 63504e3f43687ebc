#!/bin/bash
# Round 4, session w: c4 group solve with non-temporal loads in the forward sweep (the last reader
# of K, d, A, B), interleaved against the committed build (libnoc_hip_old.so); then the KKT tests.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r4w}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-120; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
B="--problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 10 --warmup 2 --no-cpu --no-ipm"
for i in 1 2 3; do
  NOC_HIP_LIB=$L/libnoc_hip_old.so run 0 200 old_c4_$i.txt python bench.py $B
  run 0 200 new_c4_$i.txt python bench.py $B
done
run 1 600 pytest_kkt.txt python -u -m pytest tests/test_kkt_gpu.py -m gpu -q --timeout 300 --timeout-method thread -rf
