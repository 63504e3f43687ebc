#!/bin/bash
# Round 3, session o: costate scan of the interior-point solvers as a reverse Sklansky scan with
# VALU partners (both the persistent and the multi-launch solver; was Hillis-Steele through
# ds_bpermute) and DPP by-one shifts for the scans' boundary hand-offs.  Every GPU test first (the
# oracle iteration counts and persistent == multi-launch pin the new association), then the
# interleaved A/B against HEAD (A = libnoc_hip_A.so), the 2048-shard lanes and the N = 400
# wide / one-wave cut-over.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3o}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
for i in 1 2; do
  run 0 200 c3_A_$i.txt env NOC_HIP_LIB=$L/libnoc_hip_A.so python tools/ipm_bench.py cartpole 200 4096 persistent
  run 0 200 c3_B_$i.txt python tools/ipm_bench.py cartpole 200 4096 persistent
  run 0 200 c2_A_$i.txt env NOC_HIP_LIB=$L/libnoc_hip_A.so python tools/ipm_bench.py pendulum 100 1024 persistent
  run 0 200 c2_B_$i.txt python tools/ipm_bench.py pendulum 100 1024 persistent
done
S="--steps 50 --warmup 5 --no-cpu --no-ipm"
for i in 1 2; do
  run 0 200 s2048_L32_$i.txt python bench.py --batch 2048 --lanes 32 $S
  run 0 200 s2048_L64_$i.txt python bench.py --batch 2048 --lanes 64 $S
done
run 0 300 phases.txt env NOC_HIP_LIB=$L/libnoc_hip_prof.so python tools/persist_phases.py
run 0 300 wide_n400.txt python tools/wide_probe.py cartpole:400 pendulum:400
