#!/bin/bash
# Round 3, session u: the wide (four waves per trajectory) solver's forward affine scan as a VALU
# Sklansky scan (was Hillis-Steele through ds_bpermute), DPP by-one hand-offs and VALU workgroup
# reductions.  Every GPU test first (the wide == one-wave checks pin the new association), then
# the B = 1 probe against HEAD (libnoc_hip_A.so), interleaved, and the phase cycles.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3u}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
P="cartpole:100 cartpole:200 cartpole:400 pendulum:100 pendulum:400"
for i in 1 2; do
  run 0 300 wide_A_$i.txt env NOC_HIP_LIB=$L/libnoc_hip_A.so python tools/wide_probe.py $P
  run 0 300 wide_B_$i.txt python tools/wide_probe.py $P
done
run 0 300 wide_prof.txt env NOC_HIP_LIB=$L/libnoc_hip_prof.so python tools/wide_probe.py cartpole:200 pendulum:100
