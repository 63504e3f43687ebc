#!/bin/bash
# c3 persistent-solve tail with the profile build (per-trajectory start / end stamps).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/tail2; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-900; if [ $rc -ne 0 ]; then exit $rc; fi; }
NOC_HIP_LIB=$L/libnoc_hip_prof.so run 300 tail_c3.log python tools/tail_probe.py --out $O
