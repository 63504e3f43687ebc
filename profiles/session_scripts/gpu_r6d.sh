#!/bin/bash
# Round 6, session d: per-phase and per-KKT-phase cycles of the structure-aware persistent solver
# (profile build; B = 1, 512, 4096), to see where a solve's time goes now that it is not
# traffic-bound.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r6d; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
NOC_HIP_LIB=$R/ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_prof.so run 300 phases.log python tools/persist_phases.py
