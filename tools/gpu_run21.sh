#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r21; mkdir -p $O
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -4 "$O/$log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
NOC_HIP_LIB=$R/ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_prof.so run 300 phases.log python tools/persist_phases.py
