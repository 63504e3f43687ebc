#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r23; mkdir -p $O
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; grep '"lanes": 32' "$O/$log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 200 a1.log python tools/kkt_sweep.py --configs c3 --lanes 32 --layouts tiled --rounds 7
NOC_HIP_LIB=$R/ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_fast.so run 200 b1.log python tools/kkt_sweep.py --configs c3 --lanes 32 --layouts tiled --rounds 7
run 200 a2.log python tools/kkt_sweep.py --configs c3 --lanes 32 --layouts tiled --rounds 7
NOC_HIP_LIB=$R/ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_fast.so run 200 b2.log python tools/kkt_sweep.py --configs c3 --lanes 32 --layouts tiled --rounds 7
