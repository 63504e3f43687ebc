#!/bin/bash
# Timeline of the c3 persistent solve (profile build: per-trajectory start / end stamps) with and
# without the heavy-first split; saves per-trajectory computed solves, times and the launch order.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5h3}; mkdir -p $O
export TMPDIR=/tmp
export NOC_HIP_LIB=$R/ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_prof.so
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-600; if [ $rc -ne 0 ]; then exit $rc; fi; }
for h in 0 64; do
  NOC_PERSIST_HEAVY=$h run 120 tail_h$h.json python tools/tail_probe.py --reps 2 --out $O
done
