#!/bin/bash
# Round 5, session o: kernel traces of the 512-shard bench with the round-4 and the current
# library (which kernels run, and how long each takes).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5o}; mkdir -p $O
export TMPDIR=/tmp
L="$R/ip-parallel-optimal-control_amd/noc/_lib"
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-120; if [ $rc -ne 0 ]; then exit $rc; fi; }
A="--steps 50 --warmup 5 --no-cpu --no-ipm --global-batch 512"
for i in 1 2; do
  NOC_HIP_LIB=$L/libnoc_hip_old.so run 240 old_trace_$i.log rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/old_$i" -o run -- python "$R/bench.py" $A
  run 240 new_trace_$i.log rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/new_$i" -o run -- python "$R/bench.py" $A
done
