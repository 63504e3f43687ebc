#!/bin/bash
# Round 6, session b: the whole GPU suite on the structure-aware persistent solvers (+ rp_shrink,
# provenance), their phase cycles (profile build, struct vs dense, B = 1 / 512 / 4096), the
# two-wave wide instance on the 8-GPU slices (512 per GPU), an A/B of raised wave priority for the
# costliest trajectories, and the c3 solve's SQ / traffic counters.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r6b; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -2 "$O/$log" | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 800 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run 300 slices8_onewave.log python tools/slice_curve.py --ws 8 --out $O/slices8_onewave.json
NOC_PERSIST_WIDE=1 run 300 slices8_wide2.log python tools/slice_curve.py --ws 8 --out $O/slices8_wide2.json
NOC_PERSIST_WIDE=1 NOC_WIDE_WAVES=4 run 300 slices8_wide4.log python tools/slice_curve.py --ws 8 --out $O/slices8_wide4.json
NOC_HIP_LIB=$R/ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_prof.so run 300 phases.log python tools/persist_phases.py
for rnd in 1 2; do
  for p in 0 256 1024; do
    NOC_PERSIST_PRIO=$p run 120 prio_${p}_$rnd.log python tools/ipm_bench.py cartpole 200 4096 persistent
  done
done
OUT=r6b/counters bash profiles/session_scripts/gpu_r5q1.sh
