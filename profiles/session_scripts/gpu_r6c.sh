#!/bin/bash
# Round 6, session c: what bounds c3 ipm_solve with the compact blocks -- the heavy-first split
# (the costliest trajectories on the one-wave instance beside the two-wave launch), the one-wave
# instance for the whole batch, the probe length, and the per-trajectory timeline.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r6c; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 300 pytest.log python -u -m pytest tests/test_ipm_gpu.py -x -q --timeout 200 --timeout-method thread -k "heavy or structured"
for rnd in 1 2; do
  for h in 0 64 128 256; do
    NOC_PERSIST_HEAVY=$h run 120 heavy_${h}_$rnd.log python tools/ipm_bench.py cartpole 200 4096 persistent
  done
  NOC_PERSIST_WAVES=1 run 120 waves1_$rnd.log python tools/ipm_bench.py cartpole 200 4096 persistent
done
for p in 16 24 48; do
  PROBE_SOLVES=$p run 120 probe_$p.log python tools/ipm_bench.py cartpole 200 4096 persistent
done
NOC_HIP_LIB=$R/ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_prof.so TAIL_TAG=h0 run 200 tail_h0.log python tools/tail_probe.py --reps 1 --out $O/tail
