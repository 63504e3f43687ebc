#!/bin/bash
# Round 6, session e: the exact two-period wrap_angle fast path (cart-pole's theta lives around
# 2 pi: the fmod loop ran in every stage cost / gradient) -- the GPU suite, the phase cycles, the
# c3 / c2 bench lines and the slice curve.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r6e; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 800 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
NOC_HIP_LIB=$R/ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_prof.so run 300 phases.log python tools/persist_phases.py
run 300 bench_c3.log python bench.py
run 300 bench_c2.log python bench.py --problem pendulum --horizon 100 --batch 1024 --steps 100 --warmup 10 --no-cpu
run 300 slices.log python tools/slice_curve.py --out $O/slices.json
