#!/bin/bash
# Round 4, session e: interior-point DDP with the full stage-cost Hessian in its record (traced
# costs): every GPU test (the new DDP parity test on the track-limited cart-pole included), then
# the reference's B = 1 runtime sweeps (DDP counts and times against session b).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r4e}; mkdir -p $O
export TMPDIR=/tmp
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
run 0 400 runtime_pendulum.txt python tools/runtime_sweep.py --problem pendulum --out $O/runtime --runs 5
run 0 600 runtime_cartpole.txt python tools/runtime_sweep.py --problem cartpole --out $O/runtime --runs 5
