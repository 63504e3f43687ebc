#!/bin/bash
# Round 3, session x: the interior-point engine's workspace carved from one allocation per dtype
# (two fill launches instead of ~40) and the solver call copying results straight to the host --
# the host cost of a B = 1 call.  Every GPU test, then the B = 1 probe (kernel vs whole call) and
# the reference's runtime sweeps (compare profiles/r03/final_c/runtime/).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3x}; mkdir -p $O
export TMPDIR=/tmp
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
run 0 300 wide.txt python tools/wide_probe.py cartpole:100 cartpole:200 pendulum:100 pendulum:400
run 0 400 runtime_pendulum.txt python tools/runtime_sweep.py --problem pendulum --out $O/runtime --runs 5
run 0 400 runtime_cartpole.txt python tools/runtime_sweep.py --problem cartpole --out $O/runtime --runs 5
