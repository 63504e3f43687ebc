#!/bin/bash
# Round 4, session f: the DDP module's building blocks on the device (bwd_pass, nonlin_rollout,
# one-stage ddp) -- every GPU test, smoke, then the reference's B = 1 runtime sweeps.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r4f}; mkdir -p $O
export TMPDIR=/tmp
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
run 0 200 smoke.txt python -c "import __graft_entry__ as g; g.smoke()"
