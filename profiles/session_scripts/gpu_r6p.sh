#!/bin/bash
# Round 6, session p: the tail schedule restricted to one wave per SIMD -- parity tests, the c3
# slice curve, bench c3 (unchanged path) and the tail ladders at 1024 again.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r6p; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-250; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 500 pytest_tail.log python -u -m pytest tests/test_ipm_gpu.py -x -v --timeout 200 --timeout-method thread -k "tail_schedule or speculative"
run 300 tail_caps.log python tools/tail_caps.py --B 1024 --ladders "off;256,384,512;224,320,448;288,384,512"
run 300 slices.log python tools/slice_curve.py --out $O/slices.json
