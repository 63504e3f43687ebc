#!/bin/bash
# Round 3, session g: traced user costs / state constraints (register_family(stage_cost=...,
# final_cost=..., constraints=...)) -- every GPU test; the built-ins must be unchanged.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3g}; mkdir -p $O
export TMPDIR=/tmp
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -3 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
run 0 200 bench_c3.txt python bench.py --steps 20 --warmup 2 --no-cpu
