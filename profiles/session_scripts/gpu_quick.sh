#!/bin/bash
# GPU tests, smoke and the c3 bench line plus one non-default horizon (lanes policy in the bench blocks).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/quick; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run 200 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 200 n100.log python bench.py --horizon 100 --steps 30 --warmup 3 --no-cpu --no-ipm
run 300 bench_c3.log python bench.py
