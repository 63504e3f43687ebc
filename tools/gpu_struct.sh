#!/bin/bash
# Round 6: the structure-aware persistent solver -- its parity tests (bit-identical to the dense
# instance; resume / cap / probe order), smoke, the c3 / c2 bench lines (ipm_solve) and the
# one-GPU slice curve (tools/slice_curve.py).  Usage: gpurun --timeout 1200 -- bash tools/gpu_struct.sh [OUT]
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${1:-struct}; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -2 "$O/$log" | cut -c1-600; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 500 pytest_struct.log python -u -m pytest tests/test_ipm_gpu.py -x -v --timeout 120 --timeout-method thread -k "structured or persistent or resumed or probe or repeats or cost_ordered"
run 200 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 300 bench_c3.log python bench.py
run 300 bench_c2.log python bench.py --problem pendulum --horizon 100 --batch 1024 --steps 100 --warmup 10 --no-cpu
run 600 slices.log python tools/slice_curve.py --out $O/slices.json
