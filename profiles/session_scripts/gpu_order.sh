#!/bin/bash
# Launch order by descending initial cost (BatchedIPM.launch_order): IPM GPU tests, c3 persistent
# solve in index order vs cost order (interleaved), and the default bench line.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/order; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-330; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 600 pytest_ipm.log python -u -m pytest tests/test_ipm_gpu.py tests/test_api_gpu.py tests/test_abi.py -x -q --timeout 200 --timeout-method thread
for i in 1 2; do
  NOC_SCHEDULE=index run 300 c3_index_$i.log python tools/ipm_bench.py cartpole 200 4096 persistent
  NOC_SCHEDULE=auto run 300 c3_cost_$i.log python tools/ipm_bench.py cartpole 200 4096 persistent
done
run 300 bench_c3.log python bench.py
