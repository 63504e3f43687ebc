#!/bin/bash
# Round 5: batches beyond one resident round of waves, whole launch (NOC_KKT_SLICE=0) vs
# consecutive one-round launches (default), same build, interleaved bench lines.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r5t; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="--steps 50 --warmup 5 --no-cpu --no-ipm"
for i in 1 2; do
  NOC_KKT_SLICE=0 run 200 whole_c5_$i.log python bench.py $B --batch 8192
  run 200 slice_c5_$i.log python bench.py $B --batch 8192
  NOC_KKT_SLICE=0 run 200 whole_b16k_$i.log python bench.py $B --batch 16384
  run 200 slice_b16k_$i.log python bench.py $B --batch 16384
  NOC_KKT_SLICE=0 run 200 whole_pend8k_$i.log python bench.py $B --problem pendulum --horizon 100 --batch 8192
  run 200 slice_pend8k_$i.log python bench.py $B --problem pendulum --horizon 100 --batch 8192
  run 200 c3_$i.log python bench.py $B
done
run 600 pytest_kkt.log python -u -m pytest tests/test_kkt_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
