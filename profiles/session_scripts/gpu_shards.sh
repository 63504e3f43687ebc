#!/bin/bash
# Strong-scaling shards of the north-star curve (cart-pole N=200, global batch 4096 over 1/2/4/8
# GPUs -> 4096/2048/1024/512 per GPU) on one GPU: lanes sweep per shard size; plus a gloo
# rehearsal of bench.py's N > 1 path (all ranks on cuda:0; timings meaningless) and the real-engine
# sharded test.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/shards; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="--steps 50 --warmup 5 --no-cpu --no-ipm"
for g in 4096 2048 1024 512; do
  for L in 0 16 32 64; do
    run 200 g${g}_L${L}.log python bench.py $B --global-batch $g --lanes $L
  done
done
run 300 rehearsal_w2.log env NOC_BENCH_REHEARSAL=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29517 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu
run 300 rehearsal_w4.log env NOC_BENCH_REHEARSAL=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr=127.0.0.1 --master-port=29519 bench.py --gpus 4 --steps 10 --warmup 2 --no-cpu --no-ipm
run 400 pytest_dist.log python -u -m pytest tests/test_distributed_gpu.py tests/test_distributed.py -x -v --timeout 300 --timeout-method thread
