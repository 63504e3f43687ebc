#!/bin/bash
# Round 6 final, part c (speculative candidates on by default): the whole GPU suite, smoke, the
# c3 / c2 / one-rank torchrun bench lines, the slice curve and the reference's cart-pole runtime
# sweep at B = 1 (par, seq, DDP), all on the final build.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r6final_c}; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 800 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 300 bench_c3.log python bench.py
run 300 bench_c2.log python bench.py --problem pendulum --horizon 100 --batch 1024 --steps 100 --warmup 10 --no-cpu
run 300 bench_torchrun1.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu
run 300 slices.log python tools/slice_curve.py --out $O/slices.json
run 400 runtime_cartpole.log python tools/runtime_sweep.py --problem cartpole --out $O/runtime
