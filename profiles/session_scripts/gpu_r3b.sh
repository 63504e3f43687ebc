#!/bin/bash
# Round 3, session b: flip probe (decision-trace build of the round-2 kernels), the round-3 library
# (exec-masked Sklansky combines, closed-form nx = 2 solve) on every GPU test, c2 / c3 / shard
# bench lines, bench.py's own rank launcher rehearsed at world 2 and 4 (gloo, all ranks on
# cuda:0: timings meaningless).  pytest failures (rc 1) are reported and do not stop the session;
# a timeout or crash does.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r3b}; mkdir -p $O
export TMPDIR=/tmp
run() { local ok=$1; local t=$2; local log=$3; shift 3; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -3 "$O/$log" | cut -c1-600; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then exit $rc; fi; }
run 0 300 flip.txt env NOC_HIP_LIB="$R/ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_trace.so" python -u tools/flip_probe.py --out $O/flip.json
run 1 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
run 0 200 bench_c2.txt python bench.py --problem pendulum --horizon 100 --batch 1024 --steps 100 --warmup 10 --no-cpu --no-ipm
run 0 200 bench_c3.txt python bench.py --steps 20 --warmup 2 --no-cpu --no-ipm
for b in 512 1024 2048; do run 0 200 shard_$b.txt python bench.py --batch $b --steps 50 --warmup 5 --no-cpu --no-ipm; done
run 0 200 rehearsal_w2.txt env NOC_BENCH_REHEARSAL=1 python bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu
run 0 200 rehearsal_w4.txt env NOC_BENCH_REHEARSAL=1 python bench.py --gpus 4 --steps 5 --warmup 1 --no-cpu
