#!/bin/bash
# Round 3, session a: decision traces of the wide vs one-wave persistent solvers (flip root cause,
# trace build), bench.py's own rank launcher rehearsed at world 2 and 4 (gloo, all ranks on
# cuda:0: timings meaningless), and the wide / ABI GPU tests.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r3a; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -2 "$O/$log" | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 300 flip.txt env NOC_HIP_LIB="$R/ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_trace.so" python -u tools/flip_probe.py --out $O/flip.json
run 300 pytest_wide.txt python -u -m pytest tests/test_ipm_gpu.py tests/test_abi.py -x -q --timeout 120 --timeout-method thread -m gpu -k "wide or abi or cap or order"
run 200 rehearsal_w2.txt env NOC_BENCH_REHEARSAL=1 python bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu
run 200 rehearsal_w4.txt env NOC_BENCH_REHEARSAL=1 python bench.py --gpus 4 --steps 5 --warmup 1 --no-cpu
