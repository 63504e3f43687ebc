#!/bin/bash
# Round 5, session f: A, B slots in LDS for the SIMD-owning scan instances (interleaved A/B against
# the round-4 scan, tools/gpu_ab.sh: shards + c3 control, then the KKT / golden / IPM tests), then
# the DDP tests and the one-stage DDP flip probe (oracle cube as JAX integer_pow).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5f}; mkdir -p $O
export TMPDIR=/tmp
OUT=${OUT:-r5f} ROUNDS=3 bash tools/gpu_ab.sh s1024 s512 s2048 c3 || exit 1
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 300 ddp_probe.log python tools/ddp_flip_probe.py
run 600 pytest_ddp.log python -u -m pytest tests/test_ddp.py -m gpu -q --timeout 300 --timeout-method thread -rf
