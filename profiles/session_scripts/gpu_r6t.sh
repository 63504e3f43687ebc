#!/bin/bash
# Round 6, session t: the 4-GPU slice size (1024 cart-poles, one wave per SIMD) with the probe
# order and the costliest H trajectories on two speculative candidates each beside the rest on
# the one-wave instance (NOC_PERSIST_HEAVY=H, NOC_PERSIST_HEAVY_SPEC=2), against the default
# (tail schedule) and the plain probe schedule; repeated solves in one process.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r6t; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 300 heavy_spec_1024.log python tools/heavy_spec.py --B 1024
run 300 heavy_spec_2048.log python tools/heavy_spec.py --B 2048 --H 128,256,512
