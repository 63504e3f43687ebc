#!/bin/bash
# c4 group solve: backward / forward sweep split by ablation (timing only).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/c4_ablate; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-600; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 300 c4_ablate.log python tools/kkt_ablate.py linear8 512 16384 1
