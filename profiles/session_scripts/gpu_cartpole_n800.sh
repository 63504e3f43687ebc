#!/bin/bash
# Cart-pole B=1 at the runtime-sweep inputs, N = 400..1000, at 1 and 2 waves per SIMD (tools/n800_probe.py).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/n800b; mkdir -p $O
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; grep '^{' "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
NOC_PERSIST_WAVES=1 run 200 w1.log python tools/n800_probe.py
NOC_PERSIST_WAVES=2 run 200 w2.log python tools/n800_probe.py
