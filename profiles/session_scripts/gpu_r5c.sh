#!/bin/bash
# Round 5, session c: the DMA instance split into its two changes (tools/dma_ab.py: on-chip K, d
# vs K, d through HBM with plain phase-3 loads vs K, d through HBM + LDS-DMA phase 3), c3 and c5.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5c}; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 200 ab_c3.log python tools/dma_ab.py cartpole 200 4096
run 200 ab_c5.log python tools/dma_ab.py cartpole 200 8192
run 200 ab_c3_l64.log python tools/dma_ab.py cartpole 200 4096 64
