#!/bin/bash
# Round 5, session b: the LDS-DMA phase-3 scan instance (c3).  Parity first (the new DMA tests and
# the tiled / no-gains / full-size KKT tests), then interleaved bench lines NOC_KKT_DMA=0 (the
# on-chip-gains instance, round-4 code path) vs default (DMA), then phase stamps of both.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5b}; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 600 pytest_dma.log python -u -m pytest tests/test_kkt_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "dma or tiled or without_gains or full_size or cartpole_blocks"
B="--steps 50 --warmup 5 --no-cpu --no-ipm"
for i in 1 2 3; do
  NOC_KKT_DMA=0 run 200 lds_c3_$i.log python bench.py $B
  run 200 dma_c3_$i.log python bench.py $B
done
for i in 1 2; do
  NOC_KKT_DMA=0 run 200 lds_c5_$i.log python bench.py $B --batch 8192
  run 200 dma_c5_$i.log python bench.py $B --batch 8192
done
NOC_KKT_DMA=0 run 200 stamps_lds.log python tools/scan_stamps.py cartpole 200 4096
run 200 stamps_dma.log python tools/scan_stamps.py cartpole 200 4096
