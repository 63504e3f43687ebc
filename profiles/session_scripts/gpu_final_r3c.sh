#!/bin/bash
# Round 3 closing run on the committed tree: the c4 trace + PMC passes (its source hash moved with
# noc_internal.h), then the full validation of tools/gpu_final_r3b.sh (every GPU test, smoke, the
# c3 / c2 / c4 bench lines, the world-2 rehearsal, the B = 1 runtime sweeps) against that traffic.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/final_r3c
OUT=final_r3c/pmc CONFIGS="c4" bash tools/gpu_final_r3.sh || exit $?
cp gpurun_out/final_r3c/pmc/pmc_traffic.json profiles/pmc_traffic.json
OUT=final_r3c bash tools/gpu_final_r3b.sh
