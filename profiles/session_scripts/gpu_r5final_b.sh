#!/bin/bash
# Round 5 final, part b: same-build kernel traces + calibrated FETCH_SIZE / WRITE_SIZE passes of
# every bench configuration (c3, c2, c4 and the strong-scaling shards), written to
# $O/prof/pmc_traffic.json stamped with the KKT source hash (profiles/session_scripts/gpu_final_r3.sh).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5final_b}; mkdir -p $O
export TMPDIR=/tmp
OUT=${OUT:-r5final_b}/prof bash profiles/session_scripts/gpu_final_r3.sh || exit 1
