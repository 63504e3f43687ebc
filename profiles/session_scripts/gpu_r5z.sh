#!/bin/bash
# Round 5: the final phase-3 cache policy (two-wave instance and large-batch L = 32 instance
# non-temporal, 512-register instances default) vs the previous scan, interleaved bench lines.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=${ABOUT:-r5z} ROUNDS=2 bash tools/gpu_ab.sh ${ABCFG:-c3 c5 s2048 s512 s1024 c2} || exit $?
