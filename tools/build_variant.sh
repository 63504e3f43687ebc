#!/bin/bash
# Build a variant of libnoc_hip.so for an interleaved A/B (tools/gpu_ab.sh loads it through
# NOC_HIP_LIB): the current sources with some files replaced by another git revision's, compiled
# in a scratch copy of the package and written to noc/_lib/libnoc_hip_<name>.so.
# Usage: tools/build_variant.sh <name> <rev> <file under csrc/>...
set -e
name=$1; rev=$2; shift 2
R="$(cd "$(dirname "$0")/.." && pwd)"
P="$R/ip-parallel-optimal-control_amd"
T=$(mktemp -d /tmp/noc_variant.XXXX)
mkdir -p "$T/pkg" "$T/include"
cp -r "$P/csrc" "$P/Makefile" "$T/pkg/"
cp "$R/include/noc_hip.h" "$T/include/"
for f in "$@"; do git -C "$R" show "$rev:ip-parallel-optimal-control_amd/csrc/$f" > "$T/pkg/csrc/$f"; done
make -C "$T/pkg" -j"${JOBS:-8}" > "$T/build.log" 2>&1 || { tail -20 "$T/build.log"; exit 1; }
cp "$T/pkg/noc/_lib/libnoc_hip.so" "$P/noc/_lib/libnoc_hip_$name.so"
rm -rf "$T"
echo "built $P/noc/_lib/libnoc_hip_$name.so ($rev: $*)"
