#!/usr/bin/env python3
"""Summarise an interleaved A/B directory of bench lines (tools/gpu_ab.sh: old_<cfg>_<i>.log /
new_<cfg>_<i>.log): per config the per-round kernel times (roofline.kernel_ms, HIP events on the
kernel's stream) and bench ms_per_step of both builds, in us.  Usage: ab_summary.py <dir>"""
import glob, json, os, re, sys
from collections import defaultdict

d = sys.argv[1]
rows = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "*_*_*.log"))):
    m = re.match(r"(\w+?)_(\w+)_(\d+)\.log", os.path.basename(f))
    if not m:
        continue
    who, cfg, _ = m.groups()
    for ln in open(f):
        if ln.startswith("{"):
            j = json.loads(ln)
            rows[cfg][who].append((round(j["roofline"]["kernel_ms"] * 1e3, 2), round(j["ms_per_step"] * 1e3, 2)))
for cfg, by in rows.items():
    print(cfg, {w: v for w, v in sorted(by.items())})
