#!/usr/bin/env python3
"""Per-launch HBM traffic of the KKT scan from rocprofv3 --pmc CSVs (separate FETCH_SIZE and
WRITE_SIZE passes) of the KKT kernel (name filter, default "kkt_"), corrected as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE (KB) counts half
the bytes of 16-byte-per-lane coalesced reads on gfx950, and the calibration of the scan's other
access widths (tools/pmc_calib.hip, profiles/r02/pmc_calib: 8 B/lane reads, contiguous or as the
L = 32 two-piece tiled pattern, also count half; 8 and 16 B/lane stores count exactly) extends
that to the whole kernel: bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  Writes
profiles/pmc_traffic.json."""
import csv, json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "ip-parallel-optimal-control_amd"))
from noc._lib import source_hash  # noqa: E402  (pure Python: no library load)
fetch_csv, write_csv, key, out = sys.argv[1:5]
kname = sys.argv[5] if len(sys.argv) > 5 else "kkt_scan"  # or kkt_group8

def mean(path, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kname in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return sum(vals) / len(vals), len(vals)

f, nf = mean(fetch_csv, "FETCH_SIZE")
w, nw = mean(write_csv, "WRITE_SIZE")
try:
    d = json.load(open(out))
except Exception:
    d = {}
d[key] = (2 * f + w) * 1024
d[key + "_raw"] = {"FETCH_SIZE_KB": f, "WRITE_SIZE_KB": w, "launches": [nf, nw],
                   "kernel_filter": kname, "source_hash": source_hash(kname),
                   "fetch_csv": fetch_csv, "write_csv": write_csv,
                   "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950; calibrated for 16 and 8 B/lane reads and stores, profiles/r02/pmc_calib)"}
json.dump(d, open(out, "w"), indent=1)
print(key, d[key])
