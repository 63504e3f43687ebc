#!/usr/bin/env python3
"""Per-level / per-phase instruction counts of a KKT scan kernel from its gfx950 assembly (built
with -DNOC_ISA_MARKS: assembler comments at every scan level and phase boundary).

  python tools/isa_levels.py <file.s> <kernel-substring>   (e.g. 'ILi2ELi1ELi64ELb0ELb1ELi2E')

Counts, between consecutive markers of the kernel: all instructions, VALU (v_*), fp64 FMA/MUL/ADD,
DPP movs, v_readlane, LDS (ds_*), divisions (v_div_scale_f64 = one fp64 division), waits."""
import re
import sys


def kernel_body(lines, sub):
    start = None
    for i, ln in enumerate(lines):
        if start is None and ln.startswith("_Z") and sub in ln.split(":")[0]:
            start = i
        elif start is not None and ln.strip().startswith(".Lfunc_end"):
            return lines[start:i]
    raise SystemExit(f"kernel matching {sub!r} not found")


def classify(body):
    seg, name, out = [], "entry", []
    for ln in body:
        m = re.search(r"; NOC_MARK (\w+) (\d+)", ln)
        if m:
            out.append((name, seg))
            name, seg = f"{m.group(1)}{m.group(2)}", []
            continue
        t = ln.strip()
        if not t or t.startswith((";", ".", "_")) or t.endswith(":"):
            continue
        seg.append(t.split()[0])
    out.append((name, seg))
    return out


def stats(ops):
    return dict(total=len(ops), valu=sum(o.startswith("v_") for o in ops),
                f64=sum(o.endswith("_f64") for o in ops),
                dpp=sum("dpp" in o for o in ops), readlane=sum("readlane" in o for o in ops),
                lds=sum(o.startswith("ds_") for o in ops),
                div=sum(o.startswith("v_div_scale_f64") for o in ops) // 2,
                rcp=sum(o.startswith("v_rcp_f64") for o in ops),
                wait=sum(o.startswith("s_waitcnt") for o in ops))


def main():
    path, sub = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    for name, ops in classify(kernel_body(lines, sub)):
        print(f"{name:8s} " + " ".join(f"{k}={v}" for k, v in stats(ops).items()))


if __name__ == "__main__":
    main()
