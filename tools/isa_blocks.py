#!/usr/bin/env python3
"""Per-basic-block instruction counts of one kernel in a gfx950 assembly file (hipcc -S
--cuda-device-only; with -DNOC_ISA_MARKS the scan's level / phase markers are listed per block).
Splits at both .LBB labels and the unlabelled fall-through blocks ("; %bb.N:"), so a level's
executed path can be told apart from a skipped fallback block (e.g. the partial-pivoting solve).

  python tools/isa_blocks.py <file.s> <kernel-name-substring>

Columns: instructions, VALU, fp64 (any *_f64 op), v_cndmask, DPP moves, v_readlane, scratch
accesses, branch targets, markers."""
import sys,re,collections
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.abspath(__file__)))
import isa_levels as I
lines=open(sys.argv[1]).read().splitlines()
body=I.kernel_body(lines,sys.argv[2])
blocks=[];name='entry';ops=[]
for ln in body:
    t=ln.strip()
    m=re.match(r'^(\.LBB[\w_]+):',t) or re.match(r'^; (%bb\.\d+):',t)
    if m:
        blocks.append((name,ops)); name=m.group(1); ops=[]; continue
    mm=re.search(r'; NOC_MARK (\w+) (\d+)',t)
    if mm: ops.append('MARK_'+mm.group(1)+mm.group(2)); continue
    if not t or t.startswith((';','.','_')): continue
    ops.append(t)
blocks.append((name,ops))
for i,(n,ops) in enumerate(blocks):
    ins=[o for o in ops if not o.startswith('MARK')]
    c=collections.Counter(o.split()[0] for o in ins)
    valu=sum(v for k,v in c.items() if k.startswith('v_'))
    f64=sum(v for k,v in c.items() if '_f64' in k)
    cnd=sum(v for k,v in c.items() if 'cndmask' in k)
    dpp=c['v_mov_b32_dpp']; rl=c['v_readlane_b32']
    br=[o.split()[-1] for o in ins if o.startswith(('s_cbranch','s_branch'))]
    marks=[o for o in ops if o.startswith('MARK')]
    print(f"{i:3d} {n:12s} n={len(ins):5d} valu={valu:5d} f64={f64:4d} cnd={cnd:4d} dpp={dpp:4d} rl={rl:4d} scr={sum(v for k,v in c.items() if 'scratch' in k)} br={br} {marks}")
