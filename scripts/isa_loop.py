"""Instruction histogram of the innermost loops of a kernel in a hipcc -S listing (gfx950).
Usage: python scripts/isa_loop.py listing.s <kernel-name-substring> [depth]"""
import collections
import re
import sys

src, name = sys.argv[1], sys.argv[2]
depth = sys.argv[3] if len(sys.argv) > 3 else None
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(name) + r"\S*:", l))
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
body = lines[start:end]
# blocks tagged "in Loop: Header=H Depth=d" or the header itself
loops = collections.defaultdict(list)
cur = None
for l in body:
    m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):\s*;.*(?:Header=(BB\d+_\d+)|Loop Header: Depth=(\d+))", l)
    if re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):", l):
        h = re.search(r"Header=(BB\d+_\d+) Depth=(\d+)", l)
        hh = re.search(r"Loop Header: Depth=(\d+)", l)
        lab = l.split(":")[0].lstrip(". ")
        if hh:
            cur = (lab, hh.group(1))
        elif h:
            cur = (h.group(1), h.group(2))
        else:
            cur = None
        continue
    if cur and l.startswith("\t") and not l.strip().startswith(";"):
        loops[cur].append(l.split()[0])
for (hdr, d), ins in sorted(loops.items(), key=lambda x: -len(x[1])):
    if depth and d != depth:
        continue
    c = collections.Counter(ins)
    valu = sum(v for k, v in c.items() if k.startswith("v_") and not k.startswith("v_mfma") and "readfirstlane" not in k)
    print(f"loop {hdr} depth {d}: {len(ins)} instr, VALU {valu}, SALU {sum(v for k, v in c.items() if k.startswith('s_'))}, "
          f"LDS {sum(v for k, v in c.items() if k.startswith('ds_'))}, MFMA {c['v_mfma_f32_16x16x32_bf16']}, "
          f"exp {c['v_exp_f32_e32']}")
    if "-v" in sys.argv:
        for k, v in c.most_common():
            print(f"   {v:4d} {k}")
