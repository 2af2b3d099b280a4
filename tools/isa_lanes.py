"""Per-source-line count of chosen opcodes inside one loop (the loop's header block and every block LLVM's comments
place in it, nested loops included) of an `-S -gline-tables-only` listing.
Usage: python tools/isa_lanes.py <file.s> <loop header, e.g. BB0_72> [opcode prefix ...]"""
import re, sys, collections
L = open(sys.argv[1]).read().split("\n")
hdr = sys.argv[2]
ops = tuple(sys.argv[3:]) or ("v_readlane_b32", "v_writelane_b32", "scratch_")
inside, loc = False, None
cnt, tot = collections.Counter(), collections.Counter()
for i, raw in enumerate(L):
    s = raw.strip()
    m = re.match(r"^(\.LBB\w+):(.*)", s)
    if m:
        c = m.group(2)
        j = i + 1
        while j < len(L) and L[j].strip().startswith(";"):
            c += L[j]; j += 1
        inside = (m.group(1) == "." + "L" + hdr) or (hdr + " " in c + " ") or ("Header=" + hdr + " " in c + " ")
        continue
    m = re.match(r"\.loc\s+\d+\s+(\d+)", s)
    if m:
        loc = int(m.group(1))
    if s.startswith("s_endpgm"):
        inside = False
    if inside and s and not s.startswith((".", ";")):
        op = s.split()[0]
        tot["all"] += 1
        if op.startswith(ops):
            cnt[(loc, op)] += 1
            tot[op] += 1
print(dict(tot))
for k, v in sorted(cnt.items()):
    print(k, v)
