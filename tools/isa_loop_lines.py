"""Source lines of each innermost loop of one kernel in an `-S -gline-tables-only` listing: per loop header, the
instruction count and the three source lines contributing most instructions, plus SALU / branch counts.
Usage: python tools/isa_loop_lines.py <file.s> <kernel-symbol-substring> [max loops]"""
import re, sys, collections
L = open(sys.argv[1]).read().split("\n")
sym = sys.argv[2]
nmax = int(sys.argv[3]) if len(sys.argv) > 3 else 25
st = next(i for i, l in enumerate(L) if l.startswith("_Z") and sym in l.split(":")[0] and l.split(";")[0].rstrip().endswith(":"))
en = next(i for i in range(st, len(L)) if "s_endpgm" in L[i])
loop, loc = "entry", None
lines = collections.defaultdict(collections.Counter)
cnt = collections.defaultdict(collections.Counter)
for i in range(st, en + 1):
    s = L[i].strip()
    m = re.match(r"^(\.LBB\w+|; %bb\.\d+):(.*)", s)
    if m:
        c = m.group(2)
        j = i + 1
        while j < len(L) and L[j].strip().startswith(";"):
            c += L[j]; j += 1
        h = re.search(r"Header=(BB\w+)", c)
        loop = h.group(1) if h else (m.group(1)[2:] if "Loop Header" in c else "straight")
        continue
    m = re.match(r"\.loc\s+\d+\s+(\d+)", s)
    if m:
        loc = int(m.group(1))
        continue
    if not s or s.startswith((".", ";")):
        continue
    op = s.split()[0]
    lines[loop][loc] += 1
    cnt[loop]["all"] += 1
    if op.startswith("s_") and not op.startswith(("s_waitcnt", "s_cbranch", "s_branch", "s_nop")):
        cnt[loop]["salu"] += 1
    if op.startswith(("s_cbranch", "s_branch")):
        cnt[loop]["br"] += 1
for lp, c in sorted(cnt.items(), key=lambda kv: -kv[1]["all"])[:nmax]:
    top = ", ".join(f"{k}:{v}" for k, v in lines[lp].most_common(4))
    print(f"{lp:10s} n={c['all']:5d} salu={c['salu']:4d} br={c['br']:3d}  lines {top}")
