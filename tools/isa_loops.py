"""Instruction counts per innermost loop of one kernel in an `-S` listing (blocks grouped by the loop header
LLVM's block comments name).  Usage: python tools/isa_loops.py <file.s> <kernel-symbol-substring>"""
import re, sys, collections
L = open(sys.argv[1]).read().split("\n")
sym = sys.argv[2]
st = next(i for i, l in enumerate(L) if l.startswith("_Z") and sym in l.split(":")[0] and l.split(";")[0].rstrip().endswith(":"))
en = next(i for i in range(st, len(L)) if "s_endpgm" in L[i])
loop = None          # innermost loop header of the current block
depth = {}
ops = collections.defaultdict(list)
for i in range(st, en + 1):
    raw = L[i]
    s = raw.strip()
    if re.match(r"^(\.LBB\w+|; %bb\.\d+):", s) or (s.startswith(";") and "Loop" in s):
        m = re.search(r"in Loop: Header=(BB\w+) Depth=(\d+)", s)
        if re.match(r"^(\.LBB\w+|; %bb\.\d+):", s):
            loop = None
            if m:
                loop = m.group(1); depth[loop] = int(m.group(2))
            lab = re.match(r"^\.?L?(BB\w+)|^; %bb", s)
            hdr = re.match(r"^\.L(BB\w+):", s)
            if hdr and "Parent Loop" in s or (hdr and "Loop Header" in s):
                loop = hdr.group(1)
            cur_label = hdr.group(1) if hdr else None
        if "Loop Header" in s:
            m2 = re.search(r"Depth=(\d+)", s)
            if cur_label:
                loop = cur_label; depth[loop] = int(m2.group(1))
        continue
    if not s or s.startswith((".", ";")):
        continue
    if loop:
        ops[loop].append(s.split()[0])
for lp, o in sorted(ops.items(), key=lambda kv: -len(kv[1])):
    c = lambda f: sum(1 for x in o if f(x))
    print(f"{lp:10s} depth={depth.get(lp, '?')} instrs {len(o):5d}  pk_fma {c(lambda x: x.startswith('v_pk_fma')):3d}  "
          f"f64 {c(lambda x: '_f64' in x and 'cvt' not in x):4d}  cvt {c(lambda x: 'cvt' in x):3d}  lds {c(lambda x: x.startswith('ds_')):3d}  "
          f"vmem {c(lambda x: x.startswith(('global_', 'buffer_'))):3d}  salu {c(lambda x: x.startswith('s_')):4d}")
