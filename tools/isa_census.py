"""Static instruction census of one kernel in a `-gline-tables-only -S` listing: instructions per source line
(by the nearest preceding .loc), split into VALU f64 / other VALU / SALU / LDS / VMEM, with loop back-edges
marked.  Usage: python tools/isa_census.py <file.s> <kernel-symbol-substring> [top N]"""
import re, sys, collections

path, sym = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l and l.rstrip().endswith(":") or
             (l.startswith("_Z") and sym in l.split(":")[0]))
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
files = {}
for l in lines:
    m = re.match(r"\s*\.file\s+(\d+)\s+\"([^\"]*)\"(?:\s+\"([^\"]*)\")?", l)
    if m:
        files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
cur = "?"
cnt = collections.defaultdict(collections.Counter)
tot = collections.Counter()
labels = {}
for i in range(start, end + 1):
    l = lines[i].strip()
    m = re.match(r"\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        cur = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
        continue
    if not l or l.startswith((".", ";")) or l.endswith(":"):
        continue
    op = l.split()[0]
    if op.startswith("v_"):
        k = "f64" if ("_f64" in op and "cvt" not in op) or op.startswith("v_mfma_f64") else "valu"
    elif op.startswith("s_"):
        k = "salu"
    elif op.startswith("ds_"):
        k = "lds"
    elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        k = "vmem"
    else:
        k = "other"
    cnt[cur][k] += 1
    tot[k] += 1
print("total", dict(tot), "instructions", sum(tot.values()))
rows = sorted(cnt.items(), key=lambda kv: -sum(kv[1].values()))
for src, c in rows[:top]:
    print(f"{src:28s} {sum(c.values()):6d}  f64 {c['f64']:5d} valu {c['valu']:5d} salu {c['salu']:5d} lds {c['lds']:4d} vmem {c['vmem']:4d}")
