"""Effective clock per kernel from one rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE ... run (MI355X_MICROARCH.md
'DVFS give-back': clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time), with the other counters of the pass per
dispatch.  Usage: python tools/pmc_clock.py <rocprofv3 output dir> [last N dispatches per kernel (default 200)]"""
import collections, csv, glob, re, statistics, sys

def kname(s):
    m = re.search(r"::(\w+?)(<[^(]*>)?\(", s)
    return m.group(1) if m else s.split("(")[0]

d = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 200
cc = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
dur = {}
for r in csv.DictReader(open(kt)):
    dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
vals = collections.defaultdict(dict)
names = {}
for r in csv.DictReader(open(cc)):
    vals[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    names[r["Dispatch_Id"]] = kname(r["Kernel_Name"])
per = collections.defaultdict(list)
for did in sorted(vals, key=int):
    if did in dur and dur[did] > 0:
        per[names[did]].append((did, dur[did], vals[did]))
for k, rows in per.items():
    rows = rows[-last:]
    clk = [v.get("GRBM_GUI_ACTIVE", 0) / 8 / t / 1e9 for _, t, v in rows]
    ms = [t * 1e3 for _, t, _ in rows]
    extra = {c: statistics.median(v[c] for _, _, v in rows) for c in rows[0][2] if c != "GRBM_GUI_ACTIVE"}
    print(f"{k:28s} n={len(rows):4d} ms median {statistics.median(ms):.4f}  clock GHz median {statistics.median(clk):.3f} "
          f"(min {min(clk):.3f} max {max(clk):.3f})  " + "  ".join(f"{c} {x:.4g}" for c, x in extra.items()))
