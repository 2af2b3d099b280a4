"""Summarise rocprofv3 --pmc CSVs (FETCH_SIZE / WRITE_SIZE, KB per dispatch) per kernel.
Usage: python tools/pmc_summary.py <dir-with-pmc_fetch-and-pmc_write> <out.json> [robot samples]
gfx950 note (MI355X_MICROARCH.md §HBM): FETCH_SIZE reads 1/2 of the bytes of wide coalesced streaming
reads; both the raw value and the x2-corrected value are reported."""
import collections, csv, json, re, sys

def kname(s):
    m = re.search(r"::(\w+?)(<[^(]*>)?\(", s)
    return m.group(1) if m else s.split("(")[0]

d = sys.argv[1]
out = {}
for f in ("pmc_fetch", "pmc_write"):
    rows = list(csv.DictReader(open(f"{d}/{f}/run_counter_collection.csv")))
    agg = collections.defaultdict(list)
    for r in rows:
        agg[(kname(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in agg.items():
        out.setdefault(k, {})[c + "_KB_per_dispatch"] = sum(v) / len(v)
        out[k]["dispatches"] = len(v)
for k, v in out.items():
    if "FETCH_SIZE_KB_per_dispatch" in v:
        v["FETCH_bytes_corrected_x2"] = v["FETCH_SIZE_KB_per_dispatch"] * 1024 * 2
    if "WRITE_SIZE_KB_per_dispatch" in v:
        v["WRITE_bytes"] = v["WRITE_SIZE_KB_per_dispatch"] * 1024
out["_config"] = {
    "robot": sys.argv[3] if len(sys.argv) > 3 else "spot",
    "samples": int(sys.argv[4]) if len(sys.argv) > 4 else 20000,
    "flags": "EMIT_ALL",
    "command": "python bench.py --no-cpu-baseline --steps 3 --warmup 1 (rocprofv3 --kernel-trace --pmc FETCH_SIZE, "
               "then WRITE_SIZE)",
    "note": "FETCH_bytes_corrected_x2 doubles FETCH_SIZE per MI355X_MICROARCH.md (exact for 16-B/lane streaming "
            "reads; K1's input reads are 8-B gathers, uncalibrated)",
}
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(json.dumps(out, indent=1))
