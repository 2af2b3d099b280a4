"""Average per-dispatch PMC values per kernel from rocprofv3 counter_collection CSVs."""
import collections, csv, re, sys
agg = collections.defaultdict(list)
for d in sys.argv[1:]:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        m = re.search(r"::(\w+?)(<\w+>)?\(", r["Kernel_Name"])
        k = (m.group(1) if m else r["Kernel_Name"][:30])
        agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
cur = None
for (k, c), v in sorted(agg.items()):
    if k != cur:
        print(k); cur = k
    print("   %-28s %16.1f  (n=%d)" % (c, sum(v) / len(v), len(v)))
