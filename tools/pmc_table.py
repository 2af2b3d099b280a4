"""Average per-dispatch PMC values per kernel from rocprofv3 counter_collection CSVs (dev tool).
usage: python tools/pmc_table.py <pass dir> [<pass dir> ...]   (each holding run_counter_collection.csv)"""
import collections, csv, sys
agg = collections.defaultdict(list)
for d in sys.argv[1:]:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        name = r["Kernel_Name"]
        k = name.split("(")[0].split("<")[0].replace("void ", "").split("::")[-1]
        agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
cur = None
for (k, c), v in sorted(agg.items()):
    if k != cur:
        print(k); cur = k
    print("   %-28s %16.1f  (n=%d)" % (c, sum(v) / len(v), len(v)))
