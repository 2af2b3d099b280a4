"""Timeline of a rocprofv3 --kernel-trace --memory-copy-trace run (dev tool): every call of the host entry point
that starts with host-to-device copies, kernels and copies relative to its first copy.
usage: python tools/trace_timeline.py <trace dir> [calls] [events per call]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
ncalls = int(sys.argv[2]) if len(sys.argv) > 2 else 6
nev = int(sys.argv[3]) if len(sys.argv) > 3 else 24
k = list(csv.DictReader(open(glob.glob(os.path.join(d, "*kernel_trace.csv"))[0])))
m = list(csv.DictReader(open(glob.glob(os.path.join(d, "*memory_copy_trace.csv"))[0])))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:45]) for r in k]
ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C " + r.get("Direction", "").replace("MEMORY_COPY_", "")) for r in m]
ev.sort()
starts = [i for i in range(1, len(ev)) if "HOST_TO_DEVICE" in ev[i][2] and "HOST_TO_DEVICE" not in ev[i - 1][2]]
for st in starts[:ncalls]:
    t0 = ev[st][0]
    print("--- call at event", st)
    for s, e, n in ev[st:st + nev]:
        print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {n}")
