"""Summarise rocprofv3 --pmc CSVs for one kernel: python tools/pmc_summary.py DIR [kernel-substr]"""
import csv, glob, sys, collections
d = sys.argv[1]; ks = sys.argv[2] if len(sys.argv) > 2 else "riccati"
acc = collections.OrderedDict()
for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if ks in r["Kernel_Name"]:
            acc[r["Counter_Name"]] = float(r["Counter_Value"])
for k, v in acc.items():
    print(f"{k:32s} {v:16.4g}")
