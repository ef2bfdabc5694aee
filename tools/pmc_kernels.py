"""Per-kernel SQ counter summary of rocprofv3 --pmc CSVs (per dispatch and per unit).

    python tools/pmc_kernels.py UNITS CSV [CSV ...]

UNITS: the work units one dispatch processes (e.g. trajectories x knots) — counters are also
printed divided by it.  Kernel names are shortened to the template name."""
import csv, collections, sys

units = float(sys.argv[1])
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in sys.argv[2:]:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "")
        if "namespace)::" in k:
            k = k.split("namespace)::", 1)[1]
        k = k.split("(")[0]
        agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
for (k, c), v in sorted(agg.items()):
    per = v / len(disp[k])
    print(f"{k[:44]:44s} {c:28s} {per:12.4g} per dispatch  {per / units:10.1f} per unit")
