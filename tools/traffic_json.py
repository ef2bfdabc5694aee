"""Per-launch HBM traffic of one kernel from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
passes → profiles/traffic_r01.json (the `roofline.traffic` field of bench.py).

    python tools/traffic_json.py KEY KERNEL_SUBSTR FETCH_DIR WRITE_DIR [OUT_JSON]

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of wide
coalesced reads → ×2; WRITE_SIZE is exact for 16-B/lane streaming stores; both in KiB.
"""
import csv, glob, json, os, sys

key, ks, fdir, wdir = sys.argv[1:5]
out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(os.path.dirname(__file__), "..", "profiles", "traffic_r03.json")


def per_dispatch(d, counter):
    vals = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if ks in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals[r.get("Dispatch_Id", len(vals))] = vals.get(r.get("Dispatch_Id", len(vals)), 0.0) + float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for '{ks}' under {d}")
    return sum(vals.values()) / len(vals), len(vals)


fkib, nf = per_dispatch(fdir, "FETCH_SIZE")
wkib, nw = per_dispatch(wdir, "WRITE_SIZE")
tj = json.load(open(out)) if os.path.exists(out) else {}
tj[key] = {
    "hbm_bytes_per_launch": fkib * 1024 * 2 + wkib * 1024,
    "fetch_size_kib": fkib, "write_size_kib": wkib, "dispatches_averaged": min(nf, nw),
    "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes "
              f"({ks} rows only); FETCH_SIZE x2 (gfx950 wide-read undercount, "
              "MI355X_MICROARCH.md HBM section), KiB->bytes x1024",
    "source": f"{fdir}, {wdir}",
    "measured_at_head": os.environ.get("GIT_HEAD"),
}
json.dump(tj, open(out, "w"), indent=1)
print(key, tj[key]["hbm_bytes_per_launch"] / 1e9, "GB/launch")
