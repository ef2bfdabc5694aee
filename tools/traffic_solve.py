"""Per-SOLVE HBM traffic of a multi-kernel path (e.g. the large-block KKT: Schur + factor +
fused + backward kernels) from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

    python tools/traffic_solve.py KEY KERNEL_SUBSTR SOLVES FETCH_DIR WRITE_DIR [OUT_JSON]

Every dispatch whose name contains KERNEL_SUBSTR is summed, then divided by SOLVES (the number
of solves the PMC run made: bench.py --steps 1 --warmup 0 makes 2 — the output-allocating call
and the timed one).  gfx950 correction as tools/traffic_json.py: FETCH_SIZE x2, KiB -> bytes.
"""
import csv, glob, json, os, sys
from collections import defaultdict

key, ks, solves, fdir, wdir = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4], sys.argv[5]
out = sys.argv[6] if len(sys.argv) > 6 else os.path.join(os.path.dirname(__file__), "..", "profiles", "traffic_r04.json")


def per_kernel(d, counter):
    tot = defaultdict(float)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if ks in r["Kernel_Name"] and r["Counter_Name"] == counter:
                name = r["Kernel_Name"].replace("void ", "")
                if "namespace)::" in name:
                    name = name.split("namespace)::", 1)[1]
                name = name.split("(")[0]
                tot[name] += float(r["Counter_Value"])
    if not tot:
        raise SystemExit(f"no {counter} rows for '{ks}' under {d}")
    return {k: v / solves * 1024 for k, v in tot.items()}


fb, wb = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
kern = {k: {"fetch_x2_bytes": 2 * fb.get(k, 0.0), "write_bytes": wb.get(k, 0.0)} for k in sorted(set(fb) | set(wb))}
tj = json.load(open(out)) if os.path.exists(out) else {}
tj[key] = {
    "hbm_bytes_per_launch": sum(v["fetch_x2_bytes"] + v["write_bytes"] for v in kern.values()),
    "per_kernel_per_solve": kern, "solves_in_pmc_run": solves,
    "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes, every dispatch of "
              f"'{ks}' summed per solve; FETCH_SIZE x2 (gfx950 wide-read undercount, MI355X_MICROARCH.md "
              "HBM section; calibrated at 0.500 of the bytes read for 4-, 8- and 16-B-per-lane coalesced loads: profiles/r04/m/kkt_cfg4_sq_and_fetch_calib.txt), KiB->bytes x1024",
    "source": f"{fdir}, {wdir}",
    "measured_at_head": os.environ.get("GIT_HEAD"),
}
json.dump(tj, open(out, "w"), indent=1)
print(key, tj[key]["hbm_bytes_per_launch"] / 1e9, "GB per solve")
for k, v in kern.items():
    print(f"  {k[:60]:60s} fetch×2 {v['fetch_x2_bytes'] / 1e9:8.2f} GB  write {v['write_bytes'] / 1e9:7.2f} GB")
