"""HBM traffic per solve from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes →
profiles/traffic_r06.json (the `roofline.traffic` field of bench.py), stamped with what it was
measured on.

    python tools/traffic_json.py KEY RUN_DIR [--kernels SUBSTR] [--solves N] [--out JSON]

RUN_DIR is one `tools/gpu_measure.sh prof` run (gpurun_out/<tag>): its fetch/ and write/ PMC
passes, sources.json (per-file code digests of the tree on the box, the commit it was launched
from, the library's build record) and RECIPE.txt.  Every dispatch whose kernel name contains
SUBSTR (default: every lqrx kernel of the pass) is summed per kernel and divided by SOLVES (the
solves the PMC run made: bench.py --steps 1 --warmup 0 makes 2 — the output-allocating call and
the timed one).  gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes
→ ×2 (calibrated at 0.500 for 4-, 8- and 16-B-per-lane loads, profiles/r04/m); WRITE_SIZE is
exact; both in KiB.

The entry records the measured kernels and the code digests of their translation units and
headers (lqrx._lib.kernel_source_digest, from the run's own sources.json): bench.py reports the
figure only while the tree's code digests of those files still match and the line's kernel is
among the measured ones, and marks it stale otherwise.
"""
import argparse
import csv
import glob
import importlib.util
import json
import os
import re
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_spec = importlib.util.spec_from_file_location("lqrx_lib", os.path.join(ROOT, "lqr.jl_amd", "lqrx", "_lib.py"))
L = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(L)

ap = argparse.ArgumentParser()
ap.add_argument("key")
ap.add_argument("run_dir")
ap.add_argument("--kernels", default="")
ap.add_argument("--solves", type=int, default=2)
ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "traffic_r06.json"))
a = ap.parse_args()


def kname(raw):
    name = raw.replace("void ", "")
    if "namespace)::" in name:
        name = name.split("namespace)::", 1)[1]
    return name.split("(")[0].strip()


def per_kernel(d, counter):
    tot = defaultdict(float)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if a.kernels in r["Kernel_Name"] and r["Counter_Name"] == counter:
                tot[kname(r["Kernel_Name"])] += float(r["Counter_Value"])
    if not tot:
        raise SystemExit(f"no {counter} rows for '{a.kernels}' under {d}")
    return {k: v / a.solves * 1024 for k, v in tot.items()}


fb, wb = per_kernel(os.path.join(a.run_dir, "fetch"), "FETCH_SIZE"), per_kernel(os.path.join(a.run_dir, "write"), "WRITE_SIZE")
kern = {k: {"fetch_x2_bytes": 2 * fb.get(k, 0.0), "write_bytes": wb.get(k, 0.0)} for k in sorted(set(fb) | set(wb))}
prov = json.load(open(os.path.join(a.run_dir, "sources.json")))
units = sorted({u for u in (L.kernel_unit(k, ROOT) for k in kern) if u})
# digests as measured: the run's own per-file digests for every file the kernels' units pull in
files = L.kernel_source_digest(units, ROOT)
if "code_digests" in prov:
    measured = {f: prov["code_digests"].get(f) for f in files}
else:   # a run recorded before code digests (raw SHA-256/16 only): valid while the file is unchanged
    import hashlib
    raw = prov.get("sources", {})
    measured = {}
    for f in files:
        now = hashlib.sha256(open(os.path.join(ROOT, f), "rb").read()).hexdigest()[:16]
        if raw.get(f) != now:
            raise SystemExit(f"{f} changed since {a.run_dir} was measured (no code digest recorded)")
        measured[f] = files[f]
tj = json.load(open(a.out)) if os.path.exists(a.out) else {}
tj[a.key] = {
    "hbm_bytes_per_launch": sum(v["fetch_x2_bytes"] + v["write_bytes"] for v in kern.values()),
    "per_kernel_per_solve": kern,
    "kernels": sorted(kern),
    "sources": measured,
    "solves_in_pmc_run": a.solves,
    "measured_at_head": prov.get("git_head"),
    "library_build_info": prov.get("library_build_info"),
    "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes, every dispatch of the "
              "listed kernels summed per solve; FETCH_SIZE x2 (gfx950 wide-read undercount, MI355X_MICROARCH.md "
              "HBM section; calibrated at 0.500 of the bytes read for 4-, 8- and 16-B-per-lane loads: "
              "profiles/r04/m/kkt_cfg4_sq_and_fetch_calib.txt), KiB->bytes x1024",
    "source": os.path.relpath(a.run_dir, ROOT),
    "recipe": open(os.path.join(a.run_dir, "RECIPE.txt")).readline().strip()
    if os.path.exists(os.path.join(a.run_dir, "RECIPE.txt")) else None,
}
json.dump(tj, open(a.out, "w"), indent=1)
print(a.key, tj[a.key]["hbm_bytes_per_launch"] / 1e9, "GB per solve", "at", prov.get("git_head"))
for k, v in kern.items():
    print(f"  {k[:70]:70s} fetch×2 {v['fetch_x2_bytes'] / 1e9:8.3f} GB  write {v['write_bytes'] / 1e9:7.3f} GB")
