"""Copy the judged files of gpu_measure.sh runs from gpurun_out/ (scratch) into profiles/.

    python tools/keep_profiles.py TAG DEST [--note TEXT]     e.g.  r05a profiles/r05/a

A/B runs of tools/kb_ab.sh (no RECIPE.txt of their own: one <variant>.json bench line and its
<variant>.err — the KB_PROF phase lines — per library variant) keep those files as
<step>_<variant>.json / .err; --note records the command that produced them.

Every run directory gpurun_out/TAG_<step>/ (a recipe's steps) — or gpurun_out/TAG/ itself —
contributes <step>_bench.json, <step>_kernel_stats.csv, the FETCH/WRITE and other PMC counter
CSVs, the test / smoke logs and its RECIPE.txt (command, launching commit, library build), so
each profiles/ directory names the recipe and the commit behind every number in it.
"""
import glob
import os
import shutil
import sys

tag, dest = sys.argv[1], sys.argv[2]
note = sys.argv[sys.argv.index("--note") + 1] if "--note" in sys.argv else None
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
runs = sorted(glob.glob(os.path.join(root, "gpurun_out", tag + "_*")))
if os.path.isdir(os.path.join(root, "gpurun_out", tag)):
    runs.append(os.path.join(root, "gpurun_out", tag))
os.makedirs(dest, exist_ok=True)
recipes = []
for r in runs:
    step = os.path.basename(r)[len(tag) + 1:] or "run"
    keep = {
        "bench.json": f"{step}_bench.json",
        "gpu_tests.log": f"{step}_gpu_tests.log",
        "smoke.log": f"{step}_smoke.log",
    }
    for src, dst in keep.items():
        if os.path.exists(os.path.join(r, src)):
            shutil.copy(os.path.join(r, src), os.path.join(dest, dst))
    for f in glob.glob(os.path.join(r, "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(dest, f"{step}_kernel_stats.csv"))
    for f in glob.glob(os.path.join(r, "**", "*counter_collection.csv"), recursive=True):
        shutil.copy(f, os.path.join(dest, f"{step}_{os.path.basename(f)}"))
    if os.path.exists(os.path.join(r, "RECIPE.txt")):
        recipes.append(f"## {step}\n" + open(os.path.join(r, "RECIPE.txt")).read())
    # other bench lines of the run (kb_ab.sh variants, hand-named lines) and their stderr
    for f in sorted(glob.glob(os.path.join(r, "*.json")) + glob.glob(os.path.join(r, "*.err"))):
        if os.path.basename(f) not in ("sources.json", "bench.json"):
            shutil.copy(f, os.path.join(dest, f"{step}_{os.path.basename(f)}"))
with open(os.path.join(dest, "RECIPE.txt"), "w") as fh:
    fh.write(f"# gpurun_out/{tag}_* → {os.path.relpath(dest, root)} (tools/keep_profiles.py)\n\n"
             + (f"note: {note}\n\n" if note else "") + "\n".join(recipes))
print(dest, len(runs), "runs;", len(os.listdir(dest)), "files")
