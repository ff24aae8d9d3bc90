"""Summarise tools/pmc_variants.sh output: per variant, conv_body counters per launch."""
import csv, glob, sys, collections
for d in sorted(glob.glob("gpurun_out/pmcv*")):
    agg = collections.defaultdict(float); n = collections.Counter()
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "conv_body" not in r["Kernel_Name"]: continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    if not agg: continue
    g = agg["GRBM_GUI_ACTIVE"] / max(1, n["GRBM_GUI_ACTIVE"])
    out = {k: agg[k] / max(1, n[k]) for k in agg}
    print(d, {k: f"{v:.4g}" for k, v in sorted(out.items())})
    if "SQ_VALU_MFMA_BUSY_CYCLES" in out and "SQ_BUSY_CYCLES" in out:
        print("   mfma busy / (busy cycles*4 SIMD... raw ratio)", out["SQ_VALU_MFMA_BUSY_CYCLES"] / out["SQ_BUSY_CYCLES"])
