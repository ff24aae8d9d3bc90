"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel (profiling only).

    python tools/pmc_summary.py gpurun_out/pmc3/*_counter_collection.csv [--kernel conv_body]

Per kernel name: dispatch count, mean duration, and the mean of every counter.  Derived
figures follow /opt/skills/guides/MI355X_MICROARCH.md: effective clock = GRBM_GUI_ACTIVE /
8 XCDs / duration; MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 4
SIMDs * 256 CUs); FETCH_SIZE is in KiB and reports half the bytes of a wide coalesced
streaming read on gfx950 (x2); WRITE_SIZE is exact for 16-B-per-lane stores.
"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--cus", type=int, default=256)
    a = ap.parse_args()
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for f in a.files:
        for r in csv.DictReader(open(f)):
            name = re.sub(r"\(.*", "", r["Kernel_Name"]).split("::")[-1]
            if a.kernel and a.kernel not in name:
                continue
            key = (f, r["Dispatch_Id"])
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[name][key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    for name, ctr in acc.items():
        d = sum(dur[name].values()) / len(dur[name])
        print(f"{name}: dispatches={len(dur[name])} mean_dur={d * 1e3:.4f} ms")
        m = {k: sum(v) / len(v) for k, v in ctr.items()}
        for k in sorted(m):
            print(f"    {k:28s} {m[k]:.4g}")
        if "GRBM_GUI_ACTIVE" in m:
            clk = m["GRBM_GUI_ACTIVE"] / 8 / d
            print(f"    effective clock            {clk / 1e9:.3f} GHz")
            cyc = m["GRBM_GUI_ACTIVE"] / 8
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                print(f"    MFMA busy / (cycles*SIMDs) {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 4 * a.cus):.3f}")
        if "FETCH_SIZE" in m:
            print(f"    HBM read  (KiB x2)         {m['FETCH_SIZE'] * 2 * 1024 / 1e6:.2f} MB")
        if "WRITE_SIZE" in m:
            print(f"    HBM write (KiB)            {m['WRITE_SIZE'] * 1024 / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
