"""Per-launch HBM traffic of the bench's kernels from rocprofv3 PMC passes (profiling only).

    python tools/traffic_from_pmc.py profiles/r01/bench/pmc_fetch.csv profiles/r01/bench/pmc_write.csv \
        --out profiles/r01/bench/traffic.json

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE reports half the bytes
of a coalesced streaming read at every access width the kernels use: MI355X_MICROARCH.md gives
it for 16 B per lane, and the round-4 calibration probe (tools/probes/fetch_probe.hip over a
2 GiB buffer, 8x the Infinity Cache; profiles/r04/probe/) measured exactly 1/2 for 4, 8 and
16 B per lane alike, and WRITE_SIZE exact for 4- and 16-B stores.  So every kernel's
FETCH_SIZE is doubled (round 3 took the 4-B/lane prox passes as reported and read K2's
0.51 GB as "half of its reads from the MALL": it is all of them from the fabric).  bench.py
puts the conv_body entry in its roofline ``traffic`` field.
"""
import argparse
import collections
import csv
import json
import re

FETCH_CORRECTION = 2.0   # every access width (profiles/r04/probe/fetch_probe_summary.txt)


def short(name):
    n = re.sub(r"\(.*", "", name)
    mode = re.search(r"conv_body_x8_kernelILi\dELi(\d)E", name)
    if mode and mode.group(1) in "12":                                      # head + L0 / L(n-1) + tail
        return "conv_body_f2h" if mode.group(1) == "1" else "conv_body_f2t"
    if any(k in n for k in ("conv_body_x8", "conv_body_f8", "conv_body_f2")):   # the two-layer launch (bench scope "conv_body_f2")
        return "conv_body_f2"
    if "conv_s3_kernel" in n:                                               # split fp16: body (MODE 0) / tail
        return "conv_tail_s3" if "ILi1E" in n else "conv_body_s3"
    if "conv_stack" in n:
        return "conv_stack"
    for k in ("conv_body_f2", "conv_body", "conv_head", "conv_tail", "k1", "k2", "k3_l2_dual", "l1_", "ssim"):
        if k in n:
            return k
    return None


def per_dispatch(path, counter):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if k and r["Counter_Name"] == counter:
            vals[k].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    rd = per_dispatch(a.fetch_csv, "FETCH_SIZE")
    wr = per_dispatch(a.write_csv, "WRITE_SIZE")
    out = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ({a.fetch_csv}, {a.write_csv})",
           "kernels": {}}
    for k in sorted(set(rd) | set(wr)):
        r = rd.get(k, 0.0) * FETCH_CORRECTION
        out["kernels"][k] = {"read_bytes": round(r), "write_bytes": round(wr.get(k, 0.0)),
                             "bytes": round(r + wr.get(k, 0.0)), "fetch_correction": FETCH_CORRECTION}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
