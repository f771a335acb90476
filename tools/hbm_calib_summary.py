#!/usr/bin/env python3
"""HBM-counter calibration summary (tools/hbm_calib.sh): per calibration kernel, the counters
per dispatch against the bytes the access is known to move -- the algorithmic bytes and the
distinct 32 / 64 / 128-B units it touches (tools/hbm_calib.hip) -- as ratios.  The factors
tools/pmc_summary.py applies per access pattern come from this table (profiles/r04_hbm_calib.json)."""
import collections
import csv
import glob
import json
import os
import sys


def counters(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            try:
                acc[row["Kernel_Name"]][row["Counter_Name"]] += float(row["Counter_Value"])
            except (KeyError, ValueError):
                pass
    return acc


def main(d):
    known = [json.loads(ln) for ln in open(os.path.join(d, "calib.jsonl")) if ln.startswith("{")]
    acc = counters(d)
    out = []
    for k in known:
        name = k["kernel"]
        c = next((v for kn, v in acc.items() if kn.split("(")[0].split("<")[0].strip().endswith(name)), {})
        ent = dict(k)
        ent.update({n: c.get(n) for n in sorted(c)})
        if c.get("FETCH_SIZE") is not None:
            ent["fetch_bytes"] = c["FETCH_SIZE"] * 1024.0
        if c.get("WRITE_SIZE") is not None:
            ent["write_bytes"] = c["WRITE_SIZE"] * 1024.0
        rd = c.get("TCC_EA0_RDREQ_sum")
        if rd is not None:
            r32 = c.get("TCC_EA0_RDREQ_32B_sum", 0.0)
            r128 = c.get("TCC_EA0_RDREQ_128B_sum")
            ent["rdreq_64B_model_bytes"] = 32 * r32 + 64 * (rd - r32)
            if r128 is not None:
                ent["rdreq_128B_model_bytes"] = 32 * r32 + 128 * r128 + 64 * (rd - r32 - r128)
        wr = c.get("TCC_EA0_WRREQ_sum")
        if wr is not None:
            w64 = c.get("TCC_EA0_WRREQ_64B_sum", 0.0)
            ent["wrreq_model_bytes"] = 64 * w64 + 32 * (wr - w64)
        b = ent.get("fetch_bytes") if k["dir"] == "read" else ent.get("write_bytes")
        if b:
            for key in ("algorithmic_bytes", "touched_32B", "touched_64B", "touched_128B"):
                ent["counter_over_" + key] = round(b / k[key], 4)
        out.append(ent)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
