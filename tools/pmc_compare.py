"""Per-kernel before/after of two pmc_summary.py outputs (per dispatch), written into the newer one
as "vs_previous": the counters VERDICT asks to track (waits, LDS bank conflicts, write requests,
HBM bytes, SALU/VALU).  Usage: pmc_compare.py OLD.json NEW.json OUT.json OLD_TAG NEW_TAG"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short_name  # noqa: E402

KEYS = ["SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS", "TCC_EA0_WRREQ_sum",
        "TCC_EA0_WRREQ_64B_sum", "TCC_EA0_RDREQ_sum", "FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_SALU", "SQ_INSTS_VALU",
        "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE"]


def main(old, new, out, old_tag, new_tag):
    a, b = json.load(open(old)), json.load(open(new))
    cmp = {}
    for name, kb in b["kernels"].items():
        ka = a["kernels"].get(name)
        if ka is None:  # a kernel renamed between the rounds: the same operation and first template argument
            targ = re.search(r"<(\d+)", name)
            cand = [k for k in a["kernels"] if short_name(k) == short_name(name) and short_name(k) is not None and
                    (targ is None or re.search(r"<(\d+)", k) and re.search(r"<(\d+)", k).group(1) == targ.group(1))]
            if len(cand) == 1:
                ka = a["kernels"][cand[0]]
                cmp.setdefault("_renamed", {})[name] = cand[0]
        pb = {c: kb[c] for c in KEYS if c in kb}
        row = {new_tag: pb, "dispatches": {new_tag: kb.get("dispatches")}}
        if ka is not None:
            pa = {c: ka[c] for c in KEYS if c in ka}
            row[old_tag] = pa
            row["dispatches"][old_tag] = ka.get("dispatches")
            row["ratio"] = {c: round(pb[c] / pa[c], 4) for c in pb if pa.get(c)}
        for tag, p in ((new_tag, pb), (old_tag, row.get(old_tag))):
            if p and p.get("SQ_INSTS_VALU"):
                row.setdefault("salu_per_valu", {})[tag] = round(p["SQ_INSTS_SALU"] / p["SQ_INSTS_VALU"], 4)
        cmp[name] = row
    b["vs_previous"] = {"note": f"counters summed over the timed step's launches of each kernel ({old_tag} -> "
                                f"{new_tag}); ratio = {new_tag}/{old_tag}; FETCH/WRITE_SIZE in KiB as "
                                "pmc_summary.py reports them", "kernels": cmp}
    json.dump(b, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:6])
