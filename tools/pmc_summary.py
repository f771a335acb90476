#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (tools/profile_pmc.sh) per kernel: mean counter value per
dispatch.  Also derives per-launch memory-side traffic:
    traffic_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (gfx950 tallies 128-B read requests as 64 B), and
calibrated for this path's access shapes (profiles/r04_hbm_calib.json, tools/hbm_calib.hip): every
read request of coalesced streams, random 48-B record gathers (into registers or LDS) and random 4-B
gathers is a 128-B request (TCC_EA0_RDREQ_128B = TCC_EA0_RDREQ), so 2 x FETCH_SIZE is the bytes the
memory side reads for all of them; WRITE_SIZE is exact for streams and runs and counts the 32/64-B
sectors of scattered stores.  When a pass collected TCC_EA0_RDREQ_sum and TCC_EA0_RDREQ_128B_sum the
read bytes come from the request sizes directly (128 / 64 / 32 B per request) instead.
Writes <dir>/pmc_traffic.json (kernel -> bytes per launch) and <dir>/pmc_valu.json (kernel -> VALU
wave-instructions per launch, SQ_INSTS_VALU) next to the printed summary."""
import collections
import csv
import glob
import json
import os
import sys

SHORT = {"preprocess_fwd_kernel": "preprocess_fwd", "preprocess_views_kernel": "preprocess_fwd",
         "scan_lookback_kernel": "scan",
         "emit_instances_kernel": "emit_instances", "tile_ranges_kernel": "tile_ranges", "tile_hist_kernel": "tile_ranges",
         "tile_order_kernel": "tile_order", "render_fwd_kernel": "render_fwd", "render_bwd_kernel": "render_bwd",
         "preprocess_bwd_kernel": "preprocess_bwd", "preprocess_bwd_views_kernel": "preprocess_bwd",
         "preprocess_bwd_views_pipe_kernel": "preprocess_bwd",
         # the radix passes carry their sort's name tag (radix.hip): depth sort, tile sort (+ its fused
         # first pass), distCUDA2's cell sort
         "DepthSort": "depth_sort", "TileSort": "tile_sort", "fused_pass1_": "tile_sort", "CellSort": "distCUDA2",
         # SURVEY §8f side paths (bench.py aux leg)
         "knn_": "distCUDA2", "ssim_fwd_kernel": "ssim_fwd", "ssim_bwd_kernel": "ssim_bwd",
         "adam_update_multi_kernel": "sparse_adam"}
# the kernel bench.py --pmc-child launches between its warm-up and its counted steps
MARKER = "spin_kernel"
# operations made of several kernels (several dispatches per call)
MULTI = ("depth_sort", "tile_sort", "distCUDA2")


def short_name(k):
    for key, v in SHORT.items():
        if key in k:
            return v
    return None


def main(d, lib_sha256=None, workload=None, calls=None):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    marked = bool(files)
    for f in files:
        with open(f) as fh:
            rows = list(csv.DictReader(fh))
        # bench.py --pmc-child launches a marker kernel (torch.cuda._sleep: spin_kernel) after its
        # warm-up: only the dispatches after it are counted (the warm-up holds a first call's binning
        # re-run, extra geometry dispatches that no timed step has)
        marks = [int(r["Dispatch_Id"]) for r in rows if MARKER in r.get("Kernel_Name", "") and r.get("Dispatch_Id")]
        first = min(marks) if marks else None
        marked = marked and first is not None
        for row in rows:
            if first is not None and int(row.get("Dispatch_Id") or 0) < first:
                continue
            k = row.get("Kernel_Name", "")
            c = row.get("Counter_Name", "")
            try:
                v = float(row.get("Counter_Value", "nan"))
            except ValueError:
                continue
            acc[k][c].append((row.get("Dispatch_Id", ""), v))
    out = {}
    for k, cs in acc.items():
        if "gsr" not in k and "rocprim" not in k and "hipcub" not in k:
            continue
        ent = {}
        for c, vals in cs.items():
            per = collections.defaultdict(float)
            for did, v in vals:
                per[did] += v
            ent[c] = sum(per.values()) / max(1, len(per))
            ent["dispatches"] = len(per)
        out[k[:120]] = ent
    # Per short name: the counter summed over ALL its dispatches (totals) and the dispatch count.
    # A caller that knows how many times each operation ran (bench.py: launches per step x steps)
    # divides the totals by that; the per-launch figures below assume single-kernel operations run
    # once per dispatch, and for the multi-kernel sorts divide by `calls` when given.
    def totals(counter_fn):
        tot, n = collections.defaultdict(float), collections.defaultdict(int)
        for k, ent in out.items():
            s = short_name(k)
            v = counter_fn(ent)
            if not s or v is None:
                continue
            tot[s] += v * ent["dispatches"]
            n[s] += ent["dispatches"]
        return tot, n

    def per_launch(tot, n):
        res = {}
        for s in tot:
            if s in MULTI:
                if calls and calls.get(s):
                    res[s] = tot[s] / calls[s]
            elif n[s]:
                res[s] = tot[s] / n[s]
        return res

    def read_bytes(e):
        if "TCC_EA0_RDREQ_sum" in e and "TCC_EA0_RDREQ_128B_sum" in e:  # request sizes, when collected
            r32 = e.get("TCC_EA0_RDREQ_32B_sum", 0.0)
            r128 = e["TCC_EA0_RDREQ_128B_sum"]
            return 128.0 * r128 + 32.0 * r32 + 64.0 * (e["TCC_EA0_RDREQ_sum"] - r128 - r32)
        return 2 * e["FETCH_SIZE"] * 1024.0 if "FETCH_SIZE" in e else None

    t_tot, t_n = totals(lambda e: read_bytes(e) + e["WRITE_SIZE"] * 1024.0
                        if read_bytes(e) is not None and "WRITE_SIZE" in e else None)
    traffic = per_launch(t_tot, t_n)
    # stamped with the library AND the workload they were measured on: bench.py uses committed
    # figures only for that build and that workload
    json.dump({"lib_sha256": lib_sha256, "workload": workload,
               "bytes_per_launch": {k: round(v) for k, v in traffic.items()},
               "bytes_total": {k: round(v) for k, v in t_tot.items()}, "dispatches": dict(t_n),
               "marked": marked},
              open(os.path.join(d, "pmc_traffic.json"), "w"), indent=1)
    # VALU wave-instructions per launch (bench.py's secondary, VALU-issue roofline)
    v_tot, v_n = totals(lambda e: e.get("SQ_INSTS_VALU"))
    valu = per_launch(v_tot, v_n)
    json.dump({"lib_sha256": lib_sha256, "workload": workload,
               "winst_per_launch": {k: round(v) for k, v in valu.items()},
               "winst_total": {k: round(v) for k, v in v_tot.items()}, "dispatches": dict(v_n),
               "marked": marked},
              open(os.path.join(d, "pmc_valu.json"), "w"), indent=1)
    print(json.dumps({"kernels": out, "traffic_bytes_per_launch": {k: round(v) for k, v in traffic.items()},
                      "marked": marked},
                     indent=1))


def lib_sha256(path=None):
    import hashlib
    path = path or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gaussian-splatting-npu_amd", "diff_gaussian_rasterization", "libgsr_hip.so")
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


if __name__ == "__main__":
    main(sys.argv[1], lib_sha256())
