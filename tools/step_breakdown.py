"""Per-step kernel-time breakdown of a rocprofv3 trace of bench.py (run_results.db): the average
duration per step of each kernel family over the last steps.  Usage: python tools/step_breakdown.py DB"""
import collections
import sqlite3
import sys


def families(name):
    for key, fam in (("preprocess_fwd", "preprocess_fwd"), ("DepthSort", "depth_sort"), ("scan_lookback", "scans"),
                     ("fused_pass1", "tile_sort"), ("TileSort", "tile_sort"), ("tile_hist", "tile_hist"),
                     ("tile_order", "tile_order"), ("render_fwd", "render_fwd"), ("render_bwd", "render_bwd"),
                     ("preprocess_bwd", "preprocess_bwd")):
        if key in name:
            return fam
    return "other"


STEP_MARK = ("preprocess_fwd_kernel", "ELi8E")  # the 8-view batch's preprocess starts a step


def main(db):
    c = sqlite3.connect(db)
    scols = [r[1] for r in c.execute("pragma table_info(rocpd_info_kernel_symbol)")]
    name_col = "kernel_name" if "kernel_name" in scols else "display_name"
    rows = list(c.execute(f"select d.start, d.end, s.{name_col} from rocpd_kernel_dispatch d join "
                          f"rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start"))
    starts = [i for i, r in enumerate(rows) if STEP_MARK[0] in r[2] and STEP_MARK[1] in r[2]]
    steps = list(zip(starts[-6:-1], starts[-5:]))
    acc = collections.defaultdict(float)
    total = 0.0
    for a, b in steps:
        total += rows[b][0] - rows[a][0]
        for s, e, n in rows[a:b]:
            acc[families(n)] += e - s
    n = len(steps)
    print(f"step {total / n / 1e3:.1f} us (mean of {n})")
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        print(f"  {k:16s} {v / n / 1e3:8.1f} us")




def timeline(db, which=-3):
    """One step's dispatches: start offset, duration, name."""
    c = sqlite3.connect(db)
    rows = list(c.execute("select d.start, d.end, s.kernel_name from rocpd_kernel_dispatch d join "
                          "rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start"))
    starts = [i for i, r in enumerate(rows) if STEP_MARK[0] in r[2] and STEP_MARK[1] in r[2]]
    a, b = starts[which], starts[which + 1]
    t0 = rows[a][0]
    for s, e, n in rows[a:b]:
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {n[5:90]}")


if __name__ == "__main__":
    if "--single" in sys.argv:  # the single-view step: preprocess_fwd_kernel<true, 1>
        sys.argv.remove("--single")
        STEP_MARK = ("preprocess_fwd_kernel", "ELi1E")
    main(sys.argv[1])
    if len(sys.argv) > 2:
        timeline(sys.argv[1])
