"""Per-kernel average durations from rocprofv3 sqlite output (run_results.db): python tools/kstats_db.py DB [filter]"""
import sqlite3
import sys


def stats(db, filt=("radix", "fused_pass1", "scan_lookback", "tile_hist", "tile_order", "preprocess", "render")):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(rocpd_kernel_dispatch)")]
    scols = [r[1] for r in c.execute("pragma table_info(rocpd_info_kernel_symbol)")]
    name_col = "kernel_name" if "kernel_name" in scols else ("display_name" if "display_name" in scols else scols[-1])
    q = (f"select s.{name_col}, count(*), avg(d.end - d.start) from rocpd_kernel_dispatch d "
         f"join rocpd_info_kernel_symbol s on d.kernel_id = s.id group by s.{name_col}")
    out = []
    for name, n, avg in c.execute(q):
        if any(k in name for k in filt):
            out.append((name, n, avg / 1e3))
    return sorted(out, key=lambda r: -r[1] * r[2])


if __name__ == "__main__":
    for name, n, us in stats(sys.argv[1]):
        print(f"{us:9.1f} us x{n:4d}  {name[:120]}")
