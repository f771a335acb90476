"""The measurement tooling's kernel-name accounting (CPU only).

bench.py's in-run PMC passes and tools/pmc_summary.py credit each dispatch to a step stage by its
kernel name (SHORT).  A kernel renamed or added without an entry would silently drop out of the
traffic and VALU figures of the bench line (round 6: the two-chunk preprocess_bwd kernel did until
it got one), so every __global__ kernel of the library must map to a stage -- the radix passes by
the sort tag in their template arguments -- except the debug and API-completeness kernels below.
"""
import glob
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from pmc_summary import short_name  # noqa: E402

NOT_STAGES = {"debug_keys_kernel", "debug_keys_from_ranges_kernel", "mark_visible_kernel"}
RADIX = {"radix_colscan_kernel", "radix_count_kernel", "radix_rowscan_kernel", "radix_rowscan_lds_kernel",
         "radix_scatter_kernel"}


def _kernels():
    names = set()
    for f in glob.glob(os.path.join(ROOT, "gaussian-splatting-npu_amd", "csrc", "*.hip")):
        src = open(f).read()
        for m in re.finditer(r"__global__", src):
            k = re.search(r"\b(\w+_kernel)\s*\(", src[m.end():m.end() + 400])
            if k:
                names.add(k.group(1))
    return names


def test_every_kernel_maps_to_a_stage():
    names = _kernels()
    assert {"render_fwd_kernel", "render_bwd_kernel", "preprocess_bwd_views_pipe_kernel"} <= names
    for n in sorted(names - NOT_STAGES - RADIX):
        assert short_name(f"void gsr::{n}<8, 2>(gsr::Args)") is not None, n
    for n in sorted(RADIX & names):
        for tag, stage in (("DepthSort", "depth_sort"), ("TileSort", "tile_sort"), ("CellSort", "distCUDA2")):
            assert short_name(f"void gsr::{n}<8, true, gsr::{tag}, 9, 512>(gsr::Args)") == stage, (n, tag)


def test_stage_names_of_the_bench_kernels():
    assert short_name("void gsr::preprocess_bwd_views_pipe_kernel<8, 2>(gsr::PreprocessBwdViewsArgs, int)") == \
        "preprocess_bwd"
    assert short_name("void gsr::preprocess_bwd_views_kernel<1, true>(gsr::PreprocessBwdViewsArgs)") == \
        "preprocess_bwd"
    assert short_name("gsr::render_fwd_kernel(gsr::ViewBatch<gsr::RenderFwdArgs>)") == "render_fwd"
    assert short_name("void gsr::fused_pass1_scatter_kernel<8, 6>(gsr::ViewBatch<gsr::FusedPassArgs>, unsigned int)") \
        == "tile_sort"
