"""CPU-side checks of the C-ABI boundary (no GPU needed, no compute calls).

* libgsr_hip.so loads and exports every function include/gsr.h declares;
* the host-only entry points (buffer sizes, layouts, version, error string) behave as the
  reference's GeometryState/ImageState/BinningState::required + obtain do
  (rasterizer_impl.h:21-73, rasterizer_impl.cu:155-194): every chunk 128-byte aligned,
  in bounds, and sizes monotone in P / pixels / L;
* the Python surface exposes the reference's names (diff_gaussian_rasterization/__init__.py:143-207)
  plus the accelerated upstream's SparseGaussianAdam, which train.py may only find together with
  the `dc=` argument of GaussianRasterizer.forward.
"""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("gsr.h", "simple_knn.h", "fused_ssim.h")]
LIB = os.path.join(ROOT, "gaussian-splatting-npu_amd", "diff_gaussian_rasterization", "libgsr_hip.so")


def _declared():
    text = "\n".join(open(h).read() for h in HEADERS)
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(gsr_[a-z_0-9]+)\s*\(", text, flags=re.M)
    return sorted(set(names))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} missing: run __graft_entry__.build() (make -C gaussian-splatting-npu_amd)")
    lib = ctypes.CDLL(LIB)
    lib.gsr_version.restype = ctypes.c_char_p
    lib.gsr_last_error.restype = ctypes.c_char_p
    for f in ("gsr_geometry_buffer_size", "gsr_image_buffer_size", "gsr_binning_buffer_size"):
        getattr(lib, f).restype = ctypes.c_size_t
    return lib


def test_header_declares_the_boundary():
    names = _declared()
    for must in ["gsr_forward", "gsr_backward", "gsr_mark_visible", "gsr_last_error", "gsr_geometry_buffer_size",
                 "gsr_image_buffer_size", "gsr_binning_buffer_size", "gsr_knn_dist2", "gsr_knn_workspace_size", "gsr_ssim_forward",
                 "gsr_ssim_backward", "gsr_forward_dc", "gsr_forward_geometry_dc", "gsr_forward_prealloc_dc",
                 "gsr_backward_dc", "gsr_adam_update"]:
        assert must in names, must


def test_library_exports_every_declared_symbol(lib):
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, f"declared in include/*.h but not exported: {missing}"


def test_version_and_error_string(lib):
    assert lib.gsr_version().decode()
    assert isinstance(lib.gsr_last_error(), bytes)


def test_prefix_stream_modes(lib):
    """gsr_set_prefix_stream takes 0 (caller's stream), 1 (prefix stream + auxiliary stream) and 2
    (prefix on the caller's stream, side work on the auxiliary one); anything else is refused
    (no GPU is touched: the mode is host state)."""
    for mode in (0, 2, 1):
        assert lib.gsr_set_prefix_stream(mode) == 0
    for bad in (-1, 3):
        assert lib.gsr_set_prefix_stream(bad) != 0
        assert b"prefix stream mode" in lib.gsr_last_error()
    assert lib.gsr_set_prefix_stream(1) == 0


def _layout(fn, *args, n=64):
    off = (ctypes.c_size_t * n)()
    k = fn(*args, off, n)
    assert 0 < k <= n
    return [off[i] for i in range(k)]


@pytest.mark.parametrize("P", [1, 7, 1000, 1_000_000, 6_000_000])
def test_geometry_layout_aligned_and_in_bounds(lib, P):
    total = lib.gsr_geometry_buffer_size(P)
    offs = _layout(lib.gsr_geometry_layout, P)
    assert all(o % 128 == 0 for o in offs)
    assert offs == sorted(offs) and offs[-1] <= total
    # at least the reference's per-Gaussian state (rasterizer_impl.cu:155-170)
    assert total >= P * (4 + 4 + 12 + 8 + 24 + 16 + 12 + 4 + 4)


@pytest.mark.parametrize("W,H", [(1, 1), (256, 256), (1920, 1080), (4096, 2160)])
def test_image_layout(lib, W, H):
    total = lib.gsr_image_buffer_size(W, H)
    offs = _layout(lib.gsr_image_layout, W, H)
    assert all(o % 128 == 0 for o in offs) and offs[-1] <= total
    assert total >= W * H * 8


@pytest.mark.parametrize("L", [1, 1878, 5_813_426, 60_000_000])
def test_binning_layout(lib, L):
    total = lib.gsr_binning_buffer_size(L)
    offs = _layout(lib.gsr_binning_layout, L)
    assert all(o % 128 == 0 for o in offs) and offs[-1] <= total
    assert total >= L * (4 + 48)  # point list + per-instance gradient record


def test_sizes_monotone(lib):
    g = [lib.gsr_geometry_buffer_size(p) for p in (1, 10, 1000, 100000)]
    b = [lib.gsr_binning_buffer_size(p) for p in (1, 10, 1000, 100000)]
    assert g == sorted(g) and b == sorted(b)


def test_python_surface():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-npu_amd"))
    import diff_gaussian_rasterization as dgr
    for name in ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "_RasterizeGaussians"]:
        assert hasattr(dgr, name), name
    # SparseGaussianAdam makes train.py pass dc= (train.py:37-41 -> gaussian_renderer/__init__.py:90-100)
    import inspect
    assert issubclass(dgr.SparseGaussianAdam, __import__("torch").optim.Adam)
    assert "dc" in inspect.signature(dgr.GaussianRasterizer.forward).parameters
    # the reference's step(visibility, N); `rows` (a Gaussian range, for the pipelined data-parallel
    # step) is an optional extra
    params = inspect.signature(dgr.SparseGaussianAdam.step).parameters
    assert list(params)[:3] == ["self", "visibility", "N"]
    assert all(p.default is not inspect.Parameter.empty for p in list(params.values())[3:])
    assert dgr.GaussianRasterizationSettings._fields == (
        "image_height", "image_width", "tanfovx", "tanfovy", "bg", "scale_modifier", "viewmatrix", "projmatrix",
        "sh_degree", "campos", "prefiltered", "debug", "antialiasing")
    for name in ["rasterize_gaussians", "rasterize_gaussians_backward", "mark_visible", "adamUpdate"]:
        assert callable(getattr(dgr._C, name)), name
