"""Drop-in for the reference's `simple_knn` extension (un-vendored submodule simple-knn,
imported by scene/gaussian_model.py:21 as `from simple_knn._C import distCUDA2`).

The compute runs in libgsr_hip.so (include/simple_knn.h, csrc/knn.hip); there is no CPU path.
"""
from . import _C  # noqa: F401
