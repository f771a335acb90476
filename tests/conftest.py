import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "gaussian-splatting-npu_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu on the GPU box")


def pytest_sessionfinish(session, exitstatus):
    """The render-parity statistics of this session (flipped pixels, error maxima per check)."""
    import json
    import common
    if common.PARITY_LOG:
        out = os.path.join(ROOT, "gpurun_out")
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "parity_stats.json"), "w") as f:
            json.dump(common.PARITY_LOG, f, indent=1)
