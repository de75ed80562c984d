import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "zlib.wasm_amd")
for p in (os.path.dirname(os.path.abspath(__file__)), PKG):
    if p not in sys.path:
        sys.path.insert(0, p)
# The host-side tests drive z_stream calls (deflateSetDictionary's Adler-32,
# say) on machines without a GPU, where a checksum call would end the process
# by default (zgpu_api.cpp checksum_one): have it return 0 instead.  On a GPU a
# checksum never fails, and a 0 would show up as a parity failure anyway.
os.environ.setdefault("ZGPU_CHECKSUM_ERROR", "zero")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    from zhelpers import Oracle, build_oracle
    build_oracle()
    return Oracle()


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def zg():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import zgpu
    zgpu.load()
    assert zgpu.load().zgpu_init() == 0, "libzgpu could not initialise the GPU"
    return zgpu
