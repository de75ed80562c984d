import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "zlib.wasm_amd")
for p in (os.path.dirname(os.path.abspath(__file__)), PKG):
    if p not in sys.path:
        sys.path.insert(0, p)
# The host-side tests drive z_stream bookkeeping (deflateSetDictionary's
# Adler-32 before deflateBound, say) on machines without a GPU, where the
# library's own check values fail with Z_MEM_ERROR: this test-only switch makes
# them 0 instead (zgpu_api.cpp ck_internal).  It never affects crc32()/adler32()
# and a GPU run never takes it (a 0 would show up as a parity failure).
os.environ.setdefault("ZGPU_TEST_CHECKSUM_ZERO", "1")


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
