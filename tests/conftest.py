import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(autouse=True)
def _refuse_variant_library(request):
    """GPU tests run the shipped build: a library built with non-default compile-time knobs
    (pd_build_config() != "default", an A/B variant from tools/build_variant_lib.sh) is refused
    unless PRODIFF_ALLOW_VARIANT=1 says the run is an A/B on purpose."""
    if request.node.get_closest_marker("gpu") and os.environ.get("PRODIFF_ALLOW_VARIANT") != "1":
        from prodiff_amd import _lib
        cfg = _lib.lib().pd_build_config().decode()
        if cfg != "default":
            pytest.fail(f"{_lib.LIB_PATH} is a variant build ({cfg}); set PRODIFF_ALLOW_VARIANT=1 for an A/B run")
