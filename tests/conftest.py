import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "dpdk-tcp-udp_protocol_stack_amd")
for p in (PKG_DIR, os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)

# build the native libraries on first use (no-op when up to date)
if not os.path.exists(os.path.join(PKG_DIR, "librxgpu.so")) or not os.path.exists(
        os.path.join(PKG_DIR, "libnstack.so")):
    subprocess.run(["make", "-C", PKG_DIR, "-j8"], check=True)
if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the gfx950 kernels)")


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return 0
