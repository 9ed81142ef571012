"""Shared fixtures.  `-m "not gpu"` tests need no GPU; `-m gpu` tests run the
HIP path (libokv_sst.so) on a real MI355X and compare it with the oracle."""
from __future__ import annotations

import base64
import json
import os
import subprocess
import sys
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden", "golden.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    # build the checker (oracle) and the product library if they are missing
    if not os.path.exists(os.path.join(ROOT, "oracle", "build", "liboref.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    if not os.path.exists(os.path.join(ROOT, "objectkv_amd", "libokv_sst.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "objectkv_amd", "csrc")],
                       check=True)


def unpack(s: str) -> bytes:
    return zlib.decompress(base64.b64decode(s))


def rowval(b):
    """Same encoding as tests/golden/make_golden.py."""
    import hashlib
    if b is None:
        return None
    b = bytes(b)
    return b.hex() if len(b) <= 64 else f"sha256:{hashlib.sha256(b).hexdigest()}:{len(b)}"


@pytest.fixture(scope="session")
def golden():
    with open(GOLDEN) as f:
        d = json.load(f)
    return {c["name"]: c for c in d["cases"]}


@pytest.fixture(scope="session")
def decoder():
    import objectkv_amd as okv
    dec = okv.Decoder(0)
    yield dec
    dec.close()


def descs_of(case):
    return np.array([b["desc"] for b in case["blocks"]], np.uint64).reshape(-1, 4)
