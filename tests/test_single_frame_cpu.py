"""CPU: the single-frame Parse* wrappers with SINGLE_FRAME_CPU set (halo_amd.protocol, the CPU entry
point instead of a GPU round trip; go/gpurx SingleFrameCPU) return exactly the reference functions'
tuples, error strings included: the same checks as tests/test_gpu_single_frame.py — every golden
frame, every IPv4 payload and L4 segment in it through all three L4 parsers, length edges and random
corruptions, CheckSumEnable on and off, against oracle/ref_py.py — with no device."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from tests.test_gpu_single_frame import test_parse_eth_and_ipv4, test_parse_l4  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def frames():
    g = os.path.join(ROOT, "tests", "golden")
    meta = json.load(open(os.path.join(g, "frames.json")))
    blob = np.fromfile(os.path.join(g, "frames.bin"), dtype=np.uint8)
    return [blob[e["offset"]:e["offset"] + e["len"]].tobytes() for e in meta["frames"]]


@pytest.fixture(autouse=True)
def on_cpu():
    from halo_amd import protocol

    old = protocol.SINGLE_FRAME_CPU
    protocol.SINGLE_FRAME_CPU = True
    yield
    protocol.SINGLE_FRAME_CPU = old
    assert not protocol._ctx  # no host context (so no GPU) was made


@pytest.fixture(params=[True, False], ids=["csum", "nocsum"])
def csum(request):
    from halo_amd import protocol

    old = protocol.CheckSumEnable
    protocol.CheckSumEnable = request.param
    yield request.param
    protocol.CheckSumEnable = old
