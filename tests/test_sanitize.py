"""CPU: the C oracle under AddressSanitizer + UBSan over fuzzed, mutated and truncated frames,
each in an exact-size heap block (any read past a frame's end aborts). The reference panics on
some malformed inputs (protocol/ipv4.go:84); the restatement must classify them instead."""
from __future__ import annotations

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_oracle_fuzz_asan_ubsan(tmp_path):
    exe = tmp_path / "fuzz_oracle"
    subprocess.run(["gcc", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-fno-sanitize-recover=all", os.path.join(ROOT, "tools", "fuzz_oracle.c"),
                    os.path.join(ROOT, "oracle", "halo_rx_oracle.c"), "-o", str(exe), "-pthread"], check=True)
    env = dict(os.environ)
    # tolerate other preloaded libraries in the environment: ASan's link-order check is advisory
    env["ASAN_OPTIONS"] = "verify_asan_link_order=0:" + env.get("ASAN_OPTIONS", "")
    r = subprocess.run([str(exe), "30000"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "fuzzed 30000 frames" in r.stdout
