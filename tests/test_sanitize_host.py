"""CPU: the product library's host-only logic (halo_amd/csrc/host_logic.cc — the code libhalo_rx.so
runs over memory a caller or a ring producer controls: ring header validation, the ring producer,
the small poll's ReadPacket walk, the engine dispatch, the registration registry, the multi-device
split and the host path's chunk planning) built with g++ -fsanitize=address,undefined and fuzzed by
tools/fuzz_host.cc: hostile ring headers (version, fill, size, mask, buffer pointer, head, tail),
hostile length fields, random produce / consume sequences checked byte for byte and frame for
frame against the ring restatement pinned to the reference's own C ring (oracle/halo_ring_oracle.c),
random records through the dispatch, random registry operations against an interval model, and
random frame layouts through the chunk planner. The same source file is compiled into the library
(halo_amd/build.py), so what is fuzzed here is what ships."""
from __future__ import annotations

import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"]


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_logic_fuzz_asan_ubsan(tmp_path):
    inc = [f"-I{os.path.join(ROOT, 'include')}", f"-I{os.path.join(ROOT, 'halo_amd', 'csrc')}"]
    objs = []
    for src, cc, std in (("halo_amd/csrc/host_logic.cc", "g++", "-std=c++17"), ("tools/fuzz_host.cc", "g++", "-std=c++17"),
                         ("oracle/halo_ring_oracle.c", "gcc", "-std=c11"), ("oracle/halo_rx_oracle.c", "gcc", "-std=c11")):
        o = tmp_path / (os.path.basename(src) + ".o")
        subprocess.run([cc, std, *SAN, "-Wall", *inc, "-c", os.path.join(ROOT, src), "-o", str(o)], check=True)
        objs.append(str(o))
    exe = tmp_path / "fuzz_host"
    subprocess.run(["g++", "-fsanitize=address,undefined", *objs, "-o", str(exe)], check=True)
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "verify_asan_link_order=0:detect_leaks=1:" + env.get("ASAN_OPTIONS", "")
    r = subprocess.run([str(exe), "3000", "0x5EED"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    m = re.search(r"ring walk: (\d+) frames.*PARTIAL (\d+) CAPACITY (\d+) MAX (\d+); (\d+) hostile.*?(\d+) direct, (\d+) packed",
                  r.stdout)
    assert m, r.stdout
    frames, partial, capacity, mx, hostile, direct, packed = map(int, m.groups())
    assert frames > 10000 and partial > 0 and capacity > 0 and mx > 0 and hostile > 100 and direct > 0 and packed > 0


def test_library_links_the_fuzzed_source():
    """libhalo_rx.so is built from the same host_logic.cc (halo_amd/build.py SOURCES)."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("halo_build", os.path.join(ROOT, "halo_amd", "build.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert "host_logic.cc" in mod.SOURCES


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_cpu_entry_fuzz_asan_ubsan(tmp_path):
    """The shipped CPU entry point (halo_amd/csrc/rx_cpu.cc, libhalo_rx_cpu.so) under ASan/UBSan
    (tools/fuzz_cpu_entry.cc): the structured fuzz corpus with every frame in a heap block of exactly
    its length, one frame per call and in odd-aligned batches, frames and LoChan packets, flags 0..3,
    every record equal to the oracle's."""
    inc = [f"-I{os.path.join(ROOT, 'include')}", f"-I{os.path.join(ROOT, 'halo_amd', 'csrc')}"]
    objs = []
    for src, cc, std in (("halo_amd/csrc/rx_cpu.cc", "g++", "-std=c++17"), ("tools/fuzz_cpu_entry.cc", "g++", "-std=c++17"),
                         ("oracle/halo_rx_oracle.c", "gcc", "-std=c11"), ("oracle/halo_fuzz.c", "gcc", "-std=c11")):
        o = tmp_path / (os.path.basename(src) + ".o")
        subprocess.run([cc, std, *SAN, "-Wall", *inc, "-c", os.path.join(ROOT, src), "-o", str(o)], check=True)
        objs.append(str(o))
    exe = tmp_path / "fuzz_cpu_entry"
    subprocess.run(["g++", "-fsanitize=address,undefined", *objs, "-lpthread", "-o", str(exe)], check=True)
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "verify_asan_link_order=0:detect_leaks=1:" + env.get("ASAN_OPTIONS", "")
    r = subprocess.run([str(exe), "20000", "0xC9E"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    m = re.search(r"cpu entry: (\d+) records checked.*statuses(.*)", r.stdout)
    assert m, r.stdout
    assert int(m.group(1)) == 2 * 2 * 4 * 20000
    seen = {int(k): int(v) for k, v in (t.split(":") for t in m.group(2).split())}
    assert sum(1 for v in seen.values() if v) >= 12  # every status the corpus reaches, frames and packets
