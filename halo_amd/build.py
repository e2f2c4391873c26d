"""Build libhalo_rx.so (hipcc, gfx950) in-tree: ``python halo_amd/build.py [--force]``.

Standalone on purpose: importing the halo_amd package requires the library this builds.
"""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "halo_amd", "csrc")
OUT = os.path.join(ROOT, "halo_amd", "lib", "libhalo_rx.so")
SOURCES = ["rx_parse.hip", "tx_fixup.hip", "tx_build.hip", "deep_nat.hip", "flow_hash.hip", "route_lpm.hip", "synth.hip", "host_path.hip",
           "ring_rx.hip", "resident.hip", "host_logic.cc"]
# measurement tooling (bench.py's native step loop), linked against the product library
BENCH_SRC = os.path.join(ROOT, "tools", "bench_loop.hip")
BENCH_OUT = os.path.join(ROOT, "tools", "libhalo_bench.so")
# the CPU entry point of SURVEY §8b (include/halo_rx_cpu.h): host code only, its own library
CPU_SRC = os.path.join(CSRC, "rx_cpu.cc")
CPU_OUT = os.path.join(ROOT, "halo_amd", "lib", "libhalo_rx_cpu.so")
HEADERS = ["halo_common.h", "halo_limits.h", "host_logic.h", "device_util.h", os.path.join("..", "..", "include", "halo_rx.h")]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    return "hipcc"


def build(force: bool = False, verbose: bool = False) -> str:
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    deps = srcs + [os.path.join(CSRC, h) for h in HEADERS]
    if not force and os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps):
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    obj_dir = os.path.join(ROOT, "build", "obj")
    os.makedirs(obj_dir, exist_ok=True)
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall",
             "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]
    headers_mtime = max(os.path.getmtime(os.path.join(CSRC, h)) for h in HEADERS)

    def compile_one(src: str) -> str:
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), headers_mtime):
            cmd = [_hipcc(), *flags, "-c", src, "-o", obj + ".tmp"]
            if verbose:
                print(" ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)
            os.replace(obj + ".tmp", obj)
        return obj

    from concurrent.futures import ThreadPoolExecutor

    jobs = max(1, min(len(srcs), int(os.environ.get("MAX_JOBS") or os.cpu_count() or 1), 8))
    with ThreadPoolExecutor(jobs) as ex:  # one hipcc per source file, then one link
        objs = list(ex.map(compile_one, srcs))
    cmd = [_hipcc(), "--offload-arch=gfx950", "-fPIC", "-shared", *objs, "-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


def build_cpu(force: bool = False, verbose: bool = False) -> str:
    """halo_amd/lib/libhalo_rx_cpu.so (g++): halo_rx_parse_batch_cpu. No HIP, no link to libhalo_rx."""
    deps = [CPU_SRC, os.path.join(CSRC, "halo_limits.h"), os.path.join(ROOT, "include", "halo_rx.h"),
            os.path.join(ROOT, "include", "halo_rx_cpu.h")]
    if not force and os.path.exists(CPU_OUT) and os.path.getmtime(CPU_OUT) >= max(map(os.path.getmtime, deps)):
        return CPU_OUT
    os.makedirs(os.path.dirname(CPU_OUT), exist_ok=True)
    cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", "-Wall", "-Wextra",
           "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, CPU_SRC, "-o", CPU_OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(CPU_OUT + ".tmp", CPU_OUT)
    return CPU_OUT


def build_bench(force: bool = False, verbose: bool = False) -> str:
    """tools/libhalo_bench.so: the native timed step loop used by bench.py."""
    lib = build(force=False, verbose=verbose)
    if not force and os.path.exists(BENCH_OUT) and os.path.getmtime(BENCH_OUT) >= max(
            os.path.getmtime(BENCH_SRC), os.path.getmtime(lib)):
        return BENCH_OUT
    cmd = [_hipcc(), "--offload-arch=gfx950", "-O2", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden",
           "-I" + os.path.join(ROOT, "include"), BENCH_SRC,
           # the XXH3 line's load-pattern probe: flow_hash.hip's run kernel without the hashing
           os.path.join(CSRC, "flow_hash.hip"), "-DHALO_XXH3_PROBE=1", "-DHALO_XXH3_PROBE_ENTRY=1",
           "-I" + CSRC, "-L" + os.path.dirname(OUT), "-lhalo_rx",
           "-Wl,-rpath,$ORIGIN/../halo_amd/lib", "-o", BENCH_OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(BENCH_OUT + ".tmp", BENCH_OUT)
    return BENCH_OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_cpu(force="--force" in sys.argv, verbose=True))
    print(build_bench(force="--force" in sys.argv, verbose=True))
