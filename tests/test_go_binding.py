"""CPU: the cgo binding in go/ (package gpurx and the batched PacketHandle patch for package
engine) is consistent with the C ABI, although no Go toolchain exists in this image:

* the C side of the cgo preamble (go/gpurx/gpurx_shim.h) compiles with gcc -Werror against
  include/halo_rx.h, links against libhalo_rx.so and runs (host-only calls);
* every C.<name> the Go files use is declared by halo_rx.h, the shim or the C scalar types;
* every gpurx.<Name> the engine patch uses is declared in package gpurx, and every NetIf method or
  field it uses exists in the patch or in the reference's package engine;
* gpurx.Result mirrors halo_rx_result_t field for field, and the Status / Act constants equal the
  header's enums."""
from __future__ import annotations

import glob
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "go")
HDR = os.path.join(ROOT, "include", "halo_rx.h")
LIBDIR = os.path.join(ROOT, "halo_amd", "lib")
REF_ENGINE = "/root/reference/engine"


def _src(path):
    return open(path, encoding="utf-8").read()


def _strip_comments(go: str) -> str:
    go = re.sub(r"/\*.*?\*/", "", go, flags=re.S)
    return re.sub(r"//[^\n]*", "", go)


def test_shim_compiles_links_and_runs(tmp_path):
    drv = tmp_path / "drv.c"
    drv.write_text(r'''
#include <stdio.h>
#include "gpurx_shim.h"
int main(void) {
    const uint8_t mac[6] = {0xAA, 0xAA, 0xAA, 0xAA, 0xAA, 0xAA};
    halo_rx_netif_t n = gpurx_netif(mac, 0xC0A86464u, 1);
    if (n.mac[5] != 0xAA || n.ip != 0xC0A86464u || n.nat_enable != 1 || n.pad[0] || n.pad[1]) return 2;
    halo_rx_result_t r;
    memset(&r, 0, sizeof r);
    r.status = HALO_RX_OK; r.flags = HALO_RX_F_MAC_MATCH | HALO_RX_F_DST_IS_OWN; r.ethertype = 0x0800;
    r.ip_proto = 17; r.dst_ip = 0xC0A86464u;
    uint8_t act = 0xFF;
    n.nat_enable = 0;
    if (halo_rx_dispatch(&r, 1, &n, &act, NULL) != HALO_OK || act != HALO_RX_ACT_LOCAL_UDP) return 3;
    uint8_t frame[4] = {0};
    if (gpurx_parse_one(NULL, frame, 4, 1, 0, &r) != HALO_E_INVAL) return 4;
    printf("%s\n", halo_rx_strerror(HALO_E_NODEV));
    return 0;
}
''')
    exe = tmp_path / "drv"
    cmd = ["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", f"-I{os.path.join(ROOT, 'include')}",
           f"-I{os.path.join(GO, 'gpurx')}", str(drv), f"-L{LIBDIR}", "-lhalo_rx", f"-Wl,-rpath,{LIBDIR}", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)


def test_cpu_entry_preamble_compiles_links_and_runs(tmp_path):
    """go/gpurx/cpu.go's preamble: halo_rx_cpu.h + -lhalo_rx_cpu, one all-zero frame (ETH_TYPE)."""
    drv = tmp_path / "cpu.c"
    drv.write_text(r'''
#include <string.h>
#include "halo_rx_cpu.h"
int main(void) {
    halo_rx_netif_t n;
    memset(&n, 0, sizeof n);
    uint8_t frame[64] = {0};
    uint64_t off = 0;
    uint16_t len = 64;
    halo_rx_result_t r;
    if (halo_rx_parse_batch_cpu(frame, &off, &len, 1, HALO_RX_CSUM_ENABLE | HALO_RX_L3_START, &n, &r, NULL) != HALO_OK)
        return 2;
    if (r.status != HALO_RX_IP_VER) return 3;
    if (halo_rx_parse_batch_cpu(frame, &off, &len, 1, HALO_RX_CSUM_ENABLE, &n, &r, NULL) != HALO_OK) return 4;
    return r.status == HALO_RX_ETH_TYPE ? 0 : 5;
}
''')
    exe = tmp_path / "cpu"
    cmd = ["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", f"-I{os.path.join(ROOT, 'include')}", str(drv),
           f"-L{LIBDIR}", "-lhalo_rx_cpu", f"-Wl,-rpath,{LIBDIR}", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)


def _header_names():
    h = _src(HDR) + _src(os.path.join(GO, "gpurx", "gpurx_shim.h")) + _src(os.path.join(ROOT, "include", "halo_rx_cpu.h"))
    names = set(re.findall(r"\b(halo_\w+|HALO_\w+|gpurx_\w+)\b", h))
    return names | {"uint8_t", "uint16_t", "uint32_t", "uint64_t", "int64_t", "int", "GoString"}


def test_every_c_name_is_declared():
    declared = _header_names()
    used = set()
    for f in glob.glob(os.path.join(GO, "gpurx", "*.go")):
        used |= set(re.findall(r"\bC\.(\w+)", _strip_comments(_src(f))))
    assert used, "no C names found"
    missing = sorted(u for u in used if u not in declared)
    assert not missing, missing
    # the preamble of every cgo file includes the shim (static helpers are per file)
    for f in glob.glob(os.path.join(GO, "gpurx", "*.go")):
        s = _src(f)
        if 'import "C"' in s:
            assert '#include "gpurx_shim.h"' in s.split('import "C"')[0], f


def _gpurx_exports():
    out = set()
    for f in glob.glob(os.path.join(GO, "gpurx", "*.go")):
        s = _strip_comments(_src(f))
        out |= set(re.findall(r"^func (?:\([^)]*\) )?([A-Z]\w*)", s, flags=re.M))
        out |= set(re.findall(r"^type ([A-Z]\w*)", s, flags=re.M))
        out |= set(re.findall(r"^\s+([A-Z]\w*)\s*(?:=|\s+\w+\s*=)", s, flags=re.M))  # const/var blocks
        out |= set(re.findall(r"^var ([A-Z]\w*)", s, flags=re.M))
    return out


def test_engine_patch_uses_only_defined_names():
    patch = _strip_comments(_src(os.path.join(GO, "engine", "packet_handle_batched.go")))
    exports = _gpurx_exports()
    used = set(re.findall(r"\bgpurx\.([A-Za-z]\w*)", patch))
    missing = sorted(u for u in used if u not in exports)
    assert not missing, missing
    # methods called on Batch / Result / Ctx values exist in package gpurx
    for m in set(re.findall(r"\b(?:b|r|x)\.([A-Z]\w*)\(", patch)):
        assert m in exports, m
    if not os.path.isdir(REF_ENGINE):
        pytest.skip("reference engine sources not present")
    ref = "".join(_src(f) for f in glob.glob(os.path.join(REF_ENGINE, "*.go")))
    own = set(re.findall(r"^func \(i \*NetIf\) (\w+)", patch, flags=re.M))
    for m in set(re.findall(r"\bi\.([A-Za-z]\w*)\(", patch)):
        assert m in own or re.search(rf"func \(i \*NetIf\) {m}\(", ref), m
    for fld in set(re.findall(r"\bi\.([A-Z]\w*)\b(?!\()", patch)):
        assert re.search(rf"^\s+{fld}\s", ref, flags=re.M), fld
    for name in ("DhcpClientPort", "DhcpServerPort", "UdpSession", "TcpSession", "Log"):
        assert re.search(rf"\b{name}\b", ref), name


def test_result_struct_and_constants_mirror_header():
    from halo_amd._lib import ACTION_NAMES, RESULT_DTYPE, STATUS_NAMES

    go = _strip_comments(_src(os.path.join(GO, "gpurx", "gpurx.go")))
    body = re.search(r"type Result struct \{(.*?)\n\}", go, flags=re.S).group(1)
    fields = re.findall(r"^\s*(\w+)\s+(uint8|uint16|uint32)\s*$", body, flags=re.M)
    sizes = {"uint8": 1, "uint16": 2, "uint32": 4}
    assert [sizes[t] for _, t in fields] == [RESULT_DTYPE.fields[n][0].itemsize for n in RESULT_DTYPE.names]
    assert sum(sizes[t] for _, t in fields) == 32
    consts = dict((k, int(v)) for k, v in re.findall(r"^\s*(Status\w+|Act\w+)\s*=\s*(\d+)", go, flags=re.M))
    camel = lambda s: "".join(p.capitalize() for p in s.split("_"))  # noqa: E731
    for code, name in enumerate(STATUS_NAMES):
        key = "Status" + {"OK": "OK"}.get(name, camel(name).replace("Totlen", "TotLen"))
        assert consts.get(key) == code, (key, consts.get(key))
    for code, name in enumerate(ACTION_NAMES):
        assert consts.get("Act" + camel(name)) == code, name


def test_go_sources_are_balanced():
    for f in glob.glob(os.path.join(GO, "**", "*.go"), recursive=True):
        s = _strip_comments(_src(f))
        s = re.sub(r'"(\\.|[^"\\])*"', '""', s)
        s = re.sub(r"'(\\.|[^'\\])*'", "''", s)
        for a, b in ("{}", "()", "[]"):
            assert s.count(a) == s.count(b), (f, a)
        assert re.match(r"\s*package \w+", s), f
