"""The stdout line bench.py prints is what the driver parses (round 5's 20,145-char
line was not parsed). These CPU tests push recorded full bench records through the same
compaction bench.py applies before printing, and check size, strict JSON and the contract keys."""
import json
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RECORD = os.path.join(ROOT, "profiles", "r05", "r5zz3", "bench.json")  # round 5's full N=1 line
CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config")


def _strict(s: str):
    def bad(c):
        raise ValueError(f"non-strict JSON constant {c}")

    return json.loads(s, parse_constant=bad)


def _check(line: dict) -> dict:
    s = json.dumps(bench.compact_line(line))
    assert len(s.encode()) < 8192
    assert "\n" not in s
    back = _strict(s)
    for k in CONTRACT:
        assert k in back, k
    return back


def test_round5_record_fits_and_keeps_the_headline():
    full = json.load(open(RECORD))
    assert len(json.dumps(full)) > 8192  # the record that broke the driver's parse
    back = _check(full)
    assert back["value"] == full["value"] and back["ms_per_step"] == full["ms_per_step"]
    r = back["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert r[k] == full["roofline"][k]
    assert "note" not in r and "peak_measured_read_probes" not in r
    cb = back["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb
    assert back["config4_128M_one_gpu"]["roofline"]["frac"] == full["config4_128M_one_gpu"]["roofline"]["frac"]
    # every secondary survives at this size, numbers only
    assert "secondary_dropped" not in back
    assert set(back["secondary"]) == set(full["secondary"])
    for name, e in back["secondary"].items():
        src = full["secondary"][name]
        if "kernel_ms" in src:
            assert e["kernel_ms"] == src["kernel_ms"], name
        if "roofline" in src:
            assert e["roofline"]["frac"] == src["roofline"]["frac"], name
            if "frac_of_size_matched" in src["roofline"]:
                assert e["roofline"]["frac_of_size_matched"] == src["roofline"]["frac_of_size_matched"]
        for k in ("what", "note", "path", "mix", "sample", "table", "gather_probe"):
            assert k not in e, (name, k)


def test_oversized_secondaries_are_dropped_not_the_headline():
    full = json.load(open(RECORD))
    for i in range(60):  # far more secondaries than any run makes
        full["secondary"][f"extra_{i}"] = {"mpps": 1.0 + i, "kernel_ms": 0.5, "roofline": {"frac": 0.5}}
    back = _check(full)
    assert back["secondary_dropped"]
    assert back["roofline"]["frac"] == full["roofline"]["frac"]
    assert back["cpu_baseline"]["value"] == full["cpu_baseline"]["value"]


def test_n_rank_line_fits():
    full = json.load(open(RECORD))
    full.pop("secondary")
    full.pop("config4_128M_one_gpu")
    full["n_gpus"] = 8
    full["cpu_baseline"] = None
    full["per_rank"] = [dict(full["per_rank"][0], rank=r, pci_bus_id=f"0000:{r:02x}:00.0") for r in range(8)]
    full["per_rank_kernel_ms"] = [0.0219] * 8
    full["whole_shard_launch"] = {"value": 1.0, "unit": "Mpps", "steps": 200, "ms_per_step": 0.3,
                                  "per_rank_kernel_ms": [0.3] * 8, "what": "x" * 300}
    back = _check(full)
    assert len(back["per_rank"]) == 8 and all(r["valid"] for r in back["per_rank"])
    assert back["cpu_baseline"] is None
    assert "what" not in back["whole_shard_launch"]


def test_emit_line_writes_detail(tmp_path, capsys):
    full = json.load(open(RECORD))
    p = tmp_path / "d" / "detail.json"
    s = bench.emit_line(full, str(p))
    out = capsys.readouterr().out.strip().splitlines()
    assert out[-1] == s
    assert json.load(open(p)) == full


@pytest.mark.parametrize("limit", [2048, 4096])
def test_limit_is_honoured(limit):
    full = json.load(open(RECORD))
    c = bench.compact_line(full, limit=limit)
    # secondaries go first; the headline, roofline and CPU baseline are never dropped
    assert len(json.dumps(c)) <= limit or not c["secondary"]
    assert c["roofline"]["frac"] == full["roofline"]["frac"]


def test_cpu_baseline_reports_threads_and_busy_cores():
    """bench.cpu_baseline on a small shard (CPU only): one thread, the share and every CPU, each with
    its busy-core measurement, and the cgroup quota field present (None where unlimited)."""
    import numpy as np
    import torch

    from halo_amd import synth
    from oracle import oracle as O

    O.build()
    lay = synth.layout(1 << 16, length=64)
    data = O.synth_batch(lay["seed"], 0, lay["lens"], lay["kinds"], O.NetIf.make(), offsets_dw=lay["offsets_dw"])
    res = bench.cpu_baseline({"bytes": torch.from_numpy(np.ascontiguousarray(data)), "layout": lay}, 0.4, 16)
    assert res["unit"] == "Mpps" and res["cores"] == 1 and res["kind"] == "port" and res["value"] > 0
    for k in ("multi_thread", "multi_thread_share"):
        assert res[k]["value"] > 0 and res[k]["threads"] >= 1 and res[k]["cores_busy"] >= 0
    assert "cpu_quota_cores" in res["multi_thread"]
    assert "16 batches" in res["sample"]
    ce = res["cpu_entry"]
    assert ce["ok"] and ce["value"] > 0 and ce["value_threads"] > 0 and ce["threads"] == 1
    assert len(json.dumps(bench.compact_line({"cpu_baseline": res})["cpu_baseline"])) < 800


def test_cgroup_quota_parser():
    """None (unlimited / unknown) or a positive CPU count, on whatever cgroup layout this host has."""
    q = bench.cgroup_cpu_quota()
    assert q is None or q > 0
