"""Host-side checks of bench.py (no GPU): the configuration presets, the work
directory choice for the end-to-end leg (statvfs), and the failure path — any
error still prints one JSON line with an `error` field and exits 1."""
import importlib.util
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_presets():
    b = _bench()
    want = {2: (50_000_000, 31, 2, "alltoall"), 3: (50_000_000, 31, 3, "files"),
            4: (125_000_000, 31, 4, "alltoall"), 5: (20_000_000, 55, 5, "alltoall")}
    for cfg, (reads, k, seed, xch) in want.items():
        a = b.parse_args(["--config", str(cfg)])
        assert (a.reads, a.k, a.seed, a.exchange) == (reads, k, seed, xch)
        assert a.value == "device" and a.e2e is None
    a = b.parse_args(["--config", "4", "--exchange", "none", "--reads", "7"])
    assert a.exchange == "none" and a.reads == 7
    a = b.parse_args(["--mode", "e2e"])  # round-3 spelling
    assert a.value == "e2e" and a.e2e is True


def test_pick_workdir(tmp_path):
    b = _bench()
    d, free, tried = b.pick_workdir(str(tmp_path), 1 << 20)
    assert d == str(tmp_path) and free >= 1 << 20 and str(tmp_path) in tried
    d, free, tried = b.pick_workdir(str(tmp_path), 1 << 62)
    assert d is None and free == 0 and tried[str(tmp_path)] < 1 << 62


def test_failure_prints_one_json_error_line():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--k", "0", "--no-cpu"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 1
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["value"] is None and d["error"] and d["metric"].startswith("k-mers/s")
