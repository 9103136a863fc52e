"""bench.py plumbing on CPU: the --gpus N launcher (one child
torch.distributed.run, gloo in --dry-run), the JSON line contract, and the
CPU-baseline legs of every workload (bounded, host only)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _json_line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


@pytest.mark.parametrize("gpus,workload", [(1, "fwt1d"), (2, "fwt1d"), (2, "fwt2d"),
                                           (2, "modwt"), (2, "wpt")])
def test_launcher_dry_run(gpus, workload):
    """The launcher at world 1 and 2 for every workload; at world 2 the
    sharded configs 3 and 5 run their real exchanges (all-to-all transposes,
    MODWT ring halos) over gloo around placeholder compute, and report the
    exchange time apart."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus),
                        "--dry-run", "--steps", "3", "--warmup", "1", "--workload", workload],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == gpus
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d
    assert d["value"] > 0 and d["steps"] == 3
    if gpus > 1 and workload in ("fwt2d", "modwt"):
        assert d["scaling"] == "strong" and d["exchange_ms_per_step"] > 0
        assert d["roundtrip_max_abs_err"] == 0.0  # placeholder compute: exact round trip


def test_world_mismatch_is_explained():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dry-run"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0
    assert "torch.distributed.run" in (r.stderr + r.stdout)


@pytest.mark.parametrize("kind", ["fwt1d", "wpt", "modwt"])
def test_cpu_baseline_legs(kind):
    import bench
    import jwave_amd as jw
    w = jw.by_class({"fwt1d": "Daubechies4", "wpt": "Symlet8", "modwt": "Daubechies4"}[kind])
    cb = bench.cpu_baseline((kind, w), 0.01)
    assert cb["value"] > 0 and cb["unit"] == "samples/s" and cb["kind"] == "port"
    assert cb["cores"] >= 1 and cb["host"]["nproc"] >= 1 and cb["host"]["cpu_model"]


def test_load_traffic_is_keyed_by_workload():
    import bench
    # no committed summary holds a "nosuch" workload: never borrow another's bytes
    assert bench.load_traffic("nosuch", "fwt_fwd_tile", "exact") == (None, None, None)


def test_load_traffic_prefers_the_measured_library(tmp_path, monkeypatch):
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    key = "fwt2d:fwt_fwd_tile/exact"
    for name, sha, b in (("pmc_a.json", "aaaa", 1.0), ("pmc_b.json", "bbbb", 2.0)):
        (prof / name).write_text(json.dumps({"build": {"lib_sha256": sha},
                                             "kernels": {key: {"hbm_bytes_per_launch": b}}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.load_traffic("fwt2d", "fwt_fwd_tile", "exact", "aaaa") == (1.0, "profiles/pmc_a.json", "aaaa")
    # no summary of that library: the latest one, with its own digest
    assert bench.load_traffic("fwt2d", "fwt_fwd_tile", "exact", "cccc") == (2.0, "profiles/pmc_b.json", "bbbb")


def test_step_bounds_floors():
    """Both floors of a step from the algorithmic counts (DESIGN §6 'Two
    floors'): config 2 is HBM-bound, config 4 FP64-bound, and FMA math halves
    the FP64 floor."""
    import bench
    n = 1 << 24
    sb = bench.step_bounds("fwt1d", "exact", 2 * 16.0 * n, 2 * n, 0.1072)
    assert sb["bound"] == "hbm"
    assert abs(sb["hbm_floor_ms"] - 2 * 16.0 * n / 8e12 * 1e3) < 1e-4
    assert abs(sb["fp64_floor_ms"] - 32 * 2 * n / 39.3e12 * 1e3) < 1e-4
    assert abs(sb["frac"] - sb["hbm_floor_ms"] / 0.1072) < 1e-3
    b, m = 4096, 1 << 16
    ex = bench.step_bounds("wpt", "exact", 2 * 16.0 * b * m, 2 * b * m, 4.28)
    fm = bench.step_bounds("wpt", "fma", 2 * 16.0 * b * m, 2 * b * m, 3.06)
    assert ex["bound"] == "fp64" and abs(ex["fp64_floor_ms"] - 2.623) < 1e-3
    assert abs(fm["fp64_floor_ms"] * 2 - ex["fp64_floor_ms"]) < 2e-4
    assert bench.step_bounds("dry-run", "exact", 1.0, 1, 1.0) is None
