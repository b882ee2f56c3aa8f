"""bench.py's one-line JSON contract (the driver parses it), on the GPU: SC and SCL lines with the
roofline and CPU-baseline objects."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("decoder", ["sc", "scl"])
def test_bench_json_contract(decoder):
    d = _run("--decoder", decoder, "--steps", "5", "--warmup", "1", "--cpu-seconds", "0.5", "--settle-ms", "0")
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in d, key
    assert d["n_gpus"] == 1 and d["steps"] == 5 and d["scaling"] == "weak" and d["higher_is_better"] is True
    assert d["value"] > 0 and d["unit"] == "Mcodewords/s"
    assert d["config"]["kernel"] in ("specialized", "scl_subtree")
    rf = d["roofline"] if decoder == "sc" else d["roofline_hbm"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-4
    # the VALU-issue roofline from the committed per-class SQ counters and issue costs
    # (profiles/valu.json): the list decoder's own bound; next to the HBM one for SC
    rv = d["roofline"] if decoder == "scl" else d["roofline_valu"]
    assert rv["bound"] == "valu_issue" and rv["stale"] is False and rv["counter_files"]
    assert 0 < rv["frac_lo"] <= rv["frac"] <= rv["frac_hi"] < 1.2
    assert abs(rv["frac"] - rv["achieved"] / rv["peak"]) < 1e-3
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1 and cb["sample"]
    assert cb["best_of"] == 3 and cb["single_thread"]["cores"] == 1 and cb["single_thread"]["value"] > 0
    assert d["dtype"] == ("f32" if decoder == "sc" else "f64")
