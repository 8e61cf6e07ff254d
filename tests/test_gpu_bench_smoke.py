"""GPU: the default bench.py line end to end at a small batch -- every
sub-measurement and probe the driver's round-end run takes (the conv-forward
roofline probe, mode B with its weight-gradient probe, config 2, config 5
with the fp8 / token-GEMM probes, the CPU baseline), so a launch-argument
mismatch in a probe's replay fails here instead of in the driver's bench."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_default_bench_line_small_batch():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--batch", "4",
                        "--cpu-batch", "2", "--cpu-steps", "1"], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=560)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["value"] > 0 and d["n_gpus"] == 1 and d["roofline"]["frac"] > 0
    assert d["mode_b"]["value"] > 0 and d["mode_b"]["roofline"]["frac"] > 0
    assert d["config2"]["value"] > 0
    c5 = d["config5"]
    assert c5["value"] > 0 and c5["roofline"]["fp8_gemm"]["frac"] > 0 and c5["roofline"]["tok_gemm"]["frac"] > 0
    assert d["cpu_baseline"]["value"] > 0, d["cpu_baseline"]
    assert d["encoder_forward"]["ms"] > 0
