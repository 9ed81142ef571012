"""bench.py on the GPU (small configurations): the JSON line's contract fields,
the oracle check of the bench's own outputs, and the decodes-in-flight path
(two contexts, streams and output sets; outputs compared before timing)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("inflight", ["1", "2"])
def test_bench_c2_line(inflight):
    d = _bench("--config", "c2", "--steps", "3", "--warmup", "1", "--no-cpu",
               "--decode-inflight", inflight)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["value"] > 0
    assert d["decodes_in_flight"] == int(inflight)
    assert d["latency_ms_per_step"] > 0
    assert d["verify"]["verified"].startswith("all output arrays == oracle")
    r = d["roofline"]
    assert r["bound"] == "hbm" and 0 < r["frac"] < 1 and r["peak"] == 8000.0


@pytest.mark.gpu
def test_rccl_control_plane_world1():
    """The nccl (RCCL) control plane executes on the GPU: process group init with
    device_id, barriers and the all_gather of the ranks' times, at world size 1
    under torch.distributed.run (two ranks cannot share one GPU under RCCL).
    The default control plane is gloo (no data-path collective exists)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "1", "--master-addr", "127.0.0.1",
                        "--master-port", "29631", os.path.join(ROOT, "bench.py"), "--gpus", "1",
                        "--config", "c2", "--steps", "3", "--warmup", "1", "--no-cpu",
                        "--dist-backend", "nccl", "--dist-always"],
                       capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["dist"] == {"world_size": 1, "dist_backend": "nccl"}, d["dist"]
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert d["verify"]["verified"].startswith("all output arrays == oracle")
