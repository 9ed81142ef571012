"""bench.py's multi-process control plane on CPU (no GPU): `--gpus N`
spawns N rank processes with the torch.distributed environment, and the
Dist helper's barrier / max / per-rank gather work over gloo at world 2 (the
driver's N > 1 runs use the same code over RCCL)."""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RANK_SCRIPT = textwrap.dedent("""
    import argparse, json, os, sys, time
    sys.path.insert(0, %r)
    import torch
    torch.cuda.set_device = lambda *a, **k: None   # no GPU in this test
    torch.cuda.synchronize = lambda *a, **k: None
    import bench
    args = argparse.Namespace(gpus=int(os.environ["WORLD_SIZE"]), device_mod=0,
                              dist_backend="gloo")
    D = bench.Dist(args, torch)
    rank = D.rank
    t_max, per = D.timed(lambda: time.sleep(0.01 * (1 + rank)), 3)
    print(json.dumps({"rank": rank, "world": D.world, "t_max": t_max, "per": per,
                      "info": D.info(), "env": [os.environ[k] for k in
                      ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")]}), flush=True)
    D.close()
""") % ROOT


def test_spawn_ranks_gloo_world2(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    out = tmp_path / "out.txt"
    cmd = [sys.executable, str(script)]
    launcher = textwrap.dedent(f"""
        import argparse, sys
        sys.path.insert(0, {ROOT!r})
        import bench
        sys.exit(bench.spawn_ranks(argparse.Namespace(gpus=2), cmd={cmd!r}))
    """)
    with open(out, "w") as f:  # the rank processes inherit the launcher's stdout
        rc = subprocess.run([sys.executable, "-c", launcher], stdout=f,
                            stderr=subprocess.STDOUT, timeout=180).returncode
    text = out.read_text()
    assert rc == 0, text
    lines = [json.loads(ln) for ln in text.splitlines() if ln.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1]
    for x in lines:
        assert x["world"] == 2 and x["info"] == {"world_size": 2, "dist_backend": "gloo"}
        assert x["env"][0] == x["env"][1] == str(x["rank"]) and x["env"][2] == "2"
        assert x["env"][3] == "127.0.0.1"
        assert len(x["per"]) == 2 and x["t_max"] == max(x["per"])
        assert x["per"][1] > x["per"][0]  # rank 1 sleeps longer: max is over ranks


def test_world_size_mismatch_is_an_error():
    sys.path.insert(0, ROOT)
    import bench
    import pytest
    env = dict(os.environ)
    try:
        os.environ["WORLD_SIZE"] = "2"
        with pytest.raises(SystemExit):
            bench.Dist(argparse.Namespace(gpus=4, device_mod=0, dist_backend="gloo"), None)
    finally:
        os.environ.clear()
        os.environ.update(env)
