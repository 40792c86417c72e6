"""`bench.py --gpus N` starts its own ranks when no launcher did (CPU tests).

The driver runs `bench.py --gpus N` for its 1 -> 8 scaling line; without
torch.distributed.run around it, bench.launch_ranks must start N ranks with
the environment torch.distributed.run would give them, relay rank 0's line,
fail when any rank fails, refuse more nccl ranks than GPUs before starting
anything, and drop a line whose ranks_seen is not N.  The ranks here are stub
children (no GPU in this container); the GPU run is
`bench.py --gpus 2 --dist-backend gloo` on the one-GPU box.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

# a stand-in rank: reports the environment it was given; rank 0 prints the
# result line (ranks_seen from WORLD_SIZE unless STUB_SEEN overrides it);
# STUB_FAIL=k makes rank k exit 3
STUB = r"""
import json, os, sys, time
r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
if os.environ.get("STUB_FAIL") == str(r):
    sys.exit(3)
if os.environ.get("STUB_HANG") == str(r):
    time.sleep(600)
env = {k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                                  "MASTER_PORT", "HSA_ENABLE_IPC_MODE_LEGACY")}
open(os.path.join(os.environ["STUB_DIR"], f"rank{r}.json"), "w").write(json.dumps({"env": env, "argv": sys.argv[1:]}))
if r == 0:
    print("progress line of rank 0")
    seen = int(os.environ.get("STUB_SEEN", w))
    print(json.dumps({"metric": "m", "value": 1.0, "n_gpus": w, "ranks_seen": seen}))
"""


def _args(n, backend="gloo"):
    return argparse.Namespace(gpus=n, dist_backend=backend)


@pytest.fixture
def stub(tmp_path, monkeypatch):
    path = tmp_path / "stub.py"
    path.write_text(STUB)
    monkeypatch.setenv("STUB_DIR", str(tmp_path))
    for k in ("STUB_FAIL", "STUB_SEEN", "STUB_HANG", "WORLD_SIZE", "RANK"):
        monkeypatch.delenv(k, raising=False)
    return [sys.executable, str(path)], tmp_path


def test_rank_env():
    env = bench.rank_env({"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}, 2, 4, 29500)
    assert env["RANK"] == "2" and env["LOCAL_RANK"] == "2" and env["WORLD_SIZE"] == "4"
    assert env["LOCAL_WORLD_SIZE"] == "4" and env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29500"
    assert env["PATH"] == "/bin" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert bench.rank_env({}, 0, 1, 1)["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


@pytest.mark.parametrize("n", [2, 3])
def test_launch_ranks_relays_rank0_line(stub, capsys, n):
    child, d = stub
    argv = ["--gpus", str(n), "--dist-backend", "gloo", "--steps", "4", "--warmup", "1"]
    rc = bench.launch_ranks(_args(n), argv, child=child, timeout=60)
    assert rc == 0
    out = capsys.readouterr().out.strip().splitlines()
    assert out[-1].startswith("{")
    line = json.loads(out[-1])
    assert line["n_gpus"] == n and line["ranks_seen"] == n
    assert "progress line of rank 0" in out
    ports = set()
    for r in range(n):
        got = json.loads((d / f"rank{r}.json").read_text())
        assert got["argv"] == argv                           # the same flags reach every rank
        e = got["env"]
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"]) == (str(r), str(r), str(n))
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
        ports.add(e["MASTER_PORT"])
    assert len(ports) == 1


def test_launch_ranks_fails_when_a_rank_fails(stub, capsys, monkeypatch):
    child, _ = stub
    monkeypatch.setenv("STUB_FAIL", "1")
    monkeypatch.setenv("STUB_HANG", "0")           # rank 0 would wait forever for the failed rank
    rc = bench.launch_ranks(_args(2), ["--gpus", "2"], child=child, timeout=60)
    assert rc == 1
    assert "failed" in capsys.readouterr().err


def test_launch_ranks_drops_line_with_wrong_ranks_seen(stub, capsys, monkeypatch):
    child, _ = stub
    monkeypatch.setenv("STUB_SEEN", "1")
    rc = bench.launch_ranks(_args(2), ["--gpus", "2"], child=child, timeout=60)
    assert rc == 1
    out = capsys.readouterr().out.strip().splitlines()
    assert "error" in json.loads(out[-1])
    assert not any('"value"' in line for line in out)


def test_launch_ranks_refuses_more_nccl_ranks_than_gpus(stub, capsys):
    child, d = stub
    rc = bench.launch_ranks(_args(2, "nccl"), ["--gpus", "2"], child=child, device_count=1)
    assert rc == 2
    cap = capsys.readouterr()
    assert "device_count() = 1" in cap.out and "1 visible GPU" in cap.err
    assert not list(d.glob("rank*.json"))                     # nothing started


def test_bench_gpus2_nccl_without_gpus_exits_nonzero():
    """The real entry point: no GPU here, so --gpus 2 over nccl must stop
    before any rank starts and name the device count."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "device_count() = 0" in p.stdout


def test_bench_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 1 and "WORLD_SIZE=2" in p.stdout
