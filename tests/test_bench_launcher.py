"""bench.py --gpus N without a launcher: the parent starts N rank processes
(no GPU, no torch in the parent), relays rank 0's JSON line and fails when any
rank fails.  The child command is stubbed: no GPU needed."""
import json
import os
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def _child(body):
    return [sys.executable, "-c", "import json, os, sys, time\n" + body]


def test_rank_env():
    env = bench.rank_env({"PATH": "/bin"}, 3, 8, 29400)
    assert env["RANK"] == "3" and env["LOCAL_RANK"] == "3"
    assert env["WORLD_SIZE"] == "8" and env["LOCAL_WORLD_SIZE"] == "8"
    assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29400"
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert env["PATH"] == "/bin"


def test_launch_relays_rank0_line_and_child_env(tmp_path, capsys):
    body = (
        "r = int(os.environ['RANK'])\n"
        "keys = ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')\n"
        "open(os.path.join(%r, 'env%%d' %% r), 'w').write(json.dumps(\n"
        "    {k: os.environ[k] for k in keys}))\n"
        "print('progress noise')\n"
        "if r == 0:\n"
        "    print(json.dumps({'metric': 'm', 'n_gpus': int(os.environ['WORLD_SIZE'])}))\n"
        % str(tmp_path))
    rc = bench.launch(4, [], child=_child(body))
    assert rc == 0
    out = capsys.readouterr().out.strip().splitlines()
    assert json.loads(out[-1]) == {"metric": "m", "n_gpus": 4}
    envs = [json.loads((tmp_path / ("env%d" % r)).read_text())
            for r in range(4)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert {e["WORLD_SIZE"] for e in envs} == {"4"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1


def test_launch_fails_when_a_rank_fails_and_stops_the_others(capsys):
    body = ("r = int(os.environ['RANK'])\n"
            "if r == 1:\n"
            "    sys.exit(3)\n"
            "time.sleep(120)\n"
            "print(json.dumps({'n_gpus': 2}))\n")
    t0 = time.time()
    rc = bench.launch(2, [], child=_child(body))
    assert rc == 3
    assert time.time() - t0 < 60          # rank 0 was terminated, not awaited
    assert "rank 1 exited with 3" in capsys.readouterr().err


def test_launch_fails_on_wrong_world_or_no_line(capsys):
    wrong = "print(json.dumps({'n_gpus': 1})) if os.environ['RANK'] == '0' else None\n"
    assert bench.launch(2, [], child=_child(wrong)) == 1
    assert "n_gpus=1" in capsys.readouterr().err
    assert bench.launch(2, [], child=_child("pass\n")) == 1
    assert "no JSON line" in capsys.readouterr().err


def test_main_refuses_gpus_world_mismatch(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    monkeypatch.setenv("WORLD_SIZE", "1")
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert "WORLD_SIZE=1" in str(e.value)
