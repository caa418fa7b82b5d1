"""bench.py --gpus N without torchrun: the launcher starts N rank processes with the
torch.distributed environment set (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT) and
returns the first failing exit code.  Runs on CPU: the children here are stand-ins that
report their environment; no GPU is touched by the launcher itself."""

import json
import os
import sys

import bench


def test_spawn_ranks_sets_rank_environment(tmp_path):
    out = tmp_path / "env"
    code = ("import json, os, sys; keys = ['RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT'];"
            f"open(os.path.join({str(tmp_path)!r}, 'env' + os.environ['RANK']), 'w').write("
            "json.dumps({k: os.environ[k] for k in keys}))")
    rc = bench.spawn_ranks(2, [sys.executable, "-c", code], port=29555)
    assert rc == 0
    envs = [json.load(open(str(out) + str(r))) for r in range(2)]
    for r, e in enumerate(envs):
        assert e == {"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": "2", "MASTER_ADDR": "127.0.0.1",
                     "MASTER_PORT": "29555"}


def test_spawn_ranks_propagates_failure():
    code = "import os, sys; sys.exit(3 if os.environ['RANK'] == '1' else 0)"
    assert bench.spawn_ranks(2, [sys.executable, "-c", code]) == 3


def test_bench_rejects_mismatched_world(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    try:
        bench.main()
    except SystemExit as e:
        assert "WORLD_SIZE=2" in str(e.code)
    else:
        raise AssertionError("bench.main accepted --gpus 4 with WORLD_SIZE=2")


def test_spawn_ranks_stops_blocked_peer_on_failure():
    # rank 0 waits forever (as in a collective whose peer died); rank 1 fails with 3: the
    # launcher must return 3 within seconds and leave no rank running
    import time
    code = "import os, sys, time; r = os.environ['RANK']; time.sleep(3600) if r == '0' else sys.exit(3)"
    t0 = time.monotonic()
    assert bench.spawn_ranks(2, [sys.executable, "-c", code]) == 3
    assert time.monotonic() - t0 < 20


def test_spawn_ranks_timeout_kills_hung_ranks():
    import time
    code = "import time; time.sleep(3600)"
    t0 = time.monotonic()
    assert bench.spawn_ranks(2, [sys.executable, "-c", code], timeout=2) == 124
    assert time.monotonic() - t0 < 20


def test_bench_rank_refuses_missing_gpus(monkeypatch):
    # no GPU in this container: a 2-rank job must stop before set_device with a clear message
    for k, v in dict(WORLD_SIZE="2", RANK="1", LOCAL_RANK="1", LOCAL_WORLD_SIZE="2").items():
        monkeypatch.setenv(k, v)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--deadline", "0"])
    try:
        bench.main()
    except SystemExit as e:
        assert "visible GPU" in str(e.code)
    else:
        raise AssertionError("bench.main ran a 2-rank job without GPUs")
