"""bench.py's per-config tables (no GPU): every BASELINE config has its
batches-in-flight default and parse-grid CUs, and the values stay in range
(the driver runs `python bench.py` with no flags, and N>1 with the same
defaults on every rank)."""
import importlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    sys.path.insert(0, REPO)
    try:
        return importlib.import_module("bench")
    finally:
        sys.path.pop(0)


def test_in_flight_tables_cover_every_config():
    bench = _bench()
    assert set(bench.INFLIGHT) == set(bench.CONFIGS)
    assert set(bench.PARSE_CUS_INFLIGHT) == set(bench.CONFIGS)
    for cfg in bench.CONFIGS:
        assert 1 <= bench.INFLIGHT[cfg] <= 4  # streams per process stay within GPU_MAX_HW_QUEUES (4)
        assert 0 < bench.PARSE_CUS_INFLIGHT[cfg] <= 256


def test_headline_config_defaults():
    bench = _bench()
    # the default line is C2 (BASELINE configs[1]); its in-flight default is 3
    assert bench.INFLIGHT["c2"] == 3 and bench.PARSE_CUS_INFLIGHT["c2"] == 192


def test_world_from_env(monkeypatch):
    """--gpus against the launcher's WORLD_SIZE: under a
    launcher the two must agree; without one the world is 1 (N > 1 self-launches)."""
    import pytest
    bench = _bench()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.world_from_env(None) == (1, False)
    assert bench.world_from_env(8) == (1, False)
    with pytest.raises(SystemExit):
        bench.world_from_env(0)
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert bench.world_from_env(4) == (4, True)
    assert bench.world_from_env(None) == (4, True)
    with pytest.raises(SystemExit):
        bench.world_from_env(8)


def test_self_launch_command(monkeypatch):
    """bench.py --gpus N without a launcher runs the same argv as N ranks under
    torch.distributed.run on 127.0.0.1, as a child, and exits with its status."""
    import subprocess
    bench = _bench()
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7

    monkeypatch.setattr(subprocess, "call", fake_call)
    rc = bench.launch_ranks(8, ["--gpus", "8", "--config", "c3"])
    assert rc == 7
    cmd = seen["cmd"]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--config", "c3"]
    assert os.path.basename(cmd[-5]) == "bench.py"
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_main_self_launches_before_touching_torch(monkeypatch):
    """main() with --gpus 2 and no WORLD_SIZE hands off to launch_ranks before
    importing torch / initialising HIP (a parent that initialised the GPU must
    not start the rank processes)."""
    import pytest
    bench = _bench()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    calls = []
    monkeypatch.setattr(bench, "launch_ranks", lambda n, argv: calls.append((n, argv)) or 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0
    assert calls == [(2, ["--gpus", "2", "--steps", "3"])]


def test_hbm_config_validated(monkeypatch):
    import pytest
    bench = _bench()
    monkeypatch.setattr(sys, "argv", ["bench.py", "--hbm-config", "c9"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 2


def test_reference_baseline_is_the_fastest_run():
    """cpu_baseline (kind reference) reports the minimum wall of its repeats
    (VERDICT r04 item 7), and says so in its sample text."""
    bench = _bench()
    for cfg in bench.CONFIGS:
        r = bench.reference_record(cfg)
        assert r is not None, cfg
        assert r["value"] == r["value_best"] >= r["value_median"]
        assert abs(r["value"] - r["aligned_bases"] / r["wall_min_s"]) <= 1e-3 * r["value"]
        assert "fastest of" in r["sample"]
