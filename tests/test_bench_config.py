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
