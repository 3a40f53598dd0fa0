"""The CLI's job pipeline (mapped_paf_read_parser._ingest_and_pileup), CPU
only: the device step is replaced by a recorder, so the order of ingest,
launches and errors is checked without a GPU (the outputs themselves are
checked against the reference's goldens by the -m gpu CLI tests)."""
import importlib

import pytest

from test_ingest_native import paf_line

cli = importlib.import_module("minion-plasmid-consensus_amd.mapped_paf_read_parser")
pkg = importlib.import_module("minion-plasmid-consensus_amd")


def _job(tmp_path, tag, reads_name, names, reads_txt=None):
    ref = tmp_path / f"{tag}.fa"
    ref.write_text(">r\nACGTACGTAC\n")
    paf = tmp_path / f"{tag}.paf"
    paf.write_text("".join(paf_line(n, 10, 0, 10, "+", 0, ":10") for n in names))
    reads = tmp_path / reads_name
    if reads_txt is not None:
        reads.write_text(reads_txt)
    return [str(ref), str(paf), str(reads)]


def _argv(jobs, mdf="0.1"):
    argv = []
    for k, (ref, paf, reads) in enumerate(jobs):
        argv += ["--job", ref, paf, reads, f"/nonexistent/c{k}", f"/nonexistent/ch{k}", f"/nonexistent/a{k}"]
    return argv + (["--min_depth_factor", mdf] if mdf else []) + ["--global_threshold_factor", "5"]


@pytest.fixture
def launches(monkeypatch):
    calls = []

    def fake_pileup(samples, mdf, gtf, device=0, row_cap=None):
        calls.append([len(s["tstart"]) for s in samples])
        fail = getattr(fake_pileup, "fail", {})  # launch number -> failing read index in the launch
        if getattr(fake_pileup, "fail_at", None) == len(calls):
            raise pkg.engine.DataError(pkg.engine.DE_KEY, 1)
        if len(calls) in fail:
            raise pkg.engine.DataError(pkg.engine.DE_KEY, fail[len(calls)])
        return [dict(count=[], max_depth=0) for _ in samples]

    monkeypatch.setattr(pkg.engine, "pileup", fake_pileup)
    return calls, fake_pileup


def test_groups_by_reads_file_first_job_error_wins(tmp_path, launches, capsys):
    calls, _ = launches
    a = _job(tmp_path, "a", "r1.fa", ["x", "y"], ">x\nACGTACGTAC\n>y\nACGTACGTAC\n")
    b = _job(tmp_path, "b", "r2.fa", ["z"], ">q\nACGTACGTAC\n")  # z missing: KeyError (job 1)
    c = _job(tmp_path, "c", "r1.fa", ["w"])  # w missing from r1.fa: KeyError (job 2, group of job 0)
    assert cli.main(_argv([a, b, c])) == 1
    err = capsys.readouterr().err
    assert "'z'" in err or "z not in" in err, err  # job 1's error, not job 2's (reported in job order)


def test_device_error_read_index_spans_groups(tmp_path, launches, capsys):
    calls, fake = launches
    fake.fail_at = 2  # the second group's launch
    a = _job(tmp_path, "a", "r1.fa", ["x", "y"], ">x\nACGTACGTAC\n>y\nACGTACGTAC\n")
    b = _job(tmp_path, "b", "r2.fa", ["z"], ">z\nACGTACGTAC\n")
    assert cli.main(_argv([a, b])) == 1
    assert calls == [[2], [1]]  # one launch per reads file, in order
    assert "read index 3" in capsys.readouterr().err  # 1 within the second launch + 2 reads before it


def test_missing_min_depth_factor_after_reading_everything(tmp_path, launches, capsys):
    calls, _ = launches
    a = _job(tmp_path, "a", "r1.fa", ["x"], ">x\nACGTACGTAC\n")
    b = _job(tmp_path, "b", "r2.fa", ["z"], ">q\nACGTACGTAC\n")  # an ingest error still wins (:253 before :338)
    assert cli.main(_argv([a, b], mdf=None)) == 1
    assert "KeyError" in capsys.readouterr().err and calls == []
    assert cli.main(_argv([a], mdf=None)) == 1
    assert "min_depth_factor is required" in capsys.readouterr().err and calls == []


def _interleaved(tmp_path):
    """jobs A (r1.fa, 2 reads), B (r2.fa, 1 read), C (r1.fa, 1 read): the
    launches are [A, C] then [B] (one per reads file), not job order."""
    a = _job(tmp_path, "a", "r1.fa", ["x", "y"], ">x\nACGTACGTAC\n>y\nACGTACGTAC\n>w\nACGTACGTAC\n")
    b = _job(tmp_path, "b", "r2.fa", ["z"], ">z\nACGTACGTAC\n")
    c = _job(tmp_path, "c", "r1.fa", ["w"])
    return [a, b, c]


def test_device_error_interleaved_jobs_job_order_index(tmp_path, launches, capsys):
    """A device error in job C (read 2 of the launch [A, C]) is reported at
    C's index in JOB order: len(A) + len(B) + 0 = 3."""
    calls, fake = launches
    fake.fail = {1: 2}
    assert cli.main(_argv(_interleaved(tmp_path))) == 1
    assert calls == [[2, 1], [1]]
    assert "read index 3" in capsys.readouterr().err


def test_device_error_earliest_job_wins(tmp_path, launches, capsys):
    """Errors in job C (launch 1) and job B (launch 2): B comes first in job
    order, so its read is reported (index len(A) + 0 = 2)."""
    calls, fake = launches
    fake.fail = {1: 2, 2: 0}
    assert cli.main(_argv(_interleaved(tmp_path))) == 1
    assert "read index 2" in capsys.readouterr().err
