"""Rule `revcomp_antisense_consensus` (reference Snakefile:425-450, table :77),
restated as writers.revcomp_text / revcomp_consensus.  Known answers derived
from the rule's text: header lines copied, the LAST line reversed and
complemented (upper-cased first), no trailing newline, KeyError on anything
outside A/C/G/T/N (after the headers were written).  CPU only."""
import importlib

import pytest

import golden_util as gu

W = importlib.import_module("minion-plasmid-consensus_amd.writers")

KNOWN = [
    ([">consensus\n", "ACGTN\n"], ">consensus\nNACGT"),
    ([">consensus\n", "acgtt\n"], ">consensus\nAACGT"),  # x.upper() before the lookup
    ([">consensus\n", "\n"], ">consensus\n"),  # empty consensus
    ([">consensus\n", "AAAA  \n"], ">consensus\nTTTT"),  # rstrip
    ([">a\n", "GG\n", ">b\n", "CCA\n"], ">a\n>b\nTGG"),  # only the last line is used (:445)
    ([">a\n", "GG\n", "TTA"], ">a\nTAA"),  # multi-line record: still only the last line
    (["ACG\n"], "CGT"),  # no header
]
ERRORS = [
    ([">consensus\n", "ACXT\n"], ">consensus\n"),  # 'X' is not in the table
    ([">consensus\n"], ">consensus\n"),  # last line is the header: '>' reversed last -> KeyError 'S'
    ([], ""),  # empty file: the loop variable is unbound
]


@pytest.mark.parametrize("lines,expected", KNOWN)
def test_known_answers(lines, expected):
    assert W.revcomp_text(lines) == (expected, None)


@pytest.mark.parametrize("lines,partial", ERRORS)
def test_rule_errors(lines, partial):
    text, err = W.revcomp_text(lines)
    assert text == partial and isinstance(err, W.RevcompError)


@pytest.mark.parametrize("case", [c for c in gu.cases() if c.endswith("_antisense")])
def test_golden_consensus_files(case, tmp_path):
    for k, run, exp in gu.runs(case):
        if run["exit"] != 0:
            continue
        src, dst = tmp_path / f"c{k}.fa", tmp_path / f"rc{k}.fa"
        src.write_bytes(exp["c.fa"])
        W.revcomp_consensus(str(src), str(dst))
        seq = exp["c.fa"].decode().split("\n")[1]
        comp = {"A": "T", "T": "A", "C": "G", "G": "C", "N": "N"}
        assert dst.read_text() == ">consensus\n" + "".join(comp[b] for b in reversed(seq))


def test_file_error_leaves_header(tmp_path):
    src, dst = tmp_path / "c.fa", tmp_path / "rc.fa"
    src.write_text(">consensus\nAXA\n")
    with pytest.raises(W.RevcompError):
        W.revcomp_consensus(str(src), str(dst))
    assert dst.read_text() == ">consensus\n"
