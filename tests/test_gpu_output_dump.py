"""CLI outputFormat=dump: the record layout of the
reference's active output path, KMerCounter::DumpResults
(KMerCounter.cpp:91-106), which writes key word 0 (8 B LE) and the count
(4 B LE) of every distinct key of the host hash. Checked against the oracle's
sorted output with each record cut to word 0 + count (the reference's TBB hash
order is not reproducible, so records stay in key order). Needs an MI355X."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu


def _truncate(sorted_bytes, k):
    W = (k + 31) // 32
    rs = 8 * W + 4
    out = bytearray()
    for i in range(0, len(sorted_bytes), rs):
        out += sorted_bytes[i:i + 8] + sorted_bytes[i + 8 * W:i + rs]
    return bytes(out)


@pytest.mark.parametrize("k", [21, 31, 55, 100])
def test_cli_dump_format(kca, orc, tmp_path, k):
    d = tmp_path / "in"
    d.mkdir()
    fq = kca.synth_fastq(3000, 150, seed=k, n_rate=0.002)
    (d / "a.fastq").write_bytes(fq)
    cli = os.path.join(os.path.dirname(kca.LIB_PATH), "kmer-counter")
    outs = {}
    for fmt in ("sorted", "dump"):
        out = tmp_path / f"{fmt}.bin"
        subprocess.run([cli, f"kmerLength={k}", f"inputFileLocation={d}", f"outputFile={out}",
                        f"tempFileLocation={tmp_path}", f"outputFormat={fmt}", "quiet=1"],
                       check=True, capture_output=True, timeout=300)
        outs[fmt] = out.read_bytes()
    want = orc.count_fastq(fq, k)
    assert outs["sorted"] == want
    assert outs["dump"] == _truncate(want, k)
    if k <= 32:
        assert outs["dump"] == outs["sorted"]
