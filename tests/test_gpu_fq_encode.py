"""GPU parity of the FASTQ index + encode passes against each other and the
CPU oracle: the fused index after fq_count_k (fq_encode_k, one text read for
K1 emit + E; the default) and the two-pass path (fq_emit_k + fq_validate_k +
encode_reads_k, KC_NO_FQ_ENCODE=1): identical
SortedKMerFile bytes on well-formed blocks whose records straddle the kernel's
8 KiB halves and 16 KiB chunks (headers of 1..400 bytes, reads of 18..3000
bases: past the staged KiB the groups come from global memory), and the same
KC_ERR_FORMAT verdict on every malformed block. Needs an MI355X."""
import random

import pytest

pytestmark = pytest.mark.gpu


def _block(n, L, seed, n_rate=0.01, hdr_max=60):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        h = "r" + "x" * rng.randrange(0, hdr_max) + str(i)
        s = "".join("N" if rng.random() < n_rate else rng.choice("ACGT") for _ in range(L))
        q = "I" * L
        out.append(f"@{h}\n{s}\n+\n{q}\n")
    return out


MODES = ("fused", "twopass")


def _count(kca, fq, k, L, mode, monkeypatch, engine="auto"):
    if mode is True:
        mode = "fused"
    elif mode is False:
        mode = "twopass"
    monkeypatch.delenv("KC_NO_FQ_ENCODE", raising=False)
    if mode == "twopass":
        monkeypatch.setenv("KC_NO_FQ_ENCODE", "1")
    with kca.Context(kmer_length=k, line_length=L, engine=engine) as ctx:
        n = ctx.count_fastq(fq)
        return n, ctx.records()


@pytest.mark.parametrize("k,L,hdr", [(18, 20, 5), (21, 100, 60), (31, 150, 400), (31, 151, 1), (55, 150, 30),
                                     (31, 1000, 20), (31, 3000, 200), (63, 250, 90)])
def test_fused_matches_two_pass_and_oracle(kca, orc, monkeypatch, k, L, hdr):
    n = max(50, 600_000 // (2 * L + hdr))
    fq = "".join(_block(n, L, seed=k * 7 + L, hdr_max=hdr)).encode()
    want = orc.count_fastq(fq, k)
    for mode in MODES:
        assert _count(kca, fq, k, L, mode, monkeypatch) == (n, want), mode


@pytest.mark.parametrize("n", [1, 2, 7, 51, 52, 53, 3000, 61000])
def test_fused_index_block_sizes(kca, orc, monkeypatch, n):
    """Blocks from one record (one chunk, one half) to ~1,200 chunks: a block
    ending inside a chunk's first half or right at a chunk edge."""
    fq = kca.synth_fastq(n, 150, seed=40 + n, genome_length=200_000, n_rate=0.001)
    want = orc.count_fastq(fq, 31)
    for mode in MODES:
        assert _count(kca, fq, 31, 150, mode, monkeypatch) == (n, want), mode


@pytest.mark.parametrize("engine", ["skm", "partition"])
def test_fused_engines(kca, orc, monkeypatch, engine):
    fq = kca.synth_fastq(30000, 150, seed=13, genome_length=500_000, n_rate=0.001)
    n, got = _count(kca, fq, 31, 150, True, monkeypatch, engine=engine)
    assert n == 30000
    assert got == orc.count_fastq(fq, 31)


def _mutations():
    # (name, function of the record list -> text); the damaged record sits in
    # the middle of a block that spans several chunks
    def seq_short(r, i):
        h, s, p, q, _ = r[i].split("\n")
        r[i] = f"{h}\n{s[:-1]}\n{p}\n{q}\n"

    def seq_long(r, i):
        h, s, p, q, _ = r[i].split("\n")
        r[i] = f"{h}\n{s}A\n{p}\n{q}\n"

    def no_plus(r, i):
        r[i] = r[i].replace("\n+\n", "\n-\n")

    def no_at(r, i):
        r[i] = "#" + r[i][1:]

    def seq_and_qual_short(r, i):
        h, s, p, q, _ = r[i].split("\n")
        r[i] = f"{h}\n{s[:-3]}\n{p}\n{q[:-3]}\n"

    def newline_in_seq(r, i):
        # the sequence split into two lines and the next header dropped: the
        # line count stays a multiple of 4, the records do not
        h, s, p, q, _ = r[i].split("\n")
        r[i] = f"{h}\n{s[:40]}\n{s[40:]}\n{p}\n{q}\n"
        r[i + 1] = r[i + 1].split("\n", 1)[1]

    def long_seq_short_next(r, i):
        # one base moved from read i + 1 to read i: the line count stays a multiple of 4
        h, s, p, q, _ = r[i].split("\n")
        r[i] = f"{h}\n{s}C\n{p}\n{q}\n"
        h, s, p, q, _ = r[i + 1].split("\n")
        r[i + 1] = f"{h}\n{s[1:]}\n{p}\n{q}\n"

    return {"seq_short": seq_short, "seq_long": seq_long, "no_plus": no_plus, "no_at": no_at,
            "seq_and_qual_short": seq_and_qual_short, "newline_in_seq": newline_in_seq,
            "long_seq_short_next": long_seq_short_next}


@pytest.mark.parametrize("name", sorted(_mutations()))
@pytest.mark.parametrize("at", [0, 37, 1500, -1])
def test_fused_rejects_like_two_pass(kca, monkeypatch, name, at):
    L, k = 150, 31
    recs = _block(2000, L, seed=3, hdr_max=80)
    i = at if at >= 0 else len(recs) - 3
    _mutations()[name](recs, i)
    fq = "".join(recs).encode()
    verdict = []
    for mode in MODES:
        try:
            _count(kca, fq, k, L, mode, monkeypatch)
            verdict.append("ok")
        except kca.KcError as e:
            verdict.append(e.status)
    assert verdict == [kca.KC_ERR_FORMAT] * len(MODES)


def test_fused_no_final_newline_and_empty_tail(kca, monkeypatch):
    recs = _block(500, 150, seed=4)
    fq = "".join(recs).encode()
    for mode in MODES:
        with pytest.raises(kca.KcError):
            _count(kca, fq[:-1], 31, 150, mode, monkeypatch)
    n, got = _count(kca, fq, 31, 150, True, monkeypatch)
    assert n == 500
