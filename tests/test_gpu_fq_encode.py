"""GPU parity of the FASTQ index + encode passes against each other and the
CPU oracle: the one-pass index (fq_encode_k<false, true>: each chunk guesses
its line phase, rows per chunk, checked against the scanned newline counts;
the default), the fused index after fq_count_k (fq_encode_k, KC_NO_FQ_SPEC=1)
and the two-pass path (fq_emit_k + fq_validate_k + encode_reads_k,
KC_NO_FQ_ENCODE=1): identical
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


MODES = ("onepass", "fused", "twopass")


def _set_mode(monkeypatch, mode):
    monkeypatch.delenv("KC_NO_FQ_ENCODE", raising=False)
    monkeypatch.delenv("KC_NO_FQ_SPEC", raising=False)
    if mode == "twopass":
        monkeypatch.setenv("KC_NO_FQ_ENCODE", "1")
    elif mode == "fused":
        monkeypatch.setenv("KC_NO_FQ_SPEC", "1")


def _count(kca, fq, k, L, mode, monkeypatch, engine="auto"):
    if mode is True:
        mode = "onepass"
    elif mode is False:
        mode = "twopass"
    _set_mode(monkeypatch, mode)
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


@pytest.mark.parametrize("mode", ["onepass", "fused"])
@pytest.mark.parametrize("engine", ["skm", "partition"])
def test_fused_engines(kca, orc, monkeypatch, engine, mode):
    fq = kca.synth_fastq(30000, 150, seed=13, genome_length=500_000, n_rate=0.001)
    n, got = _count(kca, fq, 31, 150, mode, monkeypatch, engine=engine)
    assert n == 30000
    assert got == orc.count_fastq(fq, 31)


def _onepass_missed(capfd):
    return "one-pass FASTQ index missed" in capfd.readouterr().err


@pytest.mark.parametrize("k", [21, 31])
def test_onepass_guess_miss_falls_back(kca, orc, monkeypatch, capfd, k):
    """Headers of ~5 KiB leave chunks whose first 4 KiB hold fewer than the
    newlines the phase guess needs: the guess misses, the verify kernel flags
    the block and the two-kernel index counts it (same records as the oracle).
    With short headers the one-pass index takes the block."""
    monkeypatch.setenv("KC_DEBUG", "1")
    L = 150
    rng = random.Random(k)
    recs = [f"@{'h' * rng.randrange(4800, 5400)}{i}\n" + "".join(rng.choice("ACGT") for _ in range(L)) +
            "\n+\n" + "I" * L + "\n" for i in range(300)]
    fq = "".join(recs).encode()
    capfd.readouterr()
    assert _count(kca, fq, k, L, "onepass", monkeypatch) == (300, orc.count_fastq(fq, k))
    assert _onepass_missed(capfd)
    fq2 = "".join(_block(4000, L, seed=k, hdr_max=40)).encode()
    assert _count(kca, fq2, k, L, "onepass", monkeypatch) == (4000, orc.count_fastq(fq2, k))
    assert not _onepass_missed(capfd)


@pytest.mark.parametrize("engine", ["auto", "skm", "partition"])
@pytest.mark.parametrize("kind", ["clean", "n_base", "all_a"])
def test_onepass_key0_presence(kca, orc, monkeypatch, engine, kind):
    """Key 0 (all-A) in the output iff a read holds a not-ACGT base (count 0
    unless all-A windows were counted) or an all-A window exists: the one-pass
    rows past each chunk's records are no reads, whatever the engine makes of
    them (the skm front end skips them, the key-prefix engine reads them as
    bases that are not ACGT and key 0's presence is recomputed at the flush)."""
    L, k = 150, 31
    rng = random.Random(hash(kind) & 0xffff)
    seqs = ["".join(rng.choice("CGT") for _ in range(L)) for _ in range(3000)]
    if kind == "n_base":
        seqs[1234] = seqs[1234][:70] + "N" + seqs[1234][71:]
    elif kind == "all_a":
        seqs[77] = "A" * 40 + seqs[77][40:]
    fq = "".join(f"@r{i}\n{s}\n+\n{'I' * L}\n" for i, s in enumerate(seqs)).encode()
    want = orc.count_fastq(fq, k)
    got = {}
    for mode in MODES:
        got[mode] = _count(kca, fq, k, L, mode, monkeypatch, engine=engine)
        assert got[mode] == (3000, want), mode


@pytest.mark.parametrize("k,used", [(31, True), (19, True), (18, False), (33, False), (55, False)])
def test_onepass_only_for_the_f3_front_end(kca, orc, monkeypatch, capfd, k, used):
    """The one-pass index runs where the skm engine's F3 front end reads the
    rows (k in [19, 32]); other k take the two-kernel index (a guess miss shows
    which one ran: it is reported only by the one-pass index)."""
    monkeypatch.setenv("KC_DEBUG", "1")
    L = 150
    rng = random.Random(k)
    recs = [f"@{'h' * 5000}{i}\n" + "".join(rng.choice("ACGT") for _ in range(L)) + "\n+\n" + "I" * L + "\n"
            for i in range(100)]
    fq = "".join(recs).encode()
    capfd.readouterr()
    assert _count(kca, fq, k, L, "onepass", monkeypatch) == (100, orc.count_fastq(fq, k))
    assert _onepass_missed(capfd) == used


@pytest.mark.parametrize("first,rest,missed", [(60, (58, 62), False), (8, (1, 12), False), (300, (1, 3), True)])
def test_onepass_rows_per_chunk_from_first_header(kca, orc, monkeypatch, capfd, first, rest, missed):
    """Rows per chunk are sized from the block's first header (less a
    16-character margin): uniform long headers take the one-pass index with
    fewer empty rows; a block whose later headers are much shorter than its
    first overfills a chunk's rows and is re-indexed by the two-kernel path.
    Either way the same records as the oracle."""
    monkeypatch.setenv("KC_DEBUG", "1")
    L, k = 150, 31
    rng = random.Random(first)
    recs = []
    for i in range(6000):
        hl = first if i == 0 else rng.randrange(rest[0], rest[1] + 1)
        h = ("r" + str(i) + "x" * hl)[:hl] if hl > 0 else ""
        recs.append(f"@{h}\n" + "".join(rng.choice("ACGT") for _ in range(L)) + "\n+\n" + "I" * L + "\n")
    fq = "".join(recs).encode()
    capfd.readouterr()
    assert _count(kca, fq, k, L, "onepass", monkeypatch) == (6000, orc.count_fastq(fq, k))
    assert _onepass_missed(capfd) == missed


def test_onepass_rows_through_the_key_prefix_engine(kca, orc, monkeypatch):
    """iid reads at k = 31 (no coverage): the one-pass rows are indexed for
    F3, then the coverage sketch hands the batch to the key-prefix engine,
    whose front end skips the empty rows; key 0 follows the reads."""
    _set_mode(monkeypatch, "onepass")
    L, k, n = 150, 31, 150_000  # >= 2^24 windows: the sketch runs
    fq = kca.synth_fastq(n, L, seed=91, genome_length=0, n_rate=0.0005)
    with kca.Context(kmer_length=k, line_length=L, gpu_memory_limit=8 << 30) as ctx:
        assert ctx.count_fastq(fq) == n
        got = ctx.records()
        st = ctx.stats()
    assert st["engines_used"] == 2, st["engines_used"]
    assert got == orc.count_fastq(fq, k)


def test_onepass_mixed_pending_batch(kca, orc, monkeypatch, capfd):
    """One pending batch of one-pass rows and rows of other producers (a block
    whose phase guess misses, reference chunks, a second one-pass block),
    counted together at kc_finish: the same records as the oracle over the
    concatenated input."""
    monkeypatch.setenv("KC_DEBUG", "1")
    _set_mode(monkeypatch, "onepass")
    L, k = 150, 31
    rng = random.Random(5)
    a = "".join(_block(3000, L, seed=21, n_rate=0.002)).encode()
    long_hdr = "".join(f"@{'h' * 5000}{i}\n" + "".join(rng.choice("ACGT") for _ in range(L)) + "\n+\n" + "I" * L +
                       "\n" for i in range(200)).encode()
    c = "".join(_block(2500, L, seed=22, n_rate=0.0)).encode()
    chunk_reads = [("".join(rng.choice("ACGN") for _ in range(L))) for _ in range(500)]
    chunk = "".join(chunk_reads).encode()
    with kca.Context(kmer_length=k, line_length=L) as ctx:
        ctx.count_fastq(a)
        ctx.count_fastq(long_hdr)
        ctx.count_chunk(chunk, L)
        ctx.count_fastq(c)
        got = ctx.records()
    assert _onepass_missed(capfd)
    fq_chunk = "".join(f"@c{i}\n{s}\n+\n{'I' * L}\n" for i, s in enumerate(chunk_reads)).encode()
    assert got == orc.count_fastq(a + long_hdr + fq_chunk + c, k)


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
