"""GPU tests of the ingest layer (include/kc.h "Batching", kc_count_file,
kc_checkpoint / kc_rollback): pending batches across calls, flushes on a full
batch or a new read length, rollback, and the file reader's blocks (cut at
record boundaries, carried tails, dealt to several contexts). Every count is
compared bit-exactly with the CPU oracle."""
import os
import random
import subprocess

import pytest

import kmer_ref_py as kp

pytestmark = pytest.mark.gpu


def _fq(reads, quals=None, hdr=""):
    out = []
    for i, s in enumerate(reads):
        q = quals[i] if quals else "I" * len(s)
        out.append(f"@{hdr}r{i}\n{s}\n+\n{q}\n")
    return "".join(out).encode()


def _rand_reads(n, L, seed, n_rate=0.002):
    rng = random.Random(seed)
    return ["".join("N" if rng.random() < n_rate else rng.choice("ACGT") for _ in range(L)) for _ in range(n)]


def _quals_with_at(reads, seed):
    # quality strings that often start with '@' (Phred+33 Q31): the block cut
    # must not take a quality line for a header
    rng = random.Random(seed)
    return ["@" + "".join(rng.choice("!#@@@5?I") for _ in range(len(s) - 1)) for s in reads]


def test_small_chunks_count_as_batches(kca, orc):
    """Reference chunks of ~50 reads each through kc_count_chunk with a 4 MiB
    working set: the pending batch is counted whenever the next chunk does not
    fit (many flushes) and at kc_finish; same bytes as one chunk."""
    L, k = 150, 31
    fq = kca.synth_fastq(30000, L, seed=5, genome_length=400_000, n_rate=0.001)
    chunks = list(orc.chunks_of(fq, orc.chunk_size(L, k, 2_000_000)))
    assert len(chunks) > 20
    with kca.Context(kmer_length=k, line_length=L, gpu_memory_limit=4 << 20) as ctx:
        for chunk, ll in chunks:
            ctx.count_chunk(chunk, ll)
        got = ctx.records()
        st = ctx.stats()
    assert st["batches"] > 3
    assert got == orc.count_chunks(chunks, k)
    assert st["reads"] == 30000 and st["windows"] == 30000 * (L - k + 1)


def test_read_length_change_flushes(kca, orc):
    """Blocks of 100 bp then 150 bp then 100 bp reads: each change of L counts
    the pending batch first (its codes are laid out per L)."""
    k = 25
    blocks = [kca.synth_fastq(3000, 100, seed=1), kca.synth_fastq(2000, 150, seed=2, n_rate=0.01),
              kca.synth_fastq(1000, 100, seed=3)]
    with kca.Context(kmer_length=k, line_length=100) as ctx:
        for b in blocks:
            ctx.count_fastq(b, len(b.split(b"\n")[1]))
        got = ctx.records()
    want = orc.count_chunks([(c, ll) for b in blocks for c, ll in orc.chunks_of(b, 1 << 26)], k)
    assert got == want


def test_checkpoint_rollback(kca, orc):
    a = kca.synth_fastq(4000, 150, seed=7, n_rate=0.002)
    b = kca.synth_fastq(3000, 150, seed=8, n_rate=0.002)
    with kca.Context(kmer_length=31, line_length=150) as ctx:
        ctx.count_fastq(a)
        ctx.checkpoint()
        ctx.count_fastq(b)
        ctx.rollback()
        st = ctx.stats()
        assert st["reads"] == 4000
        got = ctx.records()
    assert got == orc.count_fastq(a, 31)


def test_rollback_after_a_counted_batch_is_refused(kca, orc):
    """A batch counted since the checkpoint (here: the read length changed)
    cannot be undone: KC_ERR_STATE, and the counts stand."""
    a = kca.synth_fastq(2000, 100, seed=9)
    b = kca.synth_fastq(2000, 150, seed=10)
    with kca.Context(kmer_length=31, line_length=100) as ctx:
        ctx.checkpoint()
        ctx.count_fastq(a, 100)
        ctx.count_fastq(b, 150)
        with pytest.raises(kca.KcError) as e:
            ctx.rollback()
        assert e.value.status == kca.KC_ERR_STATE
        got = ctx.records()
    assert got == orc.count_chunks(list(orc.chunks_of(a, 1 << 26)) + list(orc.chunks_of(b, 1 << 26)), 31)


def test_malformed_block_leaves_pending_batch_intact(kca, orc):
    good = kca.synth_fastq(3000, 120, seed=11, n_rate=0.003)
    bad = _fq(["ACGT" * 30] * 5 + ["ACG"])
    with kca.Context(kmer_length=21, line_length=120) as ctx:
        ctx.count_fastq(good)
        with pytest.raises(kca.KcError) as e:
            ctx.count_fastq(bad)
        assert e.value.status == kca.KC_ERR_FORMAT
        assert ctx.stats()["reads"] == 3000
        got = ctx.records()
    assert got == orc.count_fastq(good, 21)


def test_large_pageable_block_through_the_ring(kca, orc):
    """A ~100 MB host block (pageable) crosses several 64 MiB pinned slots."""
    fq = kca.synth_fastq(330_000, 150, seed=12, genome_length=3_000_000, n_rate=0.0005)
    assert len(fq) > 64 << 20
    with kca.Context(kmer_length=31, line_length=150, gpu_memory_limit=8 << 30) as ctx:
        assert ctx.count_fastq(fq) == 330_000
        got = ctx.records()
    want, _ = orc.refcpu(fq, 31, threads=8)
    assert got == want


@pytest.mark.parametrize("block", [4096, 65536, 1 << 20])
@pytest.mark.parametrize("mode", ["auto", "fastq"])
def test_count_file_blocks(kca, orc, tmp_path, monkeypatch, block, mode):
    """kc_count_file with small reader blocks (KC_FILE_BLOCK): every block is
    cut at a record start (quality lines starting with '@' included), its tail
    carried into the next; same bytes as the oracle."""
    monkeypatch.setenv("KC_FILE_BLOCK", str(block))
    reads = _rand_reads(4000, 90, seed=block)
    fq = _fq(reads, _quals_with_at(reads, block), hdr="h" * 40)
    p = tmp_path / "r.fq"
    p.write_bytes(fq)
    with kca.Context(kmer_length=21, line_length=90) as ctx:
        assert ctx.count_file(str(p), mode=mode) == 4000
        got = ctx.records()
    assert got == orc.count_fastq(fq, 21)


def test_count_file_exact_mode(kca, orc, tmp_path):
    fq = kca.synth_fastq(5000, 100, seed=13, n_rate=0.002)
    p = tmp_path / "r.fq"
    p.write_bytes(fq)
    with kca.Context(kmer_length=21, line_length=100, gpu_memory_limit=3_000_000) as ctx:
        ctx.count_file(str(p), mode="exact")
        got = ctx.records()
    assert got == orc.count_chunks(orc.chunks_of(fq, orc.chunk_size(100, 21, 3_000_000)), 21)


@pytest.mark.parametrize("where", [10, 2500, 3999])
def test_count_file_auto_falls_back_after_counting_blocks(kca, orc, tmp_path, monkeypatch, where):
    """A malformed record in a late block of a multi-block file: the blocks
    already decoded are rolled back and the whole file is counted in the
    reference's own chunks (header >= 2L: records lost at chunk edges, as the
    reference loses them)."""
    monkeypatch.setenv("KC_FILE_BLOCK", "65536")
    L = 40
    reads = _rand_reads(4000, L, seed=where)
    reads[where] = reads[where][:-3]  # a short read: not L-base records
    fq = _fq(reads, [("I" * len(s)) for s in reads], hdr="x" * 90)
    p = tmp_path / "r.fq"
    p.write_bytes(fq)
    with kca.Context(kmer_length=21, line_length=L, gpu_memory_limit=200_000) as ctx:
        ctx.count_fastq(kca.synth_fastq(500, L, seed=1))  # pending before the file: kept
        ctx.count_file(str(p), L, mode="auto")
        got = ctx.records()
    first = list(orc.chunks_of(kca.synth_fastq(500, L, seed=1), 1 << 26))
    want = orc.count_chunks(first + list(orc.chunks_of(fq, orc.chunk_size(L, 21, 200_000))), 21)
    assert got == want


def test_count_file_fastq_mode_rejects_malformed(kca, tmp_path):
    p = tmp_path / "r.fq"
    p.write_bytes(_fq(["ACGT" * 10] * 3) + b"@x\nAC\n+\nII\n")
    with kca.Context(kmer_length=21, line_length=40) as ctx:
        with pytest.raises(kca.KcError) as e:
            ctx.count_file(str(p), mode="fastq")
        assert e.value.status == kca.KC_ERR_FORMAT


def test_count_file_several_contexts(kca, orc, tmp_path, monkeypatch):
    """Blocks dealt to three contexts (read-shard); their sorted runs merged
    on the host equal one count of the file."""
    monkeypatch.setenv("KC_FILE_BLOCK", "262144")
    fq = kca.synth_fastq(20000, 150, seed=14, genome_length=500_000, n_rate=0.001)
    p = tmp_path / "r.fq"
    p.write_bytes(fq)
    ctxs = [kca.Context(kmer_length=31, line_length=150) for _ in range(3)]
    try:
        assert kca.count_file(ctxs, str(p)) == 20000
        runs = []
        for i, c in enumerate(ctxs):
            runs += c.write_runs(str(tmp_path / f"run{i}"))
        assert sum(c.stats()["reads"] for c in ctxs) == 20000
        assert sum(1 for c in ctxs if c.stats()["reads"] > 0) >= 2
    finally:
        for c in ctxs:
            c.close()
    out = tmp_path / "o.bin"
    kca.merge_files(runs, str(out), 31)
    assert out.read_bytes() == orc.count_fastq(fq, 31)


def test_count_file_variable_length(kca, orc, tmp_path, monkeypatch):
    monkeypatch.setenv("KC_FILE_BLOCK", "131072")
    rng = random.Random(3)
    reads = ["".join(rng.choice("ACGT") for _ in range(rng.randint(0, 160))) for _ in range(3000)]
    fq = _fq(reads)
    p = tmp_path / "r.fq"
    p.write_bytes(fq)
    with kca.Context(kmer_length=31, line_length=160, variable_length=True) as ctx:
        assert ctx.count_file(str(p)) == 3000
        got = ctx.records()
    assert got == orc.count_fastq_varlen(fq, 31)


def test_cli_streams_files_end_to_end(kca, orc, tmp_path):
    """The CLI over a directory of files (one malformed: counted in reference
    chunks) with small reader blocks."""
    d = tmp_path / "in"
    d.mkdir()
    texts = []
    for i in range(3):
        t = kca.synth_fastq(6000, 120, seed=60 + i, n_rate=0.001)
        (d / f"f{i}.fq").write_bytes(t)
        texts.append(t)
    bad = _fq(_rand_reads(300, 120, seed=4)) + b"\n"
    (d / "g.fq").write_bytes(bad)
    out = tmp_path / "o.bin"
    env = dict(os.environ, KC_FILE_BLOCK="200000")
    subprocess.run([kca.CLI_PATH, "kmerLength=27", f"inputFileLocation={d}", f"outputFile={out}",
                    f"tempFileLocation={tmp_path}", "quiet=1"], check=True, capture_output=True, env=env)
    lim = 100000000
    chunks = [(c, ll) for t in texts + [bad] for c, ll in orc.chunks_of(t, orc.chunk_size(120, 27, lim))]
    assert out.read_bytes() == orc.count_chunks(chunks, 27)


def test_write_output_at_offsets_after_exchange(kca, orc, tmp_path):
    """kc_write_output_at: after the in-process key-space exchange every
    context writes its key range at its offset of one pre-sized file; the file
    is the whole count."""
    shards = [kca.synth_fastq(2500, 150, 31 + r, n_rate=0.001, genome_length=80_000) for r in range(3)]
    ctxs = [kca.Context(kmer_length=31, line_length=150) for _ in shards]
    out = tmp_path / "o.bin"
    try:
        for c, fq in zip(ctxs, shards):
            c.count_fastq(fq)
            c.finish()
        kca.exchange_contexts(ctxs)
        sizes = [c.finish() * c.rs for c in ctxs]
        with open(out, "wb") as f:
            f.truncate(sum(sizes))
        for i in (2, 0, 1):
            ctxs[i].write_output_at(str(out), sum(sizes[:i]))
    finally:
        for c in ctxs:
            c.close()
    assert out.read_bytes() == orc.count_fastq(b"".join(shards), 31)


@pytest.mark.parametrize("k,mem", [(31, 100_000_000), (55, 1 << 20)])
def test_gather_contexts_merges_on_first_device(kca, orc, k, mem):
    """kc_gather_contexts (read-shard merge on one GPU): three contexts count
    shards (with a 1 MiB working set they also cut runs and spill), their runs
    are merged by merge path on the first context's device."""
    shards = [kca.synth_fastq(3000, 150, 70 + r, n_rate=0.001, genome_length=120_000) for r in range(3)]
    ctxs = [kca.Context(kmer_length=k, line_length=150, gpu_memory_limit=mem) for _ in shards]
    try:
        for c, fq in zip(ctxs, shards):
            c.count_fastq(fq)
            c.finish()
        kca.gather_contexts(ctxs)
        got = ctxs[0].records()
    finally:
        for c in ctxs:
            c.close()
    assert got == orc.count_fastq(b"".join(shards), k)


@pytest.mark.parametrize("mode", ["fastq", "auto"])
def test_count_file_blocks_larger_than_pending_room(kca, orc, tmp_path, monkeypatch, mode):
    """Reader blocks holding more reads than the pending batch takes (a 4 MiB
    working set, 1 MiB blocks of ~3300 reads): each block goes through the
    two-pass index and is encoded batch by batch straight from its staging
    buffer, asynchronously; the next upload into that buffer must wait for
    those encodes (stage_free). Same bytes as the oracle."""
    monkeypatch.setenv("KC_FILE_BLOCK", str(1 << 20))
    fq = kca.synth_fastq(40000, 150, seed=21, genome_length=2_000_000, n_rate=0.001)
    p = tmp_path / "r.fq"
    p.write_bytes(fq)
    with kca.Context(kmer_length=31, line_length=150, gpu_memory_limit=4 << 20) as ctx:
        assert ctx.count_file(str(p), mode=mode) == 40000
        got = ctx.records()
        st = ctx.stats()
    assert st["batches"] >= 4
    assert got == orc.count_fastq(fq, 31)


def test_rollback_forgets_accumulated_chunks(kca, orc):
    """kc_count_chunk bytes accumulated after a checkpoint are forgotten by
    kc_rollback together with the pending reads (include/kc.h)."""
    L, k = 150, 31
    a = kca.synth_fastq(3000, L, seed=22, n_rate=0.001)
    b = kca.synth_fastq(2000, L, seed=23, n_rate=0.001)
    ca = list(orc.chunks_of(a, orc.chunk_size(L, k, 2_000_000)))
    cb = list(orc.chunks_of(b, orc.chunk_size(L, k, 2_000_000)))
    with kca.Context(kmer_length=k, line_length=L) as ctx:
        for chunk, ll in ca:
            ctx.count_chunk(chunk, ll)
        ctx.checkpoint()
        for chunk, ll in cb:
            ctx.count_chunk(chunk, ll)
        ctx.rollback()
        assert ctx.stats()["reads"] == 3000
        got = ctx.records()
    assert got == orc.count_chunks(ca, k)


def test_check_fastq_has_no_side_effects(kca, orc):
    """kc_check_fastq validates a block without reserving, encoding or
    counting anything: a held checkpoint still rolls back, and the pending
    batch is the one counted."""
    a = kca.synth_fastq(3000, 150, seed=24, n_rate=0.002)
    b = kca.synth_fastq(50000, 150, seed=25, n_rate=0.002)
    with kca.Context(kmer_length=31, line_length=150, gpu_memory_limit=8 << 20) as ctx:
        ctx.count_fastq(a)
        ctx.checkpoint()
        assert ctx.check_fastq(b) == 50000
        ctx.rollback()
        st = ctx.stats()
        assert st["reads"] == 3000 and st["batches"] == 0
        got = ctx.records()
    assert got == orc.count_fastq(a, 31)
