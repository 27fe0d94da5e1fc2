"""Variable-length reads (KC_FLAG_VARLEN, CLI readLengths=variable; SURVEY §8f
row 1). The reference has no defined result for reads of different lengths:
FASTQFileReader::readData concatenates sequence lines without separators
(FASTQFileReader.cpp:57-79) and processKMers cuts the chunk at multiples of the
first read's length (GPUHandler.cu:13-15, 397-466). The extension counts every
read as a reference read of its own length: windows need k ACGT bases, key
bases past the read end read as 0, a read shorter than k counts nothing, and
key 0^W is present iff some window of some read is invalid.

Parity anchors: the C oracle run per read with L = the read's length
(oracle.count_fastq_varlen, the spec restatement of GPUHandler.cu:129-233) and
the pure-Python statement over strings (tests/kmer_ref_py.py), which agree on
the CPU tests here; the GPU tests compare the C-ABI output with both."""
import os
import random
import subprocess

import pytest

import kmer_ref_py as kr


def _varlen_fastq(n, lmin, lmax, seed, n_rate=0.01, genome=None, hdr=0):
    rng = random.Random(seed)
    recs = []
    for i in range(n):
        L = rng.randint(lmin, lmax)
        if genome is not None and L <= len(genome):
            p = rng.randrange(0, len(genome) - L + 1)
            s = list(genome[p:p + L])
        else:
            s = [rng.choice("ACGT") for _ in range(L)]
        for j in range(L):
            if rng.random() < n_rate:
                s[j] = rng.choice("NNNnRa")
        h = "x" * rng.randint(0, hdr)
        recs.append(f"@r{i}{h}\n{''.join(s)}\n+\n{'I' * L}\n")
    return "".join(recs).encode()


def _py(fq, k):
    return kr.to_bytes(kr.count_reads(kr.fastq_reads(fq.decode()), k), k)


# ---- CPU: the oracle's per-read form against the string statement ---------

@pytest.mark.parametrize("k,lmin,lmax", [(5, 0, 40), (21, 0, 130), (31, 10, 160), (33, 30, 100), (61, 50, 140)])
def test_oracle_varlen_matches_python(orc, k, lmin, lmax):
    fq = _varlen_fastq(300, lmin, lmax, seed=k * 31 + lmax, n_rate=0.02)
    assert orc.count_fastq_varlen(fq, k) == _py(fq, k)


def test_oracle_varlen_equals_fixed_when_lengths_equal(orc):
    fq = _varlen_fastq(500, 100, 100, seed=3)
    assert orc.count_fastq_varlen(fq, 21) == orc.count_fastq(fq, 21)


def test_oracle_varlen_zero_key_rule(orc):
    # a bad base only in reads shorter than k: no window, no hole
    fq = b"@a\nACGNA\n+\nIIIII\n@b\n" + b"ACGT" * 10 + b"\n+\n" + b"I" * 40 + b"\n"
    got = kr.parse_records(orc.count_fastq_varlen(fq, 21), 21)
    assert all(key != (0,) for key, _ in got)
    # the same base in a read of >= k bases: key 0 with count 0
    fq2 = fq + b"@c\n" + b"C" * 10 + b"N" + b"G" * 20 + b"\n+\n" + b"I" * 31 + b"\n"
    got2 = kr.parse_records(orc.count_fastq_varlen(fq2, 21), 21)
    assert got2[0] == ((0,), 0)


# ---- GPU -------------------------------------------------------------------

def _gpu(kca, fq, k, L, engine="auto", **kw):
    with kca.Context(kmer_length=k, line_length=L, engine=engine, variable_length=True, **kw) as ctx:
        n = ctx.count_fastq(fq, L)
        st = ctx.stats()
        return n, ctx.records(), st


@pytest.mark.gpu
@pytest.mark.parametrize("k,lmin,lmax", [(18, 0, 60), (21, 0, 130), (31, 0, 150), (31, 140, 151), (32, 20, 300),
                                         (55, 40, 150), (63, 60, 250), (100, 90, 200)])
@pytest.mark.parametrize("engine", ["auto", "partition"])
def test_varlen_gpu_matches_oracle(kca, orc, k, lmin, lmax, engine):
    fq = _varlen_fastq(4000, lmin, lmax, seed=k + lmax, n_rate=0.003)
    n, got, st = _gpu(kca, fq, k, lmax, engine=engine)
    seqs = orc.fastq_sequences(fq)
    assert n == len(seqs)
    want = orc.count_fastq_varlen(fq, k)
    assert got == want
    assert st["windows"] == sum(max(0, len(s) - k + 1) for s in seqs)


@pytest.mark.gpu
@pytest.mark.parametrize("k,lmin,lmax", [(31, 3000, 5000), (55, 4000, 6000)])
def test_varlen_gpu_reads_past_fused_index_limit(kca, orc, k, lmin, lmax):
    """Reads of > 4065 bases exceed the fused variable-length index's item
    range (list cap x 16-base groups < 2^16): those blocks take the two-pass
    index (fq_emit + encode_reads_var) instead of failing."""
    fq = _varlen_fastq(300, lmin, lmax, seed=k + lmax, n_rate=0.001)
    n, got, st = _gpu(kca, fq, k, lmax, engine="partition")
    assert n == 300
    assert got == orc.count_fastq_varlen(fq, k)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [21, 31])
def test_varlen_gpu_genome_reads_skm(kca, orc, k):
    # coverage (the super-k-mer engine's dedup path), trimmed reads
    rng = random.Random(k)
    genome = "".join(rng.choice("ACGT") for _ in range(200_000))
    fq = _varlen_fastq(60_000, 50, 150, seed=k, n_rate=0.0005, genome=genome)
    n, got, st = _gpu(kca, fq, k, 150, engine="skm")
    assert got == orc.count_fastq_varlen(fq, k)
    assert st["engines_used"] & 1


@pytest.mark.gpu
def test_varlen_gpu_small_python(kca):
    fq = _varlen_fastq(200, 0, 70, seed=5, n_rate=0.05)
    _, got, _ = _gpu(kca, fq, 27, 70)
    assert got == _py(fq, 27)


@pytest.mark.gpu
def test_varlen_gpu_fixed_lengths_equal_fixed_mode(kca, orc):
    fq = kca.synth_fastq(20000, 150, seed=11, genome_length=300_000, n_rate=0.001)
    _, got, _ = _gpu(kca, fq, 31, 150)
    assert got == orc.count_fastq(fq, 31)


@pytest.mark.gpu
def test_varlen_gpu_zero_key_rule(kca, orc):
    # bad bases only in reads shorter than k (and padding everywhere): no key 0
    fq = b"@a\nACGNA\n+\nIIIII\n@b\n" + b"ACGT" * 10 + b"\n+\n" + b"I" * 40 + b"\n@c\n\n+\n\n"
    _, got, _ = _gpu(kca, fq, 21, 40)
    assert got == orc.count_fastq_varlen(fq, 21)
    assert all(key != (0,) for key, _ in kr.parse_records(got, 21))
    # all reads shorter than k: nothing at all
    _, got, _ = _gpu(kca, b"@a\nACGT\n+\nIIII\n@b\nAC\n+\nII\n", 21, 21)
    assert got == b""


@pytest.mark.gpu
def test_varlen_gpu_read_longer_than_L_rejected(kca):
    fq = _varlen_fastq(100, 30, 80, seed=9)
    with kca.Context(kmer_length=21, line_length=60, variable_length=True) as ctx:
        with pytest.raises(kca.KcError) as e:
            ctx.count_fastq(fq, 60)
        assert e.value.status == 4  # KC_ERR_FORMAT, nothing counted
        ctx.count_fastq(_varlen_fastq(50, 21, 60, seed=10), 60)


@pytest.mark.gpu
def test_varlen_gpu_blocks_accumulate(kca, orc):
    a = _varlen_fastq(3000, 0, 150, seed=21, n_rate=0.01)
    b = _varlen_fastq(3000, 0, 120, seed=22, n_rate=0.0)
    with kca.Context(kmer_length=31, line_length=150, variable_length=True) as ctx:
        ctx.count_fastq(a, 150)
        ctx.count_fastq(b, 120)
        got = ctx.records()
    assert got == orc.count_fastq_varlen(a + b, 31)


@pytest.mark.gpu
def test_varlen_table_engine_rejected(kca):
    with pytest.raises(kca.KcError):
        kca.Context(kmer_length=21, line_length=100, engine="table", variable_length=True)


@pytest.mark.gpu
def test_varlen_cli(kca, orc, tmp_path):
    d = tmp_path / "in"
    d.mkdir()
    fa = _varlen_fastq(2000, 0, 150, seed=31, n_rate=0.005)
    fb = _varlen_fastq(2000, 10, 90, seed=32)
    (d / "a.fastq").write_bytes(fa)
    (d / "b.fastq").write_bytes(fb)
    out = tmp_path / "out.bin"
    cli = os.path.join(os.path.dirname(kca.LIB_PATH), "kmer-counter")
    subprocess.run([cli, "kmerLength=25", f"inputFileLocation={d}", f"outputFile={out}", f"tempFileLocation={tmp_path}",
                    "readLengths=variable", "quiet=1"], check=True, capture_output=True, timeout=300)
    assert out.read_bytes() == orc.count_fastq_varlen(fa + fb, 25)


def test_synth_varlen_generator(kca, orc):
    fixed = kca.synth_fastq(300, 120, 4, genome_length=10_000)
    var = kca.synth_fastq(300, 120, 4, genome_length=10_000, min_read_length=40)
    assert len(var) == len(fixed)  # headers absorb the trimmed bases
    seqs, fseqs = orc.fastq_sequences(var), orc.fastq_sequences(fixed)
    assert all(40 <= len(s) <= 120 for s in seqs) and len({len(s) for s in seqs}) > 20
    assert all(f.startswith(s) for s, f in zip(seqs, fseqs))  # a read keeps its first bases


@pytest.mark.gpu
def test_varlen_gpu_synth_device(kca, orc):
    host = kca.synth_fastq(20000, 150, 6, genome_length=400_000, min_read_length=50)
    with kca.Context(kmer_length=31, line_length=150, variable_length=True) as ctx:
        ptr, n = ctx.synth_device(20000, 150, 6, 400_000, 0.0, 0, 50)
        assert ctx.copy_to_host(ptr, n) == host
        ctx.count_fastq_device(ptr, n, 150)
        got = ctx.records()
        ctx.free_device(ptr)
    assert got == orc.count_fastq_varlen(host, 31)


@pytest.mark.gpu
@pytest.mark.parametrize("k,lmin,lmax,hdr", [(31, 0, 150, 0), (31, 100, 150, 60), (9, 0, 12, 0), (21, 0, 24, 0), (19, 0, 40, 300),
                                             (25, 200, 1500, 5), (55, 0, 150, 20)])
def test_varlen_fused_matches_two_pass(kca, orc, monkeypatch, k, lmin, lmax, hdr):
    # the fused index (fq_encode_k<true>: per-half record lists, sequence ends
    # found past the staged KiB for long reads, dense halves falling back to
    # the two-pass index) against the two-pass one (fq_emit_k +
    # encode_reads_var_k) and the oracle
    fq = _varlen_fastq(max(200, 1_500_000 // (lmax + lmin + hdr + 20)), lmin, lmax, seed=k + lmax + hdr,
                       n_rate=0.004, hdr=hdr)
    monkeypatch.delenv("KC_NO_FQ_ENCODE", raising=False)
    n1, got, st1 = _gpu(kca, fq, k, lmax)
    monkeypatch.setenv("KC_NO_FQ_ENCODE", "1")
    n2, ref, st2 = _gpu(kca, fq, k, lmax)
    assert n1 == n2
    assert got == ref == orc.count_fastq_varlen(fq, k)
    assert st1["windows"] == st2["windows"]


@pytest.mark.gpu
def test_varlen_fused_rejects_long_and_malformed(kca):
    good = _varlen_fastq(3000, 20, 100, seed=41)
    bad_len = _varlen_fastq(3000, 20, 120, seed=41)
    with kca.Context(kmer_length=21, line_length=100, variable_length=True) as ctx:
        with pytest.raises(kca.KcError) as e:
            ctx.count_fastq(bad_len, 100)  # reads longer than the slot
        assert e.value.status == 4
        recs = good.split(b"\n")
        recs[4 * 1500 + 2] = b"-"  # no '+' line after a sequence
        with pytest.raises(kca.KcError) as e:
            ctx.count_fastq(b"\n".join(recs), 100)
        assert e.value.status == 4
        assert ctx.count_fastq(good, 100) == 3000


@pytest.mark.gpu
@pytest.mark.parametrize("exchange", ["alltoall", "none"])
def test_varlen_cli_two_contexts(kca, orc, tmp_path, exchange):
    # blocks dealt to two contexts (key-space exchange or run merge), each
    # counting variable-length reads
    d = tmp_path / "in"
    d.mkdir()
    fa = _varlen_fastq(3000, 0, 150, seed=51, n_rate=0.005)
    fb = _varlen_fastq(3000, 20, 120, seed=52)
    (d / "a.fastq").write_bytes(fa)
    (d / "b.fastq").write_bytes(fb)
    out = tmp_path / "out.bin"
    cli = os.path.join(os.path.dirname(kca.LIB_PATH), "kmer-counter")
    subprocess.run([cli, "kmerLength=31", f"inputFileLocation={d}", f"outputFile={out}", f"tempFileLocation={tmp_path}",
                    "readLengths=variable", "gpus=2", f"exchange={exchange}", "quiet=1"],
                   check=True, capture_output=True, timeout=300)
    assert out.read_bytes() == orc.count_fastq_varlen(fa + fb, 31)
