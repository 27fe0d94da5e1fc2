"""GPU parity of the super-k-mer engine (engine="skm", kc_skm.inl) against the
CPU oracle, bit-exact SortedKMerFile bytes, on the shapes that reach its
special paths: the grouped finish (>= 65536 records), P5 sub-range passes,
several batches, the pool-overflow retry, runs longer than nmax (tandem
repeats keep one minimizer), prefix skew beyond the segment sort, and every
record width (W = 1..3, K' = k or 32W). Needs an MI355X."""
import os
import random
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def _fq(reads):
    return "".join(f"@r{i}\n{s}\n+\n{'I' * len(s)}\n" for i, s in enumerate(reads)).encode()


@pytest.mark.parametrize("k,L", [(18, 60), (19, 100), (21, 100), (28, 150), (29, 150), (31, 150), (32, 150),
                                 (33, 150), (55, 150), (60, 150), (64, 150), (65, 160), (96, 150)])
def test_skm_grouped_finish(kca, orc, k, L):
    n = 4_000_000 // L
    fq = kca.synth_fastq(n, L, seed=100 + k, n_rate=0.001)
    with kca.Context(kmer_length=k, line_length=L, engine="skm") as ctx:
        assert ctx.count_fastq(fq) == n
        got = ctx.records()
        st = ctx.stats()
    assert st["output_records"] >= 65536
    assert got == orc.count_fastq(fq, k)


@pytest.mark.parametrize("k,slots", [(31, 64), (31, 256), (55, 64), (96, 128)])
def test_skm_subrange_passes(kca, orc, k, slots):
    fq = kca.synth_fastq(30000, 150, seed=k + slots, n_rate=0.0005)
    with kca.Context(kmer_length=k, line_length=150, lds_slots=slots, engine="skm") as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
        st = ctx.stats()
    assert got == orc.count_fastq(fq, k)
    assert st["spilled_kmers"] == 0


@pytest.mark.parametrize("k", [31, 55])
def test_skm_many_batches(kca, orc, k):
    fq = kca.synth_fastq(60000, 150, seed=21, genome_length=300_000, n_rate=0.0005)
    with kca.Context(kmer_length=k, line_length=150, gpu_memory_limit=1 << 21, engine="skm") as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
        st = ctx.stats()
    assert st["batches"] > 3
    assert got == orc.count_fastq(fq, k)


def test_skm_large_batch_one_run(kca, orc, monkeypatch):
    """While the global table is empty a skm batch may hold more than key_cap
    windows (up to the record pool at nw / 4 records per read): 30000 reads
    with a 44 MB working set (~19900 reads per safe batch) are one batch, so
    the finish sorts one run; same bytes as two safe batches and the oracle."""
    fq = kca.synth_fastq(30000, 150, seed=41, genome_length=500_000, n_rate=0.001)
    outs, sts = [], []
    for safe in (False, True):
        if safe:
            monkeypatch.setenv("KC_SKM_SAFE_BATCH", "1")
        with kca.Context(kmer_length=31, line_length=150, gpu_memory_limit=44_000_000, engine="skm") as ctx:
            ctx.count_fastq(fq)
            outs.append(ctx.records())
            sts.append(ctx.stats())
    assert sts[0]["batches"] == 1 and sts[1]["batches"] == 2
    assert outs[0] == outs[1] == orc.count_fastq(fq, 31)


def test_skm_large_batch_spill_overflow_retried(kca, orc, tmp_path, monkeypatch, capfd):
    """A large first batch (twice the safe size) whose spills overflow the
    spill buffer (1-slot LDS table, 1 MiB working set: nearly every key goes
    to the small global table, then to the spill buffer) is undone - table
    cleared, records and statistics restored - and counted in safe batches."""
    monkeypatch.setenv("KC_DEBUG", "1")
    fq = kca.synth_fastq(20000, 150, seed=35, genome_length=60_000)
    with kca.Context(kmer_length=31, line_length=150, gpu_memory_limit=1 << 20, engine="skm", lds_slots=1) as ctx:
        ctx.count_fastq(fq)
        got = ctx.output_bytes(str(tmp_path))
        st = ctx.stats()
    assert "overflowed the spill buffer: retried" in capfd.readouterr().err
    assert st["spilled_kmers"] > 0
    assert got == orc.count_fastq(fq, 31)


def test_skm_large_batch_record_overflow_retried(kca, orc, monkeypatch, capfd):
    """A large first batch (more reads than key_cap windows allow, taken while
    the global table is empty) whose P5 records overflow the record buffer is
    undone and counted in safe batches, instead of growing the buffer to the
    batch's window count (which can be far past gpu_memory_limit).
    KC_P5_REC_BOUND forces the overflow; the counts stay exact and the
    statistics count the kept work once."""
    monkeypatch.setenv("KC_DEBUG", "1")
    monkeypatch.setenv("KC_P5_REC_BOUND", "5000")
    n, L, k = 80000, 150, 31
    fq = kca.synth_fastq(n, L, seed=36, genome_length=400_000, n_rate=0.0005)
    with kca.Context(kmer_length=k, line_length=L, gpu_memory_limit=64 << 20, engine="skm") as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
        st = ctx.stats()
    err = capfd.readouterr().err
    assert "overflowed the record buffer: retried" in err
    assert st["batches"] >= 2 and st["windows"] == n * (L - k + 1)
    rs = 8 * ((k + 31) // 32) + 4
    assert st["valid_kmers"] == sum(int.from_bytes(got[i + rs - 4:i + rs], "little") for i in range(0, len(got), rs))
    assert got == orc.count_fastq(fq, k)


def test_test_hooks_ignored_without_switch(kca, orc, tmp_path):
    """The path-selecting variables are test hooks: without KC_TEST_HOOKS=1
    the library ignores them (a production caller cannot meet them by
    accident). Run in a child process: KC_SKM_POOL_CAP would force pool
    overflow retries (several batches) if it were honoured."""
    fq = kca.synth_fastq(20000, 150, seed=5, n_rate=0.002)
    p = tmp_path / "in.fq"
    p.write_bytes(fq)
    code = (
        "import importlib.util, json, sys\n"
        f"spec = importlib.util.spec_from_file_location('kca', {kca.__file__!r})\n"
        "m = importlib.util.module_from_spec(spec); spec.loader.exec_module(m)\n"
        f"fq = open({str(p)!r}, 'rb').read()\n"
        "with m.Context(kmer_length=31, line_length=150, engine='skm') as c:\n"
        "    c.count_fastq(fq); sys.stdout.buffer.write(c.records()); sys.stderr.write(str(c.stats()['batches']))\n")
    env = {kk: v for kk, v in os.environ.items() if kk != "KC_TEST_HOOKS"}
    env["KC_SKM_POOL_CAP"] = "20000"
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, check=True, timeout=300)
    assert r.stderr.decode().strip().splitlines()[-1] == "1"
    assert r.stdout == orc.count_fastq(fq, 31)


@pytest.mark.parametrize("cap,k", [(20000, 31), (20001, 31), (20007, 55)])
def test_skm_pool_overflow_retry(kca, orc, monkeypatch, cap, k):
    """A pool smaller than one batch's records: the batch is undone and
    retried with fewer reads until it fits; statistics are not double counted.
    Odd pool capacities put F's first-pass digit bytes at an offset that is
    not a multiple of 16 before rounding (the histogram's 16-byte loads)."""
    monkeypatch.setenv("KC_SKM_POOL_CAP", str(cap))
    fq = kca.synth_fastq(20000, 150, seed=5, n_rate=0.002)
    with kca.Context(kmer_length=k, line_length=150, engine="skm") as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
        st = ctx.stats()
    assert st["batches"] > 1
    rs = 8 * ((k + 31) // 32) + 4
    assert st["valid_kmers"] == sum(int.from_bytes(got[i + rs - 4:i + rs], "little") for i in range(0, len(got), rs))
    assert got == orc.count_fastq(fq, k)


@pytest.mark.parametrize("k", [19, 31, 55])
def test_skm_tandem_repeats_split_long_runs(kca, orc, k):
    """Tandem repeats keep one minimizer value across many windows, so runs
    exceed nmax and are split into several records."""
    rng = random.Random(k)
    reads = []
    for i in range(3000):
        unit = "".join(rng.choice("ACGT") for _ in range(rng.choice([1, 2, 3, 5, 7])))
        s = (unit * 200)[:150]
        if i % 3 == 0:
            s = s[:70] + "".join(rng.choice("ACGT") for _ in range(80))
        reads.append(s)
    fq = _fq(reads)
    with kca.Context(kmer_length=k, line_length=150, engine="skm") as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
    assert got == orc.count_fastq(fq, k)


@pytest.mark.parametrize("k", [31, 55])
def test_skm_prefix_skew_falls_back_to_radix(kca, orc, k):
    """Every read starts with the same 8 bases: > seg_sort capacity distinct
    keys share one 16-bit prefix, so the finish takes the radix sort."""
    rng = random.Random(7 * k)
    reads = ["ACGTACGA" + "".join(rng.choice("ACGT") for _ in range(142)) for _ in range(30000)]
    fq = _fq(reads)
    with kca.Context(kmer_length=k, line_length=150, engine="skm") as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
    assert got == orc.count_fastq(fq, k)


def test_skm_genome_reads_multi_block(kca, orc):
    blocks = [kca.synth_fastq(40000, 150, seed=2, genome_length=1_000_000, first_read=i * 40000) for i in range(3)]
    with kca.Context(kmer_length=31, line_length=150, engine="skm") as ctx:
        for b in blocks:
            ctx.count_fastq(b)
        got = ctx.records()
    want, _ = orc.refcpu(b"".join(blocks), 31, threads=8)
    assert got == want


def test_auto_engine_switches_on_high_cardinality(kca, orc):
    """iid reads (every key distinct): the skm sample sees no repeats and the
    key-prefix engine counts the batch instead; output identical."""
    n, L, k = 160_000, 150, 31
    fq = kca.synth_fastq(n, L, seed=77)
    with kca.Context(kmer_length=k, line_length=L, engine="auto", gpu_memory_limit=4 << 30) as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
        st = ctx.stats()
    assert st["engines_used"] == 2
    assert got == orc.count_fastq(fq, k)


@pytest.mark.parametrize("sample", [False, True])
def test_auto_engine_keeps_skm_on_genome_reads(kca, orc, monkeypatch, capfd, sample):
    """Genome reads at coverage keep the skm engine: the coverage sketch sees
    clear coverage and skips the skm bucket sample (round 6), or
    (KC_SKM_SAMPLE) the sample runs and agrees."""
    monkeypatch.setenv("KC_DEBUG", "1")
    if sample:
        monkeypatch.setenv("KC_SKM_SAMPLE", "1")
    n, L, k = 160_000, 150, 31
    fq = kca.synth_fastq(n, L, seed=78, genome_length=400_000)
    with kca.Context(kmer_length=k, line_length=L, engine="auto", gpu_memory_limit=4 << 30) as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
        st = ctx.stats()
    err = capfd.readouterr().err
    assert st["engines_used"] == 1
    assert got == orc.count_fastq(fq, k)
    # the sample's launch over the first 256 buckets (P5[0,256)) runs only when forced
    assert ("P5[0,256)" in err) == sample, err[-2000:]


def test_auto_engine_switch_after_skm_batches(kca, orc):
    """The first batch is below the sample threshold (skm), a later one is
    sampled and switches; skm and key-prefix records meet in one finish. (The
    blocks differ in read length, so the first is counted as a batch of its
    own before the second joins the pending batch.)"""
    k = 31
    blocks = [kca.synth_fastq(25_000, 140, seed=79), kca.synth_fastq(175_000, 150, seed=79, first_read=25_000)]
    with kca.Context(kmer_length=k, line_length=150, engine="auto", gpu_memory_limit=3 << 30) as ctx:
        for b in blocks:
            ctx.count_fastq(b, len(b.split(b"\n")[1]))
        got = ctx.records()
        st = ctx.stats()
    assert st["engines_used"] == 3
    assert got == orc.count_chunks([(c, ll) for b in blocks for c, ll in orc.chunks_of(b, 1 << 26)], k)


def _special_reads(L, n, seed):
    """Reads that reach F's slow path: not-ACGT bases, aligned all-A groups
    (possible key 0^W), poly-A / poly-T stretches, lowercase bases."""
    rng = random.Random(seed)
    out = []
    for i in range(n):
        s = [rng.choice("ACGT") for _ in range(L)]
        kind = i % 6
        if kind == 1:
            for _ in range(rng.randrange(1, 4)):
                s[rng.randrange(L)] = rng.choice("Nn.")
        elif kind == 2:
            a = rng.randrange(0, max(1, L - 40))
            s[a:a + 40] = "A" * min(40, L - a)
        elif kind == 3:
            s = list("A" * L)
        elif kind == 4:
            a = rng.randrange(0, max(1, L - 20))
            s[a:a + 20] = "T" * min(20, L - a)
            s[rng.randrange(L)] = "N"
        out.append("".join(s))
    return out


@pytest.mark.parametrize("front", ["f3", "f2"])
@pytest.mark.parametrize("k", list(range(18, 33)))
def test_skm_front_every_k(kca, orc, monkeypatch, k, front):
    """The W = 1 front ends for every k: F3 (skm_front3_k<k>, k >= 19; k = 18
    falls to F2) and F2 (skm_front2_k<1, k>, under KC_NO_F3) against the
    oracle, on reads that take their slow paths (not-ACGT bases, all-A
    stretches, poly-T) plus genome reads that take the fast paths."""
    if front == "f2":
        monkeypatch.setenv("KC_NO_F3", "1")
    L = 150
    reads = _special_reads(L, 3000, k)
    fq = _fq(reads) + kca.synth_fastq(20000, L, seed=k, genome_length=200_000, first_read=3000)
    with kca.Context(kmer_length=k, line_length=L, engine="skm") as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
    assert got == orc.count_fastq(fq, k)


@pytest.mark.parametrize("k,L", [(31, 40), (31, 63), (21, 200), (32, 300), (25, 530), (31, 600), (19, 1000)])
def test_skm_front_read_lengths(kca, orc, monkeypatch, k, L):
    """Read lengths from one 8-window chunk per read to past F2's 64 chunks;
    F3, F2 (KC_NO_F3) and the generic F (KC_NO_F3 + KC_NO_F2) give the same
    bytes where each applies."""
    fq = _fq(_special_reads(L, 400, L)) + kca.synth_fastq(3000, L, seed=L, genome_length=100_000, first_read=400)
    outs = []
    for env in ((), ("KC_NO_F3",), ("KC_NO_F3", "KC_NO_F2")):
        for v in env:
            monkeypatch.setenv(v, "1")
        with kca.Context(kmer_length=k, line_length=L, engine="skm") as ctx:
            ctx.count_fastq(fq)
            outs.append(ctx.records())
    assert outs[0] == outs[1] == outs[2]
    assert outs[0] == orc.count_fastq(fq, k)


@pytest.mark.parametrize("L", [27, 32, 48, 150])
def test_skm_front3_lengths_multiple_of_16(kca, orc, L):
    """F3 at read lengths around and at multiples of 16 (k = 27: the last
    window's key ends at the read end; all-A halves at the read end are real
    bases when L is a multiple of 8)."""
    k = 27
    reads = _special_reads(L, 600, L + 1) + ["A" * L, "T" * L, "A" * (L - 8) + "C" * 8]
    fq = _fq(reads) + kca.synth_fastq(2000, L, seed=L, genome_length=50_000, first_read=len(reads))
    with kca.Context(kmer_length=k, line_length=L, engine="skm") as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
    assert got == orc.count_fastq(fq, k)


@pytest.mark.parametrize("groups", [None, "64", "3", "64:nosplit", "8:room"])
def test_skm_dedup_genome_reads(kca, orc, monkeypatch, groups):
    """P5a: genome reads at ~20x, where most records repeat. With a small
    record table (KC_P5A_GROUPS) buckets overflow it: they are deduplicated
    again in 2..16 hash-split passes into overflow lists in the pool's free
    tail (dpos / kOverList), or, when the split still overflows (3 groups),
    with no splitting (KC_P5A_NO_SPLIT) or once the tail is full
    (KC_P5A_OVER_ROOM), P5 walks their own records (kRawList); KC_NO_DEDUP
    walks every bucket's own records."""
    if groups:
        g, _, mode = groups.partition(":")
        monkeypatch.setenv("KC_P5A_GROUPS", g)
        if mode == "nosplit":
            monkeypatch.setenv("KC_P5A_NO_SPLIT", "1")
        if mode == "room":
            monkeypatch.setenv("KC_P5A_OVER_ROOM", "20000")
    fq = kca.synth_fastq(60000, 150, seed=33, genome_length=400_000, n_rate=0.0005)
    with kca.Context(kmer_length=31, line_length=150, engine="skm") as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
        st = ctx.stats()
    monkeypatch.setenv("KC_NO_DEDUP", "1")
    with kca.Context(kmer_length=31, line_length=150, engine="skm") as ctx:
        ctx.count_fastq(fq)
        raw = ctx.records()
        st_raw = ctx.stats()
    if groups in ("64", "8:room"):
        assert st["dedup_records"] < st_raw["keys"]  # overflow lists deduplicated records
    assert got == raw
    assert got == orc.count_fastq(fq, 31)
    assert st["valid_kmers"] == sum(int.from_bytes(got[i + 8:i + 12], "little") for i in range(0, len(got), 12))


@pytest.mark.parametrize("L,mem", [(140, 1 << 21), (140, 3 << 20), (150, 1 << 21), (129, 5 << 20)])
def test_skm_odd_code_rows_batches(kca, orc, L, mem):
    """Reads whose code row is an odd number of words (L = 140: 9 words;
    129: 9) counted in many skm batches from one-pass index rows: batch slices
    hold an even number of reads so every slice's masks are 4-byte aligned for
    F3's DMA; L = 150 (10 words) alongside. Oracle bytes."""
    fq = kca.synth_fastq(30000, L, seed=60 + L, genome_length=200_000, n_rate=0.0005)
    with kca.Context(kmer_length=31, line_length=L, gpu_memory_limit=mem, engine="skm") as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
        st = ctx.stats()
    assert st["batches"] > 2
    assert got == orc.count_fastq(fq, 31)


@pytest.mark.parametrize("k", [21, 31])
def test_skm_dedup_weighted_spill(kca, orc, tmp_path, k):
    """Deduplicated records with multiplicities > 1 through the last-resort
    paths: a 1-slot LDS table and a 1 MiB working set send keys to the global
    table and the spill runs, where a key is written once per unit of its
    multiplicity."""
    fq = kca.synth_fastq(20000, 150, seed=35, genome_length=60_000)
    with kca.Context(kmer_length=k, line_length=150, gpu_memory_limit=1 << 20, engine="skm", lds_slots=1) as ctx:
        ctx.count_fastq(fq)
        got = ctx.output_bytes(str(tmp_path))
        st = ctx.stats()
    assert st["spilled_kmers"] > 0
    assert got == orc.count_fastq(fq, k)


@pytest.mark.parametrize("engine", ["skm", "partition"])
def test_release_build_ignores_ablation_variables(kca, orc, monkeypatch, engine):
    """Stray timing-ablation variables (they skip stages in experiment builds)
    change nothing in the release library: same bytes as the oracle."""
    for v in ("KC_F_SKIP", "KC_P2_SKIP", "KC_P5_SKIP", "KC_SEG_SKIP"):
        monkeypatch.setenv(v, "1")
    monkeypatch.setenv("KC_SKM_MMIN", "14")
    fq = kca.synth_fastq(20000, 150, seed=77, genome_length=200_000, n_rate=0.001)
    with kca.Context(kmer_length=31, line_length=150, engine=engine) as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
    assert got == orc.count_fastq(fq, 31)


@pytest.mark.parametrize("k", [21, 31, 55])
@pytest.mark.parametrize("genome", [0, 900_000], ids=["iid", "genome30x"])
def test_coverage_sketch_estimate(kca, orc, monkeypatch, capfd, k, genome):
    """The coverage sketch (sketch_k: k-mers sampled by a hash of their first
    code word, fingerprinted whole) on cfg2's shape scaled down: reads from a
    genome at 30x coverage give a distinct share near (1 - e^-1.8) / 1.8 =
    0.46 at k = 31 (0.54 at k = 55: 7 aligned k-mers per read, not 9), below
    the 0.7 threshold, and keep the super-k-mer engine; iid reads give ~1 and take the
    key-prefix engine. Output identical to the oracle either way."""
    monkeypatch.setenv("KC_DEBUG", "1")
    n, L = 180_000, 150  # >= 2^24 windows at every k here: the sketch runs
    fq = kca.synth_fastq(n, L, seed=80 + k, genome_length=genome)
    with kca.Context(kmer_length=k, line_length=L, gpu_memory_limit=4 << 30) as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
        st = ctx.stats()
    err = capfd.readouterr().err
    line = [x for x in err.splitlines() if x.startswith("kc: sketch ")]
    assert line, err[-2000:]
    d, m = int(line[0].split()[2]), int(line[0].split()[5])
    assert m >= 4096
    if genome:
        assert 0.3 < d / m < 0.7 and st["engines_used"] == 1, (d, m, st["engines_used"])
    else:
        assert d / m > 0.95 and st["engines_used"] == 2, (d, m, st["engines_used"])
    assert got == orc.count_fastq(fq, k)
