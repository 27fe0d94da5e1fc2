"""GPU parity: the HIP path (through the C ABI of libkc_hip.so) against the CPU
oracle, bit-exact SortedKMerFile bytes. Needs an MI355X."""
import json
import os
import random
import subprocess

import numpy as np
import pytest

import kmer_ref_py as kp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
MANIFEST = json.load(open(os.path.join(GOLD, "MANIFEST.json")))


def _fq(reads):
    return "".join(f"@r{i}\n{s}\n+\n{'I' * len(s)}\n" for i, s in enumerate(reads))


@pytest.fixture(params=["partition", "table", "skm"])
def engine(request):
    return request.param


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_golden_fastq_path(kca, name, engine):
    m = MANIFEST[name]
    data = open(os.path.join(GOLD, m["fastq"]), "rb").read()
    want = open(os.path.join(GOLD, m["expected"]), "rb").read()
    L = len(data.split(b"\n")[1])
    with kca.Context(kmer_length=m["k"], line_length=L, engine=engine) as ctx:
        ctx.count_fastq(data)
        assert ctx.records() == want


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_golden_chunk_path(kca, orc, name, engine):
    """Reference-exact chunks (readData restatement) through kc_count_chunk."""
    m = MANIFEST[name]
    data = open(os.path.join(GOLD, m["fastq"]), "rb").read()
    want = open(os.path.join(GOLD, m["expected"]), "rb").read()
    L = len(data.split(b"\n")[1])
    with kca.Context(kmer_length=m["k"], line_length=L, engine=engine) as ctx:
        for chunk, ll in orc.chunks_of(data, orc.chunk_size(L, m["k"], 100000000)):
            ctx.count_chunk(chunk, ll)
        assert ctx.records() == want


@pytest.mark.parametrize("k,L,n_rate", [(21, 100, 0.002), (31, 150, 0.0), (31, 150, 0.01), (32, 150, 0.001),
                                        (33, 120, 0.001), (55, 150, 0.002), (64, 150, 0.0), (96, 150, 0.001),
                                        (127, 150, 0.0), (128, 250, 0.001), (16, 64, 0.01), (31, 96, 0.0),
                                        (25, 1000, 0.001), (31, 5000, 0.0005), (1, 12, 0.05)])
def test_synthetic_vs_oracle(kca, orc, k, L, n_rate, engine):
    n = max(50, 300000 // L)
    fq = kca.synth_fastq(n, L, seed=k * 7 + L, n_rate=n_rate)
    with kca.Context(kmer_length=k, line_length=L, engine=engine) as ctx:
        assert ctx.count_fastq(fq) == n
        got = ctx.records()
        st = ctx.stats()
    assert got == orc.count_fastq(fq, k)
    assert st["windows"] == n * (L - k + 1)


def test_genome_reads_k31(kca, orc, engine):
    fq = kca.synth_fastq(200000, 150, seed=2, genome_length=2_000_000)
    with kca.Context(kmer_length=31, line_length=150, engine=engine) as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
    want, _ = orc.refcpu(fq, 31, threads=8)
    assert got == want


def test_special_reads(kca, engine):
    reads = ["A" * 80, "N" * 80, "T" * 80, "acgt" * 20, "A" * 40 + "N" + "A" * 39, "C" * 79 + "N",
             "ACGT" * 20, "T" * 31 + "G" + "T" * 48]
    for k in (1, 21, 31, 32, 33, 64, 80):
        text = _fq(reads)
        want = kp.to_bytes(kp.count_reads(reads, k), k)
        with kca.Context(kmer_length=k, line_length=80, engine=engine) as ctx:
            ctx.count_fastq(text.encode())
            assert ctx.records() == want, k


def test_only_invalid_reads_give_key0_count0(kca):
    text = _fq(["N" * 50] * 3)
    with kca.Context(kmer_length=31, line_length=50) as ctx:
        ctx.count_fastq(text.encode())
        assert kp.parse_records(ctx.records(), 31) == [((0,), 0)]


def test_empty_input(kca):
    with kca.Context(kmer_length=31, line_length=150) as ctx:
        ctx.count_fastq(b"")
        ctx.count_chunk(b"", 150)
        assert ctx.records() == b""


def test_chunk_trailing_partial_read_is_ignored(kca):
    reads = ["ACGTTGCA" * 4 + "AC"] * 3
    chunk = "".join(reads).encode() + b"ACGTACGTAC"  # 10 bytes of a 4th read
    with kca.Context(kmer_length=21, line_length=34) as ctx:
        ctx.count_chunk(chunk, 34)
        assert ctx.records() == kp.to_bytes(kp.count_reads(reads, 21), 21)


def test_malformed_fastq_is_rejected_without_counting(kca):
    good = _fq(["ACGT" * 25] * 4)
    bad = good + "@x\nACGT\n+\nIIII\n"  # a short read
    with kca.Context(kmer_length=21, line_length=100) as ctx:
        with pytest.raises(kca.KcError) as e:
            ctx.count_fastq(bad.encode())
        assert e.value.status == kca.KC_ERR_FORMAT
        with pytest.raises(kca.KcError):
            ctx.count_fastq(good.encode()[:-1])  # no final newline
        with pytest.raises(kca.KcError):
            ctx.count_fastq(good.replace("\n+\n", "\n-\n", 1).encode())
        ctx.count_fastq(good.encode())
        assert ctx.records() == kp.to_bytes(kp.count_reads(["ACGT" * 25] * 4, 21), 21)


def test_device_generator_matches_host(kca):
    with kca.Context(kmer_length=31, line_length=150) as ctx:
        for spec in [(5000, 150, 9, 0, 0.003, 0), (3000, 150, 2, 1_000_000, 0.0, 12345)]:
            ptr, n = ctx.synth_device(*spec)
            dev = ctx.copy_to_host(ptr, n)
            ctx.free_device(ptr)
            assert dev == kca.synth_fastq(*spec)


def test_device_resident_fastq_and_reset(kca, orc):
    with kca.Context(kmer_length=31, line_length=150) as ctx:
        ptr, n = ctx.synth_device(20000, 150, 4, 500_000, 0.001, 0)
        host = ctx.copy_to_host(ptr, n)
        assert ctx.count_fastq_device(ptr, n) == 20000
        first = ctx.records()
        ctx.reset()
        ctx.count_fastq_device(ptr, n)
        again = ctx.records()
        ctx.free_device(ptr)
    assert first == again == orc.count_fastq(host, 31)


@pytest.mark.parametrize("k,temp", [(31, False), (31, True), (55, False), (21, True), (100, False)])
def test_spill_path(kca, orc, tmp_path, k, temp, engine):
    """A tiny working set forces the spill -> radix sort -> run -> merge path
    (partition engine: a 1-slot LDS table forces the global-table fallback
    first)."""
    L = 150
    fq = kca.synth_fastq(20000, L, seed=k, n_rate=0.001)
    with kca.Context(kmer_length=k, line_length=L, gpu_memory_limit=1 << 20, engine=engine, lds_slots=1,
                     temp_dir=str(tmp_path) if temp else None) as ctx:
        ctx.count_fastq(fq)
        got = ctx.output_bytes(str(tmp_path))
        st = ctx.stats()
    assert st["spill_runs"] >= 2 and st["spilled_kmers"] > 0
    assert got == orc.count_fastq(fq, k)


def test_multiple_blocks_accumulate(kca, orc, engine):
    blocks = [kca.synth_fastq(3000, 150, seed=11, n_rate=0.001, first_read=i * 3000) for i in range(4)]
    with kca.Context(kmer_length=31, line_length=150, engine=engine) as ctx:
        for b in blocks:
            ctx.count_fastq(b)
        got = ctx.records()
    assert got == orc.count_fastq(b"".join(blocks), 31)


@pytest.mark.parametrize("k", [31, 55])
def test_partition_many_batches(kca, orc, k):
    """A small working set splits one block into many partition batches whose
    records are summed at finish."""
    fq = kca.synth_fastq(60000, 150, seed=21, genome_length=300_000, n_rate=0.0005)
    with kca.Context(kmer_length=k, line_length=150, gpu_memory_limit=1 << 21, engine="partition") as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
        st = ctx.stats()
    assert st["batches"] > 3
    assert got == orc.count_fastq(fq, k)


def _write_dir(tmp_path, name, text):
    d = tmp_path / name
    d.mkdir()
    (d / "reads.fq").write_text(text)
    return d


@pytest.mark.parametrize("mode", ["auto", "fastq", "exact"])
def test_cli_end_to_end(kca, orc, tmp_path, mode):
    fq = kca.synth_fastq(5000, 150, seed=3, n_rate=0.002).decode()
    d = _write_dir(tmp_path, "in", fq)
    out = tmp_path / "out.bin"
    o = kca.Options()
    o.SetKmerLength(31)
    o.SetInputFileDirectory(str(d))
    o.setOutputFile(str(out))
    o.setTempFileLocation(str(tmp_path))
    kca.KMerCounter(o, [f"inputMode={mode}", "quiet=1"]).Start()
    assert out.read_bytes() == orc.count_fastq(fq.encode(), 31)


def test_cli_auto_falls_back_to_exact_on_malformed_input(kca, orc, tmp_path):
    rng = random.Random(1)
    text = "".join(f"@{'h' * 70}{i}\n{''.join(rng.choice('ACGT') for _ in range(30))}\n+\n{'I' * 30}\n"
                   for i in range(200))
    text = text.replace("\n+\n", "\n+\n", 1) + "\n"  # trailing blank line: not 4-line records
    d = _write_dir(tmp_path, "in", text)
    out = tmp_path / "out.bin"
    limit = 20000
    subprocess.run([kca.CLI_PATH, "kmerLength=21", f"inputFileLocation={d}", f"outputFile={out}",
                    f"gpuMemoryLimit={limit}", f"tempFileLocation={tmp_path}", "quiet=1"], check=True,
                   capture_output=True)
    # the reference's reader loses reads at chunk edges here (header >= 2L)
    want = orc.count_chunks(orc.chunks_of(text.encode(), orc.chunk_size(30, 21, limit)), 21)
    assert out.read_bytes() == want


def test_cli_multi_context(kca, orc, tmp_path):
    """gpus=3: three device contexts (sharing the one GPU of a 1-GPU box) count
    round-robin blocks of several files; their sorted runs are k-way merged."""
    d = tmp_path / "in"
    d.mkdir()
    texts = []
    for i in range(5):
        t = kca.synth_fastq(2000, 150, seed=30 + i, n_rate=0.001)
        (d / f"f{i}.fq").write_bytes(t)
        texts.append(t)
    out = tmp_path / "o.bin"
    subprocess.run([kca.CLI_PATH, "kmerLength=31", f"inputFileLocation={d}", f"outputFile={out}",
                    f"tempFileLocation={tmp_path}", "gpus=3", "quiet=1"], check=True, capture_output=True)
    want = orc.count_chunks([(c, ll) for t in texts for c, ll in orc.chunks_of(t, orc.chunk_size(150, 31, 100000000))],
                            31)
    assert out.read_bytes() == want


def test_cli_spill_and_merge_knobs(kca, orc, tmp_path):
    fq = kca.synth_fastq(30000, 100, seed=8, n_rate=0.001).decode()
    d = _write_dir(tmp_path, "in", fq)
    want = orc.count_fastq(fq.encode(), 25)
    for fan, thr in ((2, 2), (3, 1), (8, 4)):
        out = tmp_path / f"o{fan}.bin"
        subprocess.run([kca.CLI_PATH, "kmerLength=25", f"inputFileLocation={d}", f"outputFile={out}",
                        "gpuMemoryLimit=1048576", f"tempFileLocation={tmp_path}", f"noOfMergersAtOnce={fan}",
                        f"noOfMergeThreads={thr}", "quiet=1"], check=True, capture_output=True)
        assert out.read_bytes() == want
    assert not [p for p in os.listdir(tmp_path) if p.startswith("kc.")]  # spill runs cleaned up


@pytest.mark.slow
def test_config2_full_size_properties(kca, orc):
    """BASELINE config 2 (k=31, 50M x 150 bp from a 250 Mbp genome) with a
    24 GiB working set (several batches whose runs are merged): the window
    checksums of the whole input (CPU) equal the records' (a count moved
    between keys fails it), strictly ascending keys, counts sum to the valid
    windows, and every k-mer of sampled reads is present with a count no lower
    than its multiplicity in the sample."""
    n, L, k = 50_000_000, 150, 31
    with kca.Context(kmer_length=k, line_length=L, gpu_memory_limit=24 << 30) as ctx:
        ptr, nb = ctx.synth_device(n, L, 2, 250_000_000, 0.0, 0)
        fq = _host_fastq(ctx, ptr, nb)
        assert ctx.count_fastq_device(ptr, nb) == n
        ctx.free_device(ptr)
        raw = _host_records(ctx)
        st = ctx.stats()
    assert st["spilled_kmers"] == 0 and st["batches"] >= 2
    _assert_window_checksum(orc, fq, raw, k, _usable_cpus())
    del fq
    recs = raw.view(dtype=[("k", "<u8"), ("c", "<u4")])
    assert np.all(recs["k"][1:] > recs["k"][:-1])
    assert int(recs["c"].astype(np.uint64).sum()) == n * (L - k + 1) == st["valid_kmers"]
    sample = kca.synth_fastq(2000, L, 2, genome_length=250_000_000, first_read=n - 2000).decode()
    cnt = kp.count_reads(kp.fastq_reads(sample), k)
    keys = np.array([key[0] for key in cnt], dtype=np.uint64)
    idx = np.searchsorted(recs["k"], keys)
    assert np.all(recs["k"][idx] == keys)
    assert np.all(recs["c"][idx] >= np.array([cnt[key] for key in cnt], dtype=np.uint32))


def _usable_cpus():
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return n


@pytest.mark.slow
def test_config2_prefix_bit_exact_through_file_path(kca, orc, tmp_path):
    """BASELINE config 2's read stream (k=31, 150 bp from the 250 Mbp genome,
    seed 2), its first 10M reads (1.2e9 k-mers), end to end through the
    product path: FASTQ file -> kc_count_file -> kc_write_output. The output
    file's sha256 equals that of the reference-structured CPU pipeline (oracle
    refcpu: readData chunks at gpuMemoryLimit=1e8, bitEncode / extractKMers /
    reduceKMers restated, hash aggregation, sorted) run on every usable core."""
    import hashlib

    n, L, k = 10_000_000, 150, 31
    fq_path, out = tmp_path / "cfg2_prefix.fq", tmp_path / "out.bin"
    with kca.Context(kmer_length=k, line_length=L, gpu_memory_limit=24 << 30) as ctx:
        ptr, nb = ctx.synth_device(n, L, 2, 250_000_000, 0.0, 0)
        host = np.empty(nb, dtype=np.uint8)
        ctx.copy_to_host_addr(host.ctypes.data, ptr, nb)
        ctx.free_device(ptr)
        host.tofile(str(fq_path))
        assert ctx.count_file(str(fq_path)) == n
        ctx.write_output(str(out))
        st = ctx.stats()
    got = hashlib.sha256(out.read_bytes()).hexdigest()
    fq = host.tobytes()
    del host
    want, windows = orc.refcpu(fq, k, threads=_usable_cpus())
    assert windows == n * (L - k + 1) == st["windows"]
    assert st["spilled_kmers"] == 0
    assert got == hashlib.sha256(want).hexdigest()


def _host_records(ctx):
    """The finished run's SortedKMerFile records as a host numpy uint8 array."""
    import torch

    n = ctx.finish()
    t = torch.empty(max(1, n * ctx.rs), dtype=torch.uint8)
    ctx.export_records(t)
    return t.numpy()[: n * ctx.rs]


def _host_fastq(ctx, ptr, nb):
    host = np.empty(nb, dtype=np.uint8)
    ctx.copy_to_host_addr(host.ctypes.data, ptr, nb)
    return host


def _assert_window_checksum(orc, fq, recs, k, threads):
    """Full-size parity property (kc_oracle.c window checksums): the sums of two
    64-bit key hashes over every valid window of the FASTQ (CPU, spec form)
    equal the count-weighted sums over the GPU's records; keys strictly
    ascending; key 0^W present when a window was invalid."""
    a = orc.window_checksum(fq, k, threads=threads)
    b = orc.records_checksum(recs, k, threads=threads)
    assert b["unordered"] == 0
    assert b["count"] == a["valid"]
    assert (b["h1"], b["h2"]) == (a["h1"], a["h2"])
    if a["hole"]:
        assert not recs[: 8 * ((k + 31) // 32)].any()
    return a


@pytest.mark.slow
@pytest.mark.timeout(900)
def test_config2_benched_step_bit_exact(kca, orc):
    """The configuration bench.py times, byte-compared at full size: BASELINE
    config 2 (k=31, 50M x 150 bp from the 250 Mbp genome, seed 2) with the
    bench's 160 GiB working set, through exactly bench.py's dev_step
    (kc_reset, kc_count_fastq_device, kc_finish): all 50M reads are one
    super-k-mer batch (5.9e8 records, ~9K per bucket against P5a's LDS table,
    so its raw-bucket and sub-range fallbacks run at scale). The records'
    sha256 equals that of the reference-structured CPU pipeline (oracle refcpu:
    readData chunks at gpuMemoryLimit=1e8, bitEncode / extractKMers /
    reduceKMers restated, hash aggregation, sorted; GPUHandler.cu:129-233,
    KMerCounter.cpp:61-82,91-106) on every usable core; the window checksum
    is checked first (seconds) so a mismatch is reported early."""
    import hashlib

    n, L, k = 50_000_000, 150, 31
    with kca.Context(kmer_length=k, line_length=L, gpu_memory_limit=160 << 30) as ctx:
        ptr, nb = ctx.synth_device(n, L, 2, 250_000_000, 0.0, 0)
        fq = _host_fastq(ctx, ptr, nb)
        ctx.reset()
        assert ctx.count_fastq_device(ptr, nb) == n
        ctx.finish()
        st = ctx.stats()
        ctx.free_device(ptr)
        recs = _host_records(ctx)
    assert st["batches"] == 1 and st["engines_used"] == 1 and st["spilled_kmers"] == 0
    threads = _usable_cpus()
    a = _assert_window_checksum(orc, fq, recs, k, threads)
    assert a["windows"] == n * (L - k + 1) == st["windows"]
    got = hashlib.sha256(recs).hexdigest()
    del recs
    want, windows = orc.refcpu(fq, k, threads=threads)
    assert windows == n * (L - k + 1)
    assert got == hashlib.sha256(want).hexdigest()


@pytest.mark.slow
@pytest.mark.timeout(900)
def test_config4_shard_one_batch_checksum(kca, orc):
    """BASELINE config 4's per-GPU shard as bench.py --config 4 counts it:
    k=31, 125M x 150 bp reads (seed 4, 250 Mbp genome), 160 GiB working set,
    one super-k-mer batch up to the record pool (1.5e9 records, ~22.6K per
    bucket: P5a's LDS table overflows in about half the buckets, which P5 then
    counts raw). 15e9 k-mers are too many to recount by hash on the host in
    the test's time, so the full-size parity property is checked: window
    checksums over every valid window (CPU, spec form) equal the
    count-weighted record checksums, keys strictly ascending."""
    n, L, k = 125_000_000, 150, 31
    with kca.Context(kmer_length=k, line_length=L, gpu_memory_limit=160 << 30) as ctx:
        ptr, nb = ctx.synth_device(n, L, 4, 250_000_000, 0.0, 0)
        fq = _host_fastq(ctx, ptr, nb)
        ctx.reset()
        assert ctx.count_fastq_device(ptr, nb) == n
        ctx.finish()
        st = ctx.stats()
        ctx.free_device(ptr)
        recs = _host_records(ctx)
    assert st["batches"] == 1 and st["engines_used"] == 1 and st["spilled_kmers"] == 0
    a = _assert_window_checksum(orc, fq, recs, k, _usable_cpus())
    assert a["windows"] == n * (L - k + 1) == st["windows"]


def _owner_slices(kca, recs, rs, world):
    out = [bytearray() for _ in range(world)]
    for i in range(0, len(recs), rs):
        out[kca.owner_of(int.from_bytes(recs[i:i + 8], "little"), world)] += recs[i:i + rs]
    return [bytes(o) for o in out]


@pytest.mark.parametrize("k,world", [(31, 3), (55, 2), (21, 8), (100, 5)])
def test_keyspace_split_and_merge_device(kca, orc, k, world, engine):
    """cfg4 device side in one process: `world` contexts count disjoint shards;
    kc_owner_counts splits each sorted run into contiguous owner slices; owner
    o's context merges (kc_merge_records_device) the slices it would receive;
    the owners' runs concatenated are the oracle count of the whole stream."""
    import torch

    per, L = 1500, 150
    dev = torch.device("cuda", 0)
    shards = [kca.synth_fastq(per, L, 11, n_rate=0.001, genome_length=100_000, first_read=r * per)
              for r in range(world)]
    ctxs = [kca.Context(kmer_length=k, line_length=L, engine=engine) for _ in range(world)]
    try:
        slices = []
        for c, fq in zip(ctxs, shards):
            c.count_fastq(fq)
            recs = c.records()
            counts = c.owner_counts(world)
            sl = _owner_slices(kca, recs, c.rs, world)
            assert counts == [len(s) // c.rs for s in sl]
            assert b"".join(sl) == recs
            t = torch.empty(len(recs), dtype=torch.uint8, device=dev)
            assert c.export_records(t) == len(recs) // c.rs
            assert bytes(t.cpu().numpy().tobytes()) == recs
            slices.append(sl)
        owned = []
        for o, c in enumerate(ctxs):
            buf = b"".join(slices[r][o] for r in range(world))
            src = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to(dev) if buf else \
                torch.empty(0, dtype=torch.uint8, device=dev)
            n = c.merge_records(src, len(buf) // c.rs)
            got = c.records()
            assert n == len(got) // c.rs
            owned.append(got)
        assert b"".join(owned) == orc.count_fastq(b"".join(shards), k)
    finally:
        for c in ctxs:
            c.close()


def test_merge_records_device_sums_shuffled_duplicates(kca, orc):
    """kc_merge_records_device takes records in any order with repeated keys:
    shuffled records of two runs (and a run merged with itself) come back
    sorted with summed counts; u32 wrap as in the reference's uint32 counts."""
    import torch

    k, L = 55, 120
    a = orc.count_fastq(kca.synth_fastq(3000, L, 5, n_rate=0.002), k)
    b = orc.count_fastq(kca.synth_fastq(3000, L, 6, n_rate=0.002), k)
    rs = orc.rs_of(k)
    recs = [a[i:i + rs] for i in range(0, len(a), rs)] + [b[i:i + rs] for i in range(0, len(b), rs)]
    random.Random(3).shuffle(recs)
    with kca.Context(kmer_length=k, line_length=L) as ctx:
        ctx.count_fastq(kca.synth_fastq(3000, L, 5, n_rate=0.002))
        ctx.count_fastq(kca.synth_fastq(3000, L, 6, n_rate=0.002))
        want = ctx.records()
        src = torch.frombuffer(bytearray(b"".join(recs)), dtype=torch.uint8).cuda()
        assert ctx.merge_records(src, len(recs)) * rs == len(want)
        assert ctx.records() == want
        big = bytearray(want[:rs])
        big[-4:] = (0xFFFFFFFF).to_bytes(4, "little")
        two = torch.frombuffer(bytearray(bytes(big) * 2), dtype=torch.uint8).cuda()
        assert ctx.merge_records(two, 2) == 1
        assert ctx.records() == bytes(big[:-4]) + (0xFFFFFFFE).to_bytes(4, "little")
        assert ctx.merge_records(torch.empty(0, dtype=torch.uint8).cuda(), 0) == 0
        assert ctx.records() == b""


def test_keyspace_exchange_rccl_world1(kca, orc):
    """keyspace_exchange over RCCL (backend nccl) at world size 1: the count
    all-to-all, the record all-to-all and the device merge run on HBM-resident
    tensors; the result is the rank's own count. Ranks > 1 are covered by the
    gloo tests in tests/test_dist.py (the 1-GPU box cannot host two RCCL ranks)."""
    import socket

    import torch
    import torch.distributed as dist

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        fq = kca.synth_fastq(4000, 150, 9, n_rate=0.001)
        with kca.Context(kmer_length=31, line_length=150) as ctx:
            ctx.count_fastq(fq)
            n = kca.keyspace_exchange(ctx, dist, torch.device("cuda", 0))
            got = ctx.records()
        assert got == orc.count_fastq(fq, 31) and n * 12 == len(got)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("k", [31, 55])
def test_exchange_contexts_in_process(kca, orc, k):
    """kc_exchange_contexts: four contexts of one process (hipMemcpyPeer
    slices), each then owns one key range; concatenation = whole count."""
    shards = [kca.synth_fastq(1200, 150, 21 + r, n_rate=0.002, genome_length=50_000) for r in range(4)]
    ctxs = [kca.Context(kmer_length=k, line_length=150) for _ in shards]
    try:
        for c, fq in zip(ctxs, shards):
            c.count_fastq(fq)
            c.finish()
        kca.exchange_contexts(ctxs)
        parts = [c.records() for c in ctxs]
    finally:
        for c in ctxs:
            c.close()
    assert b"".join(parts) == orc.count_fastq(b"".join(shards), k)
    assert all(parts)


@pytest.mark.parametrize("mem", [100000000, 1048576])
def test_cli_exchange_alltoall(kca, orc, tmp_path, mem):
    """exchange=alltoall with gpus=3: output by concatenation of the contexts'
    key ranges; with a 1 MiB gpuMemoryLimit the contexts spill and the CLI
    takes the k-way merge instead. Same bytes either way."""
    d = tmp_path / "in"
    d.mkdir()
    texts = []
    for i in range(4):
        t = kca.synth_fastq(3000, 150, seed=50 + i, n_rate=0.001)
        (d / f"f{i}.fq").write_bytes(t)
        texts.append(t)
    out = tmp_path / "o.bin"
    subprocess.run([kca.CLI_PATH, "kmerLength=31", f"inputFileLocation={d}", f"outputFile={out}",
                    f"tempFileLocation={tmp_path}", "gpus=3", "exchange=alltoall", f"gpuMemoryLimit={mem}",
                    "quiet=1"], check=True, capture_output=True)
    want = orc.count_chunks([(c, ll) for t in texts for c, ll in orc.chunks_of(t, orc.chunk_size(150, 31, mem))], 31)
    assert out.read_bytes() == want


@pytest.mark.parametrize("k,slots", [(31, 64), (55, 64), (31, 128), (100, 96)])
def test_partition_subrange_passes(kca, orc, k, slots):
    """High cardinality per bucket (SURVEY cfg5 shape, scaled down by a small
    LDS table): buckets overflow the table and are counted in m sub-range
    passes, still entirely in LDS (no spill, no fallback-table claims)."""
    n, L = 40000, 150
    fq = kca.synth_fastq(n, L, seed=k + slots, n_rate=0.0005)
    with kca.Context(kmer_length=k, line_length=L, lds_slots=slots, engine="partition") as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
        st = ctx.stats()
    assert got == orc.count_fastq(fq, k)
    assert st["spilled_kmers"] == 0 and st["table_used"] == 0


@pytest.mark.parametrize("k", [31, 55, 100])
def test_presplit_buckets_high_cardinality(kca, orc, monkeypatch, k):
    """High cardinality on the key-prefix engine: after a batch whose keys
    were mostly distinct, the next batches split every bucket once more by key
    bits 40..47 (P3b, an MSD regional radix pass) and P5 counts runs of
    consecutive sub-buckets in one pass each; the runs cut from the records
    merge on the device. Runs of sub-buckets are sorted in LDS (P5s), into
    records or (KC_P5S_DIRECT_MIN=1) straight into each batch's finished
    packed run; the LDS hash table for every run (KC_NO_SORT_RUNS) and no P3b
    pass (KC_NO_P3B) give the same bytes as the oracle."""
    monkeypatch.setenv("KC_P3B_MIN", "1")
    fq = kca.synth_fastq(30000, 150, seed=k + 3, n_rate=0.0005)
    outs = []
    for env in ((), ("KC_P5S_DIRECT_MIN",), ("KC_NO_SORT_RUNS",), ("KC_NO_P3B",)):
        for v in env:
            monkeypatch.setenv(v, "1")
        with kca.Context(kmer_length=k, line_length=150, gpu_memory_limit=24 << 20, engine="partition") as ctx:
            ctx.count_fastq(fq)
            outs.append(ctx.records())
            st = ctx.stats()
        assert st["batches"] >= 3
        for v in env:
            monkeypatch.delenv(v)
    assert outs[0] == outs[1] == outs[2] == outs[3] == orc.count_fastq(fq, k)


@pytest.mark.parametrize("knob", ["KC_P2_SOA", "KC_P3_SOA", "KC_P3B_SOA", "KC_P2_NO_DIGS", "KC_P3_SCATTER",
                                  "KC_NO_DUAL_PASS"])
@pytest.mark.parametrize("k", [31, 55])
def test_layout_knobs_same_counts(kca, orc, monkeypatch, knob, k):
    """The key-prefix engine's layout and path knobs (word arrays instead of
    AoS keys from P2 / P3 / P3b, P3b's histogram from word 0 instead of P3's
    digit bytes, the older P3 scatter, no dual key-range walk) are documented
    as giving the same counts: each alone, on high-cardinality reads counted
    in batches with P3b, and through key-range passes, against the oracle."""
    monkeypatch.setenv("KC_P3B_MIN", "1")
    monkeypatch.setenv(knob, "1")
    fq = kca.synth_fastq(30000, 150, seed=k + 5, n_rate=0.0005)
    want = orc.count_fastq(fq, k)
    with kca.Context(kmer_length=k, line_length=150, gpu_memory_limit=24 << 20, engine="partition") as ctx:
        ctx.count_fastq(fq)
        assert ctx.records() == want
        assert ctx.stats()["presplit_batches"] >= 1 or knob == "KC_NO_P3B"
    monkeypatch.setenv("KC_KEY_PASSES_MIN", "2")
    with kca.Context(kmer_length=k, line_length=150, gpu_memory_limit=24 << 20, engine="partition") as ctx:
        ctx.count_fastq(fq)
        assert ctx.records() == want


@pytest.mark.parametrize("k", [31, 55])
def test_direct_runs_with_equal_keys(kca, orc, monkeypatch, capfd, k):
    """P5s direct mode on batches whose runs hold equal keys (a fifth of the
    reads repeat earlier reads, so k-mers occur several times while most are
    distinct): the runs leave gaps in the packed run, which a segment copy
    closes. Key 0 (an all-A read) takes record 0. Same bytes as the oracle;
    the direct path is seen in the debug line."""
    import numpy as np
    monkeypatch.setenv("KC_P3B_MIN", "1")
    monkeypatch.setenv("KC_P5S_DIRECT_MIN", "1")
    monkeypatch.setenv("KC_DEBUG", "1")
    rng = np.random.default_rng(k + 11)
    L = 150
    reads = rng.integers(0, 4, size=(40000, L), dtype=np.uint8)
    rep = rng.integers(0, 40000, size=8000)
    reads[32000:] = reads[rep]
    reads[5] = 0
    fq = _fastq_from_codes(reads[rng.permutation(len(reads))])
    with kca.Context(kmer_length=k, line_length=L, gpu_memory_limit=24 << 20, engine="partition") as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
    err = capfd.readouterr().err
    kept = [x for x in err.splitlines() if "kc: P5s direct" in x and "kept=1" in x]
    gaps = [x for x in kept if int(x.split("records=")[1].split()[0]) < int(x.split(" n=")[1].split()[0])]
    assert kept and gaps, err[-2000:]
    assert got == orc.count_fastq(fq, k)


def _fastq_from_codes(codes):
    """FASTQ bytes of reads given as base codes 0..3 (ACGT), one row a read."""
    import numpy as np
    seq = np.frombuffer(b"ACGT", dtype=np.uint8)[codes]
    L = codes.shape[1]
    qual = b"I" * L
    out = []
    for i, row in enumerate(seq):
        out.append(b"@r%d\n%s\n+\n%s\n" % (i, row.tobytes(), qual))
    return b"".join(out)


@pytest.mark.parametrize("k", [31, 55])
def test_sorted_runs_hand_off_to_hash_path(kca, orc, monkeypatch, capfd, k):
    """P5s hands the runs it cannot sort to the LDS hash table: a sub-bucket
    of more keys than a sorted run holds (12k reads sharing their first 12
    bases) and runs whose keys crowd one sort bin (3k reads sharing their first
    24 bases), among iid reads. One batch of >= 2^24 keys: the coverage sketch
    marks it high-cardinality, so P3b and P5s run on it. Same bytes as the
    oracle; the hand-off is seen in the P5s debug line."""
    import numpy as np
    monkeypatch.setenv("KC_DEBUG", "1")
    rng = np.random.default_rng(k)
    L = 150
    reads = rng.integers(0, 4, size=(180000, L), dtype=np.uint8)
    reads[:12000, :12] = rng.integers(0, 4, size=12, dtype=np.uint8)
    reads[12000:15000, :24] = rng.integers(0, 4, size=24, dtype=np.uint8)
    fq = _fastq_from_codes(reads[rng.permutation(len(reads))])
    with kca.Context(kmer_length=k, line_length=L, gpu_memory_limit=2 << 30, engine="partition") as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
    err = capfd.readouterr().err
    flagged = [int(x.split("flagged=")[1].split()[0]) for x in err.splitlines() if "kc: P5s" in x and "flagged=" in x]
    assert flagged and max(flagged) > 0, err[-2000:]
    assert got == orc.count_fastq(fq, k)


def _hc_reads(rng, n, L, dup=0, clusters=()):
    """n iid reads of L bases (codes 0..3); the last `dup` reads repeat earlier
    ones (equal keys), read 5 is all A (key 0); clusters = ((reads, bases), ...)
    give groups of reads sharing their first `bases` bases."""
    import numpy as np
    reads = rng.integers(0, 4, size=(n, L), dtype=np.uint8)
    if dup:
        reads[n - dup:] = reads[rng.integers(0, n - dup, size=dup)]
    r0 = 10
    for cnt, nb in clusters:
        reads[r0:r0 + cnt, :nb] = rng.integers(0, 4, size=nb, dtype=np.uint8)
        r0 += cnt
    reads[5] = 0
    return reads[rng.permutation(n)]


@pytest.mark.parametrize("k", [31, 55, 100])
def test_key_range_passes(kca, orc, monkeypatch, capfd, k):
    """High cardinality with more keys than one batch holds (SURVEY cfg5's
    shape, scaled down to a 128 MB working set): the default engine counts
    all reads in key-range passes (each pass re-walks the reads and keeps one
    range of word0 >> 56; P5s direct appends it to one run, so the run is the
    concatenation of the passes and kc_finish merges nothing). Repeated reads
    put equal keys into runs (per-pass gap compaction), an all-A read gives
    key 0. Same bytes as the oracle and as read batches + run merge
    (KC_NO_KEY_PASSES)."""
    import numpy as np
    monkeypatch.setenv("KC_P3B_MIN", "1")
    monkeypatch.setenv("KC_DEBUG", "1")
    L = 150
    n = max(180000, (1 << 24) // (L - k + 1) + 2000)  # the coverage sketch needs 2^24 keys
    fq = _fastq_from_codes(_hc_reads(np.random.default_rng(k + 101), n, L, dup=n // 20))
    outs, sts = [], []
    for env in ((), ("KC_NO_DUAL_PASS",), ("KC_NO_KEY_PASSES",)):
        for v in env:
            monkeypatch.setenv(v, "1")
        with kca.Context(kmer_length=k, line_length=L, gpu_memory_limit=128 << 20) as ctx:
            ctx.count_fastq(fq)
            outs.append(ctx.records())
            sts.append(ctx.stats())
        for v in env:
            monkeypatch.delenv(v)
    err = capfd.readouterr().err
    assert sts[0]["key_passes"] >= 2 and sts[2]["key_passes"] == 0, err[-3000:]
    # two passes per P2 walk by default, one per walk under KC_NO_DUAL_PASS
    assert sts[0]["insert_launches"] == (sts[0]["key_passes"] + 1) // 2
    assert sts[1]["insert_launches"] == sts[1]["key_passes"]
    direct = [x for x in err.splitlines() if "kc: P5s direct pass" in x]
    assert len(direct) == sts[0]["key_passes"] + sts[1]["key_passes"] and all("kept=1" in x for x in direct), \
        err[-3000:]
    assert sts[2]["spill_runs"] >= 2
    assert outs[0] == outs[1] == outs[2] == orc.count_fastq(fq, k)


@pytest.mark.parametrize("k", [31, 55])
def test_key_range_pass_hands_off(kca, orc, monkeypatch, capfd, k):
    """A key-range pass that P5s cannot take direct (a sub-bucket of 12k keys:
    reads sharing their first 12 bases, among iid reads): the passes before it
    become a finished run, that pass and the later ones count into records
    (the LDS hash table for the flagged runs), kc_finish merges the two. Same
    bytes as the oracle."""
    import numpy as np
    monkeypatch.setenv("KC_P3B_MIN", "1")
    monkeypatch.setenv("KC_DEBUG", "1")
    L = 150
    n = 190000
    fq = _fastq_from_codes(_hc_reads(np.random.default_rng(k + 7), n, L, clusters=((12000, 12),)))
    with kca.Context(kmer_length=k, line_length=L, gpu_memory_limit=128 << 20) as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
        st = ctx.stats()
    err = capfd.readouterr().err
    direct = [x for x in err.splitlines() if "kc: P5s direct pass" in x]
    assert st["key_passes"] >= 2 and any("kept=0" in x for x in direct), err[-3000:]
    assert got == orc.count_fastq(fq, k)


def _u64_sortable(lo32, hi32):
    """(hi << 32 | lo) as int64 whose signed order is the unsigned order."""
    import torch
    v = (hi32.to(torch.int64) << 32) | (lo32.to(torch.int64) & 0xFFFFFFFF)
    return v ^ (-(1 << 63))


@pytest.mark.slow
@pytest.mark.parametrize("batches,mem", [(False, 24 << 30), (True, 24 << 30), (False, 48 << 30)],
                         ids=["key_passes", "read_batches", "bench_48GiB"])
def test_config5_full_size_properties(kca, orc, monkeypatch, batches, mem):
    """BASELINE config 5 (k=55 two-word keys, 20M x 150 bp iid reads, ~1.92e9
    distinct) on the default engine with a working set below the distinct
    count: the records outgrow it, are cut into sorted runs (the reference's
    spill -> sort path) and kc_finish merges the runs on the device. Checked
    on the device: keys strictly ascending (two-word order), counts sum to the
    valid windows, and every k-mer of sampled reads is present with a count
    no lower than its multiplicity in the sample; and on the host the window
    checksums of the whole input equal the records'. Default: key-range passes
    (one run, concatenated); read_batches (KC_NO_KEY_PASSES): one sorted run
    per read batch, merged on the device. bench_48GiB: exactly bench.py
    --config 5's working set (48 GiB), whose pass plan (two key-range passes,
    one P2 walk, direct P5s runs) produces the cfg5 bench lines."""
    import torch
    if batches:
        monkeypatch.setenv("KC_NO_KEY_PASSES", "1")

    n, L, k = 20_000_000, 150, 55
    dev = torch.device("cuda", 0)
    with kca.Context(kmer_length=k, line_length=L, gpu_memory_limit=mem) as ctx:
        ptr, nb = ctx.synth_device(n, L, 5, 0, 0.0, 0)
        checksum = (orc, _host_fastq(ctx, ptr, nb))
        assert ctx.count_fastq_device(ptr, nb) == n
        ctx.free_device(ptr)
        nrec = ctx.finish()
        st = ctx.stats()
        assert st["valid_kmers"] == n * (L - k + 1)
        if batches:
            assert st["spill_runs"] >= 2 and st["key_passes"] == 0
        elif mem == 48 << 30:
            assert st["key_passes"] == 2 and st["spill_runs"] == 1 and st["spilled_kmers"] == 0
            assert st["engines_used"] == 2 and st["sorted_run_batches"] >= 1
        else:
            assert st["key_passes"] >= 2 and st["spill_runs"] == 1
        rec = torch.empty(nrec * 20, dtype=torch.uint8, device=dev)
        ctx.export_records(rec)
    if checksum is not None:
        # the full-size parity property over all 1.92e9 records (CPU)
        _assert_window_checksum(checksum[0], checksum[1], rec.cpu().numpy(), k, _usable_cpus())
        checksum = None
    words = rec.view(torch.int32).view(nrec, 5)
    total = 0
    prev = None
    step = 100_000_000
    for s0 in range(0, nrec, step):
        w = words[s0:s0 + step]
        a = _u64_sortable(w[:, 0], w[:, 1])
        b = _u64_sortable(w[:, 2], w[:, 3])
        if prev is not None:
            a = torch.cat([prev[0], a])
            b = torch.cat([prev[1], b])
        asc = (a[1:] > a[:-1]) | ((a[1:] == a[:-1]) & (b[1:] > b[:-1]))
        assert bool(asc.all())
        total += int(w[:, 4].to(torch.int64).sum())
        prev = (a[-1:], b[-1:])
        del a, b, asc
    assert total == n * (L - k + 1)
    sample = kca.synth_fastq(1000, L, 5, first_read=n - 1000).decode()
    cnt = kp.count_reads(kp.fastq_reads(sample), k)
    keys = list(cnt)
    a_all = _u64_sortable(words[:, 0], words[:, 1])
    qa = torch.tensor([(key[0] ^ (1 << 63)) - (1 << 64) if (key[0] ^ (1 << 63)) >= (1 << 63)
                       else (key[0] ^ (1 << 63)) for key in keys], dtype=torch.int64, device=dev)
    idx = torch.searchsorted(a_all, qa).cpu().tolist()
    for key, i in zip(keys, idx):
        found = False
        j = i
        while j < nrec:
            r = words[j].cpu().tolist()
            w0 = (r[0] & 0xFFFFFFFF) | ((r[1] & 0xFFFFFFFF) << 32)
            if w0 != key[0]:
                break
            w1 = (r[2] & 0xFFFFFFFF) | ((r[3] & 0xFFFFFFFF) << 32)
            if w1 == key[1]:
                assert (r[4] & 0xFFFFFFFF) >= cnt[key]
                found = True
                break
            j += 1
        assert found, key


@pytest.mark.parametrize("k", [31, 55])
def test_skewed_segment_uses_lsd_fallback(kca, orc, k):
    """Reads that all start with the same 14 bases put >2000 distinct k-mers
    into one 12-bit bin of one P5 segment: the segment sort's MSD pass hands
    that segment to the LSD fallback kernel; output still bit-exact."""
    rng = random.Random(k)
    prefix = "ACGTTGCAACGTGA"
    reads = [prefix + "".join(rng.choice("ACGT") for _ in range(136)) for _ in range(3000)]
    fq = _fq(reads).encode()
    with kca.Context(kmer_length=k, line_length=150, engine="partition") as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
    assert got == orc.count_fastq(fq, k)


@pytest.mark.parametrize("k,nruns", [(31, 1), (31, 2), (31, 5), (55, 8), (100, 3)])
def test_merge_runs_device(kca, orc, k, nruns):
    """kc_merge_runs_device: nruns sorted runs (overlapping key ranges, shared
    keys summed, empty runs allowed) merged by merge path == one count of all."""
    import torch

    L = 120
    shards = [kca.synth_fastq(700 * (r % 3), L, 40 + r, n_rate=0.002, genome_length=30_000) for r in range(nruns)]
    runs = [orc.count_fastq(fq, k) if fq else b"" for fq in shards]
    rs = orc.rs_of(k)
    with kca.Context(kmer_length=k, line_length=L) as ctx:
        ctx.finish()
        buf = b"".join(runs)
        src = torch.frombuffer(bytearray(buf), dtype=torch.uint8).cuda() if buf else \
            torch.empty(0, dtype=torch.uint8).cuda()
        n = ctx.merge_runs(src, [len(r) // rs for r in runs])
        got = ctx.records()
    want = orc.count_fastq(b"".join(shards), k)
    assert got == want and n * rs == len(want)


@pytest.mark.parametrize("k", [31, 55])
def test_key_range_hand_off_cuts_runs(kca, orc, monkeypatch, capfd, k):
    """A hand-off in the first key-range pass with several passes left (a
    cluster of reads sharing their first 12 bases, all starting with A): the
    later passes count into records, which are cut into sorted runs between
    passes whenever they outgrow half the working set, instead of growing
    past it. Same bytes as the oracle."""
    import numpy as np
    monkeypatch.setenv("KC_P3B_MIN", "1")
    monkeypatch.setenv("KC_DEBUG", "1")
    L = 150
    n = 260000
    rng = np.random.default_rng(k + 19)
    reads = _hc_reads(rng, n, L)
    reads[:12000, :12] = np.array([0, 0, 1, 2, 3, 0, 1, 2, 3, 3, 2, 1], dtype=np.uint8)
    fq = _fastq_from_codes(reads[rng.permutation(n)])
    mem = 128 << 20
    with kca.Context(kmer_length=k, line_length=L, gpu_memory_limit=mem) as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
        st = ctx.stats()
    err = capfd.readouterr().err
    direct = [x for x in err.splitlines() if "kc: P5s direct pass" in x]
    assert st["key_passes"] >= 3, err[-3000:]
    assert direct and "kept=0" in direct[0], err[-3000:]
    assert st["spill_runs"] >= 2, (st, err[-3000:])
    assert got == orc.count_fastq(fq, k)


def test_key_range_passes_skewed_prefixes(kca, orc, monkeypatch, capfd):
    """High cardinality with a skewed base composition (A at 2/3): the keys'
    two-base groups (word0 >> 60) are far from balanced, the AA group alone
    holding ~44% of the keys. The planner gives an oversize group a pass of
    its own instead of falling back to read batches. Same bytes as the
    oracle. Sizes: ~24M keys, a 210 MB working set (11.4M keys per batch):
    3 passes of ~8M, the AA group ~10.7M, above the balanced cap (10M) and
    within a batch."""
    import numpy as np
    monkeypatch.setenv("KC_P3B_MIN", "1")
    monkeypatch.setenv("KC_DEBUG", "1")
    L, k = 150, 31
    n = 200000
    rng = np.random.default_rng(77)
    reads = rng.choice(4, size=(n, L), p=[2 / 3, 1 / 9, 1 / 9, 1 / 9]).astype(np.uint8)
    reads[5] = 0
    fq = _fastq_from_codes(reads)
    with kca.Context(kmer_length=k, line_length=L, gpu_memory_limit=210_000_000) as ctx:
        ctx.count_fastq(fq)
        got = ctx.records()
        st = ctx.stats()
    err = capfd.readouterr().err
    assert st["key_passes"] >= 2, (st, err[-3000:])
    assert got == orc.count_fastq(fq, k)


def test_config1_full_size(kca, orc, tmp_path):
    """BASELINE config 1 at its stated size: k=21, 10k x 100 bp iid reads with
    N rate 0.002 (seed 1), through the block path (kc_count_fastq), the file
    path (kc_count_file) and the reference's own chunks (kc_count_chunk at
    gpuMemoryLimit=1e8): all three equal the oracle's spec form and the
    reference-structured CPU pipeline (refcpu)."""
    n, L, k = 10_000, 100, 21
    fq = kca.synth_fastq(n, L, seed=1, n_rate=0.002)
    p = tmp_path / "cfg1.fq"
    p.write_bytes(fq)
    outs = []
    with kca.Context(kmer_length=k, line_length=L) as ctx:
        assert ctx.count_fastq(fq) == n
        outs.append(ctx.records())
        ctx.reset()
        assert ctx.count_file(str(p)) == n
        outs.append(ctx.records())
        ctx.reset()
        for chunk, ll in orc.chunks_of(fq, orc.chunk_size(L, k, 100_000_000)):
            ctx.count_chunk(chunk, ll)
        outs.append(ctx.records())
        st = ctx.stats()
    assert st["reads"] == n and st["windows"] == n * (L - k + 1)
    want, windows = orc.refcpu(fq, k, threads=4)
    assert windows == n * (L - k + 1)
    assert want == orc.count_fastq(fq, k)
    assert outs[0] == outs[1] == outs[2] == want


@pytest.mark.slow
def test_config5_prefix_bit_exact_key_passes(kca, orc, monkeypatch, capfd):
    """BASELINE config 5's read stream (k=55, iid 150 bp reads, seed 5), its
    first 2M reads (1.92e8 k-mers, nearly all distinct), counted from HBM by
    the default engine with a 2.4 GB working set: the keys are cut into 3
    key-range passes (one P2 walk for the first two, the second pass's keys
    staged in the run buffer), each P5s direct-written after the previous
    ones; the run is their concatenation. Its sha256 equals that of the
    reference-structured CPU pipeline (refcpu) on every usable core."""
    import hashlib

    monkeypatch.setenv("KC_DEBUG", "1")
    n, L, k = 2_000_000, 150, 55
    with kca.Context(kmer_length=k, line_length=L, gpu_memory_limit=2_400_000_000) as ctx:
        ptr, nb = ctx.synth_device(n, L, 5, 0, 0.0, 0)
        fq = ctx.copy_to_host(ptr, nb)
        assert ctx.count_fastq_device(ptr, nb) == n
        ctx.free_device(ptr)
        got = hashlib.sha256(ctx.records()).hexdigest()
        st = ctx.stats()
    err = capfd.readouterr().err
    direct = [x for x in err.splitlines() if "kc: P5s direct pass" in x]
    assert st["key_passes"] >= 3 and st["insert_launches"] < st["key_passes"], (st, err[-2000:])
    assert len(direct) == st["key_passes"] and all("kept=1" in x for x in direct), err[-2000:]
    want, windows = orc.refcpu(fq, k, threads=_usable_cpus())
    assert windows == n * (L - k + 1) == st["windows"]
    assert got == hashlib.sha256(want).hexdigest()
