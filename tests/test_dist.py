"""Multi-process (world size 2, gloo on the CPU) coverage of the read-shard
path of bench.py / the CLI: disjoint shards whose sorted runs, k-way merged
on the host (bench.host_merge_runs, cfg3 as stated), equal the count of the
whole read stream; the step time is the max over ranks. The per-shard counts come from the CPU oracle here (no GPU in
this container); the GPU side of the same path is covered by
tests/test_gpu_parity.py::test_cli_multi_context."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _FileRun:
    """Stand-in for a finished Context (no GPU here): its sorted run is the
    oracle's, written as a SortedKMerFile by write_output."""

    def __init__(self, records, k):
        self.k, self.rs, self._r = k, 8 * ((k + 31) // 32) + 4, records

    def write_output(self, path):
        with open(path, "wb") as f:
            f.write(self._r)


class _GlooRanks:
    def __init__(self, dist, rank, world):
        self.dist, self.rank, self.world = dist, rank, world

    def barrier_sync(self):
        self.dist.barrier()

    def all_gather_int(self, v):
        import torch
        t = torch.tensor([int(v)], dtype=torch.int64)
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [int(x.item()) for x in out]


def _worker(rank, world, port, tmpdir, per, k, where):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist

    import bench
    import oracle
    from conftest import load_pkg

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    kca = load_pkg()
    first = bench.shard_first(rank, per)
    fq = kca.synth_fastq(per, 150, 2, genome_length=400_000, first_read=first)
    run = oracle.count_fastq(fq, k)
    with open(os.path.join(tmpdir, f"run{rank}"), "wb") as f:
        f.write(run)
    # bench's cfg3 step as stated (--exchange files): run files + the host
    # k-way merge, shared by the ranks (each merges one key range of every
    # run file and writes it at its offset) or on rank 0 alone
    n, mine = bench.host_merge_runs(kca, _FileRun(run, k), _GlooRanks(dist, rank, world), tmpdir,
                                    os.path.join(tmpdir, "node.bin"), k, threads=2, where=where)
    with open(os.path.join(tmpdir, f"n{rank}"), "w") as f:
        f.write(f"{n} {mine}")
    t = bench.max_over_ranks(dist, float(rank + 1), torch.device("cpu"))
    with open(os.path.join(tmpdir, f"t{rank}"), "w") as f:
        f.write(repr(t))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,k,where", [(2, 31, "ranks"), (2, 55, "ranks"), (3, 31, "ranks"), (8, 21, "ranks"),
                                           (2, 31, "rank0"), (2, 55, "rank0")])
def test_read_shard_merge_equals_whole(kca, orc, tmp_path, world, k, where):
    per = 3000 if world < 8 else 600
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), per, k, where), nprocs=world, join=True)
    runs = [str(tmp_path / f"run{r}") for r in range(world)]
    out = tmp_path / "merged.bin"
    kca.merge_files(runs, str(out), k)
    whole = kca.synth_fastq(world * per, 150, 2, genome_length=400_000)
    assert out.read_bytes() == orc.count_fastq(whole, k)
    assert (tmp_path / "node.bin").read_bytes() == out.read_bytes()
    rs = 8 * ((k + 31) // 32) + 4
    ns = [tuple(map(int, (tmp_path / f"n{r}").read_text().split())) for r in range(world)]
    if where == "ranks":
        assert all(n * rs == out.stat().st_size for n, _ in ns)
        assert sum(m for _, m in ns) == out.stat().st_size
    else:
        assert ns[0] == (out.stat().st_size // rs, out.stat().st_size)
    for r in range(world):
        assert float((tmp_path / f"t{r}").read_text()) == float(world)


def test_shards_are_disjoint_and_cover(kca):
    import bench
    per = 1000
    parts = [kca.synth_fastq(per, 100, 7, first_read=bench.shard_first(r, per)) for r in range(3)]
    assert b"".join(parts) == kca.synth_fastq(3 * per, 100, 7)


class _OracleRun:
    """Test stand-in for a finished Context on a rank without a GPU: holds the
    oracle's sorted run and implements the four methods keyspace_exchange
    uses (finish/owner_counts/export_records/merge_records) on the host, so
    the protocol (count all-to-all, contiguous owner slices, record
    all-to-all, merge on the owner) is exercised over gloo. The device side
    of the same methods is tests/test_gpu_parity.py::test_keyspace_*."""

    def __init__(self, records: bytes, k: int, kca):
        self.W = (k + 31) // 32
        self.rs = 8 * self.W + 4
        self.data = records
        self.kca = kca

    def _keys(self, data):
        import numpy as np
        n = len(data) // self.rs
        a = np.frombuffer(data, dtype=np.uint8).reshape(n, self.rs)
        return a, n

    def finish(self):
        return len(self.data) // self.rs

    def owner_counts(self, world):
        a, n = self._keys(self.data)
        counts = [0] * world
        for i in range(n):
            key0 = int.from_bytes(a[i, 0:8].tobytes(), "little")
            counts[self.kca.owner_of(key0, world)] += 1
        return counts

    def export_records(self, dst):
        import torch
        dst[: len(self.data)] = torch.frombuffer(bytearray(self.data), dtype=torch.uint8)
        return self.finish()

    def merge_records(self, src, m):
        raw = bytes(src[: m * self.rs].numpy().tobytes())
        acc = {}
        for i in range(m):
            r = raw[i * self.rs:(i + 1) * self.rs]
            key = tuple(int.from_bytes(r[8 * j:8 * j + 8], "little") for j in range(self.W))
            acc[key] = (acc.get(key, 0) + int.from_bytes(r[-4:], "little")) & 0xFFFFFFFF
        out = bytearray()
        for key in sorted(acc):
            for w in key:
                out += w.to_bytes(8, "little")
            out += acc[key].to_bytes(4, "little")
        self.data = bytes(out)
        return len(acc)


def _ks_worker(rank, world, port, tmpdir, per, k):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist

    import bench
    import oracle
    from conftest import load_pkg
    from test_dist import _OracleRun

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    kca = load_pkg()
    fq = kca.synth_fastq(per, 150, 2, genome_length=200_000, first_read=bench.shard_first(rank, per))
    run = _OracleRun(oracle.count_fastq(fq, k), k, kca)
    n = kca.keyspace_exchange(run, dist, torch.device("cpu"))
    assert n == run.finish()
    with open(os.path.join(tmpdir, f"owned{rank}"), "wb") as f:
        f.write(run.data)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,k", [(2, 31), (3, 55)])
def test_keyspace_exchange_concatenates_to_whole(kca, orc, tmp_path, world, k):
    """cfg4: after the exchange every rank holds only its own key range, and
    the ranks' outputs concatenated in rank order are the whole stream's
    SortedKMerFile (no merge)."""
    per = 800
    mp.spawn(_ks_worker, args=(world, _free_port(), str(tmp_path), per, k), nprocs=world, join=True)
    parts = [(tmp_path / f"owned{r}").read_bytes() for r in range(world)]
    whole = kca.synth_fastq(world * per, 150, 2, genome_length=200_000)
    assert b"".join(parts) == orc.count_fastq(whole, k)
    rs = 8 * ((k + 31) // 32) + 4
    for r, p in enumerate(parts):
        assert len(p) > 0
        for i in range(0, len(p), rs):
            assert kca.owner_of(int.from_bytes(p[i:i + 8], "little"), world) == r


def test_owner_of_is_monotone_and_top_bits(kca):
    import random
    rng = random.Random(4)
    keys = sorted(rng.getrandbits(64) for _ in range(2000)) + [0, (1 << 64) - 1]
    keys.sort()
    for world in (1, 2, 3, 5, 8):
        owners = [kca.owner_of(x, world) for x in keys]
        assert owners == sorted(owners) and owners[0] == 0 and owners[-1] == world - 1
    assert all(kca.owner_of(x, 8) == x >> 61 for x in keys)
