"""Multi-process GPU coverage of bench.py's N > 1 paths with real
device contexts: 2-3 ranks on the box's one GPU, torch.distributed over gloo
(RCCL refuses two ranks on one device; the protocol and the library calls are
the ones the RCCL run makes, with the records staged through host memory).
Each rank counts its own shard of the read stream on the GPU, then
  alltoall (cfg4): kca.keyspace_exchange; every rank writes its key range as
                   its own part file; the parts in rank order == the oracle's
                   count of the whole stream;
  none           : bench.gather_runs_to_rank0 (rank 0 merges every rank's run
                   on its GPU by merge path) and rank 0 writes the file;
  files (cfg3)   : bench.host_merge_runs (every rank writes its run as a
                   SortedKMerFile; the ranks merge one key range each of all
                   the files and write it at its offset of the one output
                   file; files0: rank 0 merges them alone).
All go through bench.write_node_output, bench.Dist and bench.shard_first, at
2, 3 and 8 ranks (the node's rank count: the key-space owner is then the top 3
key bits, and the files merge is 8-way with 8 parts). The full-size cfg3 test
runs two ranks on BASELINE config 3's real shards (50M reads each)."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, tmpdir, per, k, exchange, mem):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "KC_BENCH_BACKEND": "gloo"})
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bench
    from conftest import load_pkg

    D = bench.Dist()  # torch opens the GPU first, then the library
    if exchange == "files0":
        exchange, D.files_merge = "files", "rank0"
    kca = load_pkg()
    ctx = kca.Context(kmer_length=k, line_length=150, device=D.device, gpu_memory_limit=mem)
    fq = kca.synth_fastq(per, 150, 2, genome_length=300_000, n_rate=0.001,
                         first_read=bench.shard_first(D.rank, per))
    ctx.count_fastq(fq)
    ctx.finish()
    out = os.path.join(tmpdir, "out.bin")
    nbytes = bench.write_node_output(kca, ctx, D, out, exchange)
    with open(os.path.join(tmpdir, f"bytes{rank}"), "w") as f:
        f.write(str(nbytes))
    ctx.close()
    D.dist.barrier()
    D.dist.destroy_process_group()


_CASES = [(x, w, k, mem) for x in ("alltoall", "none", "files")
          for w, k, mem in ((2, 31, 100_000_000), (3, 55, 1 << 20), (8, 31, 100_000_000))]
_CASES.append(("files0", 2, 31, 100_000_000))


@pytest.mark.parametrize("exchange,world,k,mem", _CASES)
def test_bench_multirank_output(kca, orc, tmp_path, exchange, world, k, mem):
    """(mem 1 MiB at k = 55: every rank also cuts sorted runs, merged before
    the exchange.)"""
    per = 4000 if world < 8 else 1500
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), per, k, exchange, mem), nprocs=world, join=True)
    whole = orc.count_fastq(kca.synth_fastq(world * per, 150, 2, genome_length=300_000, n_rate=0.001), k)
    rs = 8 * ((k + 31) // 32) + 4
    if exchange == "alltoall":
        parts = [(tmp_path / f"out.bin.part{r}").read_bytes() for r in range(world)]
        assert b"".join(parts) == whole
        for r, p in enumerate(parts):
            assert len(p) > 0 and int((tmp_path / f"bytes{r}").read_text()) == len(p)
            for i in range(0, len(p), rs):
                assert kca.owner_of(int.from_bytes(p[i:i + 8], "little"), world) == r
    else:
        assert (tmp_path / "out.bin").read_bytes() == whole
        written = [int((tmp_path / f"bytes{r}").read_text()) for r in range(world)]
        if exchange == "files":  # every rank wrote its key range of the one file
            assert sum(written) == len(whole) and all(b > 0 for b in written)
        else:
            assert written[0] == len(whole)


def _cfg3_worker(rank, world, port, tmpdir, per, mem):
    import json
    import time

    import numpy as np

    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "KC_BENCH_BACKEND": "gloo",
                       "LOCAL_WORLD_SIZE": str(world)})
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bench
    import oracle  # test infrastructure: the checker only
    from conftest import load_pkg

    D = bench.Dist()
    kca = load_pkg()
    k, L = 31, 150
    res = {}
    with kca.Context(kmer_length=k, line_length=L, device=D.device, gpu_memory_limit=mem) as ctx:
        # bench.py --config 3's shard of this rank: seed 3, reads [r R, (r+1) R)
        ptr, nb = ctx.synth_device(per, L, 3, 250_000_000, 0.0, bench.shard_first(D.rank, per))
        host = np.empty(nb, dtype=np.uint8)
        ctx.copy_to_host_addr(host.ctypes.data, ptr, nb)
        ctx.reset()
        assert ctx.count_fastq_device(ptr, nb) == per
        ctx.finish()
        ctx.free_device(ptr)
        st = ctx.stats()
        res["batches"], res["spilled"] = st["batches"], st["spilled_kmers"]
        # the window checksums of this shard (their sums over the shards are
        # the node's)
        res["checksum"] = oracle.window_checksum(host, k, threads=max(1, bench.merge_threads(D)))
        del host
        # cfg3's step after the count: run files + the merge shared by the
        # ranks (bench's default), then rank 0's merge of the same files
        for where, out in (("ranks", "node.bin"), ("rank0", "node0.bin")):
            tm = {}
            D.barrier_sync()
            t = time.perf_counter()
            n, mine = bench.host_merge_runs(kca, ctx, D, tmpdir, os.path.join(tmpdir, out), k, where=where,
                                            timing=tm)
            res[where] = {"s": time.perf_counter() - t, "records": n, "bytes_this_rank": mine,
                          **{key: round(v, 3) for key, v in tm.items()}}
    res["merge_threads"] = bench.merge_threads(D)
    with open(os.path.join(tmpdir, f"cfg3_rank{rank}.json"), "w") as f:
        json.dump(res, f)
    D.dist.barrier()
    D.dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.timeout(900)
def test_config3_full_shards_files_merge(kca, orc, tmp_path):
    """BASELINE config 3 as bench.py --config 3 runs it, at real shard size on
    the box's one GPU: two ranks (gloo) each count a full cfg3 shard (50M x
    150 bp, seed 3, reads [r 50M, (r+1) 50M) of the 250 Mbp genome's read
    stream) with a working set that lets both contexts share the GPU, write
    their sorted runs as SortedKMerFiles and merge them on the host: the
    default merge shared by the ranks (each merges one key range of both files
    and writes it at its offset of the one output file), then rank 0's merge
    of the same files. Both outputs are byte-equal; the output's window
    checksums (records, count-weighted) equal the sums of the two shards'
    window checksums over every valid window (full-size parity property);
    keys strictly ascending. The merge times go to the test's log."""
    import json

    import numpy as np

    world, per, mem = 2, 50_000_000, 90 << 30
    mp.spawn(_cfg3_worker, args=(world, _free_port(), str(tmp_path), per, mem), nprocs=world, join=True)
    res = [json.loads((tmp_path / f"cfg3_rank{r}.json").read_text()) for r in range(world)]
    print("cfg3 full shards:", json.dumps(res))
    a = {"h1": 0, "h2": 0, "valid": 0, "windows": 0, "hole": False}
    for r in res:
        c = r["checksum"]
        a["h1"] = (a["h1"] + c["h1"]) & ((1 << 64) - 1)
        a["h2"] = (a["h2"] + c["h2"]) & ((1 << 64) - 1)
        a["valid"] += c["valid"]
        a["windows"] += c["windows"]
        a["hole"] |= c["hole"]
        assert r["spilled"] == 0
    assert a["windows"] == world * per * (150 - 31 + 1)
    out, out0 = tmp_path / "node.bin", tmp_path / "node0.bin"
    assert out.stat().st_size == out0.stat().st_size
    recs = np.fromfile(str(out), dtype=np.uint8)
    b = orc.records_checksum(recs, 31, threads=16)
    assert b["unordered"] == 0
    assert b["count"] == a["valid"]
    assert (b["h1"], b["h2"]) == (a["h1"], a["h2"])
    n = recs.size // 12
    assert all(r["ranks"]["records"] == n for r in res) and res[0]["rank0"]["records"] == n
    assert sum(r["ranks"]["bytes_this_rank"] for r in res) == recs.size
    for lo in range(0, recs.size, 1 << 30):
        assert np.array_equal(recs[lo:lo + (1 << 30)], np.fromfile(str(out0), dtype=np.uint8, count=1 << 30,
                                                                   offset=lo))
