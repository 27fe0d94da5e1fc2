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
                   SortedKMerFile, rank 0 k-way merges them on the host).
Both go through bench.write_node_output, bench.Dist and bench.shard_first."""
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


@pytest.mark.parametrize("exchange", ["alltoall", "none", "files"])
@pytest.mark.parametrize("world,k,mem", [(2, 31, 100_000_000), (3, 55, 1 << 20)])
def test_bench_multirank_output(kca, orc, tmp_path, exchange, world, k, mem):
    """(mem 1 MiB at k = 55: every rank also cuts sorted runs, merged before
    the exchange.)"""
    per = 4000
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
        assert int((tmp_path / "bytes0").read_text()) == len(whole)
