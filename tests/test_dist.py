"""Multi-process (world size 2, gloo on the CPU) coverage of the read-shard
path of bench.py / the CLI: disjoint shards whose sorted runs, k-way merged
on the host, equal the count of the whole read stream; the step time is the
max over ranks. The per-shard counts come from the CPU oracle here (no GPU in
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


def _worker(rank, world, port, tmpdir, per, k):
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
    with open(os.path.join(tmpdir, f"run{rank}"), "wb") as f:
        f.write(oracle.count_fastq(fq, k))
    t = bench.max_over_ranks(dist, float(rank + 1), torch.device("cpu"))
    with open(os.path.join(tmpdir, f"t{rank}"), "w") as f:
        f.write(repr(t))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("k", [31, 55])
def test_read_shard_merge_equals_whole(kca, orc, tmp_path, k):
    world, per = 2, 3000
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), per, k), nprocs=world, join=True)
    runs = [str(tmp_path / f"run{r}") for r in range(world)]
    out = tmp_path / "merged.bin"
    kca.merge_files(runs, str(out), k)
    whole = kca.synth_fastq(world * per, 150, 2, genome_length=400_000)
    assert out.read_bytes() == orc.count_fastq(whole, k)
    for r in range(world):
        assert float((tmp_path / f"t{r}").read_text()) == float(world)


def test_shards_are_disjoint_and_cover(kca):
    import bench
    per = 1000
    parts = [kca.synth_fastq(per, 100, 7, first_read=bench.shard_first(r, per)) for r in range(3)]
    assert b"".join(parts) == kca.synth_fastq(3 * per, 100, 7)
