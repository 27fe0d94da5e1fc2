#!/usr/bin/env python3
"""Benchmark of the k-mer count hot path (BASELINE.json metric).

Workload (BASELINE.json configs[1], SURVEY §8d cfg 2): k=31, 150 bp reads
sampled from a 250 Mbp random genome (splitmix64 generator, seed 2), 50M reads
per GPU, FASTQ text resident in HBM (generated on the device, untimed), in-HBM
hash table only. One step = one full count of the GPU's reads: clear the table,
index the FASTQ block (K1), encode + window + insert every k-mer (K2), compact
and radix-sort the table into SortedKMerFile records (K3/K4). N GPUs: one
process per GPU, each counts its own disjoint 50M-read shard (weak scaling),
then by default (`--exchange alltoall`) the ranks exchange
their sorted (key, count) records by key-space owner with one RCCL
all-to-all and each merges what it receives on the device, so the node's
SortedKMerFile is the concatenation of the ranks' runs — all inside the timed
step. `--exchange none` is the read-shard mode (cfg3): no collective, the
per-GPU runs are left for the host k-way merge (not timed).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--reads R] [--exchange alltoall|none] [--no-cpu]

Prints one JSON line on rank 0 (contract in the task statement).
"""
import argparse
import importlib.util
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))

METRIC = "k-mers/s (whole node) at k=31, 150bp reads; bit-exact vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def load_pkg():
    spec = importlib.util.spec_from_file_location("kmer_counter_amd", os.path.join(ROOT, "kmer-counter_amd",
                                                                                   "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["kmer_counter_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def cpu_baseline(kca, reads, L, k, genome, seed, first):
    """The CPU port of the reference pipeline (oracle refcpu) on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: timed as the CPU baseline only

    threads = min(16, os.cpu_count() or 1)
    fq = kca.synth_fastq(reads, L, seed, genome_length=genome, first_read=first)
    t0 = time.perf_counter()
    distinct, windows = oracle.refcpu_count_only(fq, k, gpu_memory_limit=100000000, threads=threads)
    dt = time.perf_counter() - t0
    return {"value": windows / dt, "unit": "k-mers/s", "cores": threads, "kind": "port",
            "sample": f"{reads} reads x {L} bp of the same workload ({windows} k-mers, {distinct} distinct): "
                      f"oracle refcpu = the reference count path on the CPU (readData chunking at "
                      f"gpuMemoryLimit=1e8, bitEncode/extractKMers/reduceKMers restated, hash insert into a "
                      f"sharded-lock table standing in for TBB); timed up to the complete table, as the "
                      f"reference's DumpResults writes in hash order; {threads} threads, {dt:.2f} s"}


def shard_first(rank: int, reads_per_gpu: int) -> int:
    """Read-shard: rank r counts reads [r*R, (r+1)*R) of the
    one synthetic read stream; shards are disjoint and their union is the
    whole stream."""
    return rank * reads_per_gpu


def max_over_ranks(dist, value: float, device) -> float:
    """The step time of a multi-rank run is the slowest rank's."""
    if dist is None:
        return value
    import torch

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def load_traffic():
    p = os.path.join(ROOT, "profiles", "pmc_count_kmers.json")
    if not os.path.exists(p):
        return None
    try:
        return json.load(open(p))
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=2, choices=[2, 5],
                    help="SURVEY §8d preset: 2 = k=31, 50M x 150 bp from a 250 Mbp genome (the metric's "
                         "config); 5 = k=55, 20M x 150 bp iid reads (~1.9e9 distinct, high cardinality)")
    ap.add_argument("--reads", type=int, default=None, help="reads per GPU")
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--L", type=int, default=150)
    ap.add_argument("--genome", type=int, default=None, help="0 = iid uniform reads")
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--mem", type=int, default=None, help="gpuMemoryLimit per GPU (bytes)")
    ap.add_argument("--engine", default="partition", choices=["partition", "table"])
    ap.add_argument("--cpu-reads", type=int, default=2_000_000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--exchange", default="alltoall", choices=["alltoall", "none"],
                    help="N>1: key-space all-to-all (cfg4) or read-shard only (cfg3); ignored at N=1")
    args = ap.parse_args()
    preset = {2: dict(reads=50_000_000, k=31, genome=250_000_000, seed=2, mem=160 << 30),
              5: dict(reads=20_000_000, k=55, genome=0, seed=5, mem=64 << 30)}[args.config]
    for key, v in preset.items():
        if getattr(args, key) is None:
            setattr(args, key, v)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist_mod

        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        # nccl (= RCCL) by default; KC_BENCH_BACKEND=gloo rehearses several
        # ranks on one GPU (RCCL refuses duplicate devices)
        dist_mod.init_process_group(backend=os.environ.get("KC_BENCH_BACKEND", "nccl"))
        dist = dist_mod

    kca = load_pkg()
    k, L = args.k, args.L
    device = local
    if world > 1:
        import torch
        device = local % max(1, torch.cuda.device_count())  # rehearsal: ranks may share a GPU
    ctx = kca.Context(kmer_length=k, line_length=L, device=device, gpu_memory_limit=args.mem, engine=args.engine)
    first = shard_first(rank, args.reads)
    ptr, nbytes = ctx.synth_device(args.reads, L, args.seed, args.genome, 0.0, first)

    exchange = args.exchange if world > 1 else "none"
    xdev = None
    if exchange == "alltoall":
        import torch
        xdev = torch.device("cpu") if dist.get_backend() == "gloo" else torch.device("cuda", device)
    xch_ms = [0.0]

    def step():
        ctx.reset()
        ctx.count_fastq_device(ptr, nbytes)
        n = ctx.finish()
        if exchange == "alltoall":
            t = time.perf_counter()
            n = kca.keyspace_exchange(ctx, dist, xdev)
            xch_ms[0] += (time.perf_counter() - t) * 1e3
        return n

    def barrier_sync():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier_sync()
    xch_ms[0] = 0.0
    t0 = time.perf_counter()
    insert_ms = 0.0
    launches = 0
    finish_ms = 0.0
    decode_ms = 0.0
    part_ms = [0.0] * 5
    n_rec = 0
    for _ in range(args.steps):
        n_rec = step()
        st = ctx.stats()
        insert_ms += st["insert_ms"]
        launches += st["insert_launches"]
        finish_ms += st["finish_ms"]
        decode_ms += st["decode_ms"]
        part_ms = [a + b for a, b in zip(part_ms, st["part_ms"])]
    barrier_sync()
    elapsed = time.perf_counter() - t0
    st = ctx.stats()
    if dist is not None:
        import torch
        dev = torch.device("cpu") if dist.get_backend() == "gloo" else torch.device("cuda", torch.cuda.current_device())
        elapsed = max_over_ranks(dist, elapsed, dev)
    windows_per_gpu = args.reads * (L - k + 1)
    total_kmers = windows_per_gpu * world * args.steps
    value = total_kmers / elapsed

    # roofline of the dominant kernel (count_kmers): algorithmic bytes per k-mer
    # = FASTQ bytes per k-mer (read once) + 8W key bytes + 8 count bytes (read +
    # write of the u32); per launch = that x the launch's k-mers.
    W = (k + 31) // 32
    b_per_kmer = nbytes / windows_per_gpu + 8 * W + 8
    avg_launch_ms = insert_ms / max(1, launches)
    kmers_per_launch = windows_per_gpu * args.steps / max(1, launches)
    achieved = b_per_kmer * kmers_per_launch / (avg_launch_ms / 1e3) / 1e9
    traffic = load_traffic()
    kernel = f"count_front<{W},SINK_SCATTER> (P2)" if args.engine == "partition" else f"count_front<{W},SINK_TABLE>"
    step_s = elapsed / args.steps
    path_achieved = b_per_kmer * windows_per_gpu / step_s / 1e9
    t_bytes = None
    if traffic and traffic.get("kernel") == kernel and traffic.get("reads_per_gpu") == args.reads:
        t_bytes = traffic.get("bytes_per_launch")
    roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": t_bytes,
                "kernel": kernel, "avg_launch_ms": round(avg_launch_ms, 3),
                "algorithmic_bytes_per_kmer": round(b_per_kmer, 3), "kmers_per_launch": int(kmers_per_launch),
                "path_achieved": round(path_achieved, 2), "path_frac": round(path_achieved / HBM_PEAK_GBS, 4)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(kca, args.cpu_reads, L, k, args.genome, args.seed, 0)

    src = (f"sampled from a {args.genome} bp random genome" if args.genome else "of iid uniform bases")
    base = (f"k={k}, {args.reads} x {L} bp reads per GPU {src} (seed {args.seed}), FASTQ in HBM, "
            f"in-HBM count")
    if world == 1:
        workload, parallelism = f"cfg{args.config}: " + base, "single GPU"
    elif exchange == "alltoall":
        workload = (f"cfg4 pattern at {world} GPUs: " + base + "; key-space all-to-all of the sorted (key, count) "
                    "records + per-GPU merge inside the step (output = concatenation of the ranks' runs)")
        parallelism = f"read-shard count + key-space all-to-all x{world}"
    else:
        workload = f"cfg3 pattern at {world} GPUs: " + base + "; per-GPU sorted runs, host merge not timed"
        parallelism = f"read-shard x{world}"
    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "k-mers/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": workload, "k": k, "read_length": L, "reads_per_gpu": args.reads,
                       "parallelism": parallelism, "gpu_memory_limit": args.mem},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "breakdown_ms_per_step": {"insert": insert_ms / args.steps, "fastq_index": decode_ms / args.steps,
                                      "finish": finish_ms / args.steps,
                                      "exchange_rank0": xch_ms[0] / args.steps,
                                      "partition_passes": [round(x / args.steps, 3) for x in part_ms]},
            "engine": args.engine,
            "distinct_kmers_per_gpu": n_rec, "spilled_kmers": st["spilled_kmers"],
        }
        print(json.dumps(line), flush=True)
    ctx.free_device(ptr)
    ctx.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
