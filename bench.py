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
                    [--min-read-length M]

--min-read-length M (0 < M < L): variable-length input (SURVEY §8f row 1,
KC_FLAG_VARLEN): read i keeps its first M..L bases (generator in
kc_synth.h); k-mers per step = the reads' own windows (kc_stats.windows).

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


def cpu_baseline(kca, reads, L, k, genome, seed, first, threads=None):
    """The CPU port of the reference pipeline (oracle refcpu) on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: timed as the CPU baseline only

    if threads is None:
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


def cpu_baseline_varlen(kca, reads, L, lmin, k, genome, seed):
    """Variable-length input has no reference pipeline to port (the reference
    concatenates reads without separators): the CPU baseline is the oracle's
    per-read statement (spec form, one thread, sorted output) on a sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: timed as the CPU baseline only

    fq = kca.synth_fastq(reads, L, seed, genome_length=genome, min_read_length=lmin)
    windows = sum(max(0, len(s) - k + 1) for s in oracle.fastq_sequences(fq))
    t0 = time.perf_counter()
    out = oracle.count_fastq_varlen(fq, k)
    dt = time.perf_counter() - t0
    return {"value": windows / dt, "unit": "k-mers/s", "cores": 1, "kind": "port",
            "sample": f"{reads} reads of {lmin}..{L} bp of the same workload ({windows} k-mers, "
                      f"{len(out) // (8 * ((k + 31) // 32) + 4)} distinct): oracle count_fastq_varlen (each read "
                      f"as a reference chunk of its own length, spec form, sorted output); 1 thread, {dt:.2f} s"}


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
    ap.add_argument("--engine", default="auto", choices=["auto", "skm", "partition", "table"])
    ap.add_argument("--cpu-reads", type=int, default=2_000_000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--min-read-length", type=int, default=0,
                    help="variable-length reads of M..L bases (KC_FLAG_VARLEN); 0 = every read has L bases")
    ap.add_argument("--exchange", default="alltoall", choices=["alltoall", "none"],
                    help="N>1: key-space all-to-all (cfg4) or read-shard only (cfg3); ignored at N=1")
    args = ap.parse_args()
    preset = {2: dict(reads=50_000_000, k=31, genome=250_000_000, seed=2, mem=160 << 30),
              5: dict(reads=20_000_000, k=55, genome=0, seed=5, mem=72 << 30)}[args.config]
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
    varlen = 0 < args.min_read_length < L
    ctx = kca.Context(kmer_length=k, line_length=L, device=device, gpu_memory_limit=args.mem, engine=args.engine,
                      variable_length=varlen)
    first = shard_first(rank, args.reads)
    ptr, nbytes = ctx.synth_device(args.reads, L, args.seed, args.genome, 0.0, first,
                                   args.min_read_length if varlen else 0)

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
    dedup_ms = 0.0
    n_rec = 0
    for _ in range(args.steps):
        n_rec = step()
        st = ctx.stats()
        insert_ms += st["insert_ms"]
        launches += st["insert_launches"]
        finish_ms += st["finish_ms"]
        decode_ms += st["decode_ms"]
        part_ms = [a + b for a, b in zip(part_ms, st["part_ms"])]
        dedup_ms += st.get("dedup_ms", 0.0)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    st = ctx.stats()
    if dist is not None:
        import torch
        dev = torch.device("cpu") if dist.get_backend() == "gloo" else torch.device("cuda", torch.cuda.current_device())
        elapsed = max_over_ranks(dist, elapsed, dev)
    # variable-length reads: the reads' own windows (ctx stats are per step)
    windows_per_gpu = st["windows"] if varlen else args.reads * (L - k + 1)
    if dist is not None and varlen:
        import torch
        dev = torch.device("cpu") if dist.get_backend() == "gloo" else torch.device("cuda", torch.cuda.current_device())
        t = torch.tensor([float(windows_per_gpu)], dtype=torch.float64, device=dev)
        dist.all_reduce(t)
        windows_per_gpu = t.item() / world
    total_kmers = windows_per_gpu * world * args.steps
    value = total_kmers / elapsed

    # Rooflines. Each main kernel of the partition engine is priced by its own
    # algorithmic HBM bytes: P2 reads the encoded reads
    # (6 B per 16 bases) and writes 8W B per key; the P3 scatter reads and
    # writes 8W B per key; P5 reads 8W B per key and writes 8W+4 B per
    # distinct record. `roofline` is the one with the longest launch; each
    # achieved = algorithmic bytes per launch / its HIP-event launch time on
    # the ctx stream. `path_achieved` is SURVEY §8d's whole-path figure:
    # k-mers/s per GPU x (FASTQ bytes per k-mer + 8W + 8).
    W = (k + 31) // 32
    G = (L + 15) // 16
    steps = args.steps
    windows_step = windows_per_gpu
    keys_step = st["keys"] or windows_step  # ctx stats are per step (reset at each step)
    recs_step = st["output_records"]
    kernels = {}
    used = st.get("engines_used", 0)
    if used & 1:
        # super-k-mer engine: F reads the encoded reads (6 B per 16 bases) and
        # writes the records (8(W+1) B each); each of the two grouping scatters
        # reads and writes every record; P5 reads the records and writes the
        # distinct (key, count) records
        # (S: two scatter launches per batch, each over all records; P5: the
        # cardinality sample and the main launch together are one pass over
        # the records, priced per batch)
        rec_step = st["keys"] or 1  # records handed out by F per step
        rb = 8 * (W + 1)
        # F3 (skm_front3_k<k>, a lane per read) covers W = 1, 19 <= k <= 32
        # with rows of <= 40 KiB per wave; F2 (skm_front2_k<1, k>) W = 1,
        # 18 <= k <= 32 with at most 64 8-window chunks per read; the generic F
        # otherwise
        nw = L - k + 1
        ng = max((L + 15) // 16 + 1, (nw - 1) // 16 + 5) | 1
        f3 = (W == 1 and 19 <= k <= 32 and (320 + 64) * 8 + 256 + 256 * ng <= 40 * 1024
              and not os.environ.get("KC_NO_F3"))
        f2 = W == 1 and 18 <= k <= 32 and (nw + 7) // 8 <= 64 and not os.environ.get("KC_NO_F2")
        fname = f"skm_front3_k<{k}>" if f3 else (f"skm_front2_k<1,{k}>" if f2 else f"skm_front_k<{W}>")
        dd_step = st.get("dedup_records", 0)  # ctx stats are per step
        specs = [
            ("F", fname, part_ms[1], launches, windows_step, "k-mers",
             (G * 6) / max(1, L - k + 1) + rb * rec_step / windows_step),
            ("S", f"rp_scatter_k<{W + 1},false>", part_ms[2], 2 * steps * st["batches"], 2 * rec_step, "records",
             2 * rb + 1),
        ]
        if dedup_ms > 0:
            # P5a reads every record and writes each distinct one with its
            # multiplicity; P5 then reads the distinct records and writes the
            # distinct (key, count) records
            specs += [
                ("P5a", "count_rec_k", dedup_ms, steps * st["batches"], rec_step, "records",
                 rb + (rb + 4) * dd_step / rec_step),
                ("P5", f"count_skm_k<{W}>", part_ms[4], steps * st["batches"], max(1, dd_step), "distinct records",
                 (rb + 4) + (8 * W + 4) * recs_step / max(1, dd_step)),
            ]
        else:
            specs.append(("P5", f"count_skm_k<{W}>", part_ms[4], steps * st["batches"], rec_step, "records",
                          rb + (8 * W + 4) * recs_step / rec_step))
    elif used & 2:
        p5_per_step = max(1, st["p5_launches"])
        specs = [
            ("P2", f"count_front<{W},2,true,1024>", part_ms[1], launches, windows_step,
             "k-mers", (G * 6) / max(1, L - k + 1) + 8 * W),
            ("P3", f"p3_scatter_k<{W}>", part_ms[2], steps * st["batches"], keys_step, "keys", 16 * W),
            ("P5", f"count_buckets<{W}>", part_ms[4], steps * p5_per_step, keys_step, "keys",
             8 * W + (8 * W + 4) * recs_step / max(1, keys_step)),
        ]
    else:
        specs = [("insert", f"count_front<{W},0,false,256>", insert_ms, launches, windows_step, "k-mers",
                  nbytes / windows_per_gpu + 8 * W + 8)]
    for tag, name, ms_total, nl, units_step, unit_name, bpu in specs:
        nl = max(1, nl)
        avg = ms_total / nl
        units = units_step * steps / nl
        ach = bpu * units / (avg / 1e3) / 1e9 if avg > 0 else 0.0
        kernels[tag] = {"kernel": name, "avg_launch_ms": round(avg, 3), "units_per_launch": int(units),
                        "unit": unit_name, "algorithmic_bytes_per_unit": round(bpu, 3),
                        "achieved": round(ach, 2), "frac": round(ach / HBM_PEAK_GBS, 4)}
    dom = max(kernels, key=lambda t: kernels[t]["avg_launch_ms"])
    d = kernels[dom]
    traffic = load_traffic()
    t_bytes = None
    # (the committed PMC summary is of the fixed-length cfg2 run)
    if traffic and not varlen and traffic.get("reads_per_gpu") == args.reads and traffic.get("k") == k:
        t_bytes = traffic.get("kernels", {}).get(d["kernel"].replace(" ", ""), {}).get("bytes_per_launch")
    b_path = nbytes / windows_per_gpu + 8 * W + 8
    step_s = elapsed / args.steps
    path_achieved = b_path * windows_per_gpu / step_s / 1e9
    roofline = {"bound": "hbm", "achieved": d["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": d["frac"], "traffic": t_bytes, "kernel": f"{dom}: {d['kernel']}",
                "avg_launch_ms": d["avg_launch_ms"], "units_per_launch": d["units_per_launch"],
                "unit_of_work": d["unit"], "algorithmic_bytes_per_unit": d["algorithmic_bytes_per_unit"],
                "path_achieved": round(path_achieved, 2), "path_frac": round(path_achieved / HBM_PEAK_GBS, 4),
                "path_bytes_per_kmer": round(b_path, 3), "kernels": kernels}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and varlen:
        cpu = cpu_baseline_varlen(kca, max(1, args.cpu_reads // 20), L, args.min_read_length, k, args.genome,
                                  args.seed)
    elif rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(kca, args.cpu_reads, L, k, args.genome, args.seed, 0)
        t1 = cpu_baseline(kca, max(1, args.cpu_reads // 10), L, k, args.genome, args.seed, 0, threads=1)
        cpu["value_t1"] = t1["value"]
        cpu["sample_t1"] = t1["sample"]

    src = (f"sampled from a {args.genome} bp random genome" if args.genome else "of iid uniform bases")
    lens = f"{args.min_read_length}..{L} bp (variable-length, KC_FLAG_VARLEN)" if varlen else f"{L} bp"
    base = (f"k={k}, {args.reads} x {lens} reads per GPU {src} (seed {args.seed}), FASTQ in HBM, "
            f"in-HBM count")
    if world == 1:
        workload, parallelism = f"cfg{args.config}{'v' if varlen else ''}: " + base, "single GPU"
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
            "breakdown_ms_per_step": {"p2_scatter": insert_ms / args.steps, "fastq_index": decode_ms / args.steps,
                                      "finish": finish_ms / args.steps,
                                      "exchange_rank0": xch_ms[0] / args.steps,
                                      "partition_passes": [round(x / args.steps, 3) for x in part_ms],
                                      "p5a_dedup": round(dedup_ms / args.steps, 3)},
            "engine": args.engine, "engines_used": {1: "skm", 2: "key-prefix partition", 3: "skm + key-prefix",
                                                    4: "table"}.get(st.get("engines_used", 0), str(st.get("engines_used"))),
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
