#!/usr/bin/env python3
"""Benchmark of the k-mer count path (BASELINE.json metric).

Workload (BASELINE.json configs[1], cfg 2): k=31, 50M x 150 bp reads per GPU
sampled from a 250 Mbp random genome (splitmix64 generator, seed 2),
generated in HBM before timing.

`value` (the task contract: inputs resident in HBM when the timed region
starts) is the device-resident rate: one step = kc_reset; kc_count_fastq_device
(GPU FASTQ decode + 2-bit encode + counting) ; kc_finish (the sorted
SortedKMerFile records in HBM); at N > 1 also the exchange below. The timed
region is exactly K such steps after W warmup steps, bracketed by barrier +
device synchronize, max over ranks. `roofline` prices the step's dominant
kernel and `path_frac` the whole step (SURVEY §8d bytes per k-mer).

Sub-objects of the same line (same input, same context):
  end_to_end      : SURVEY §8d's PCIe-inclusive rate, from the first FASTQ byte
                    of a file (page cache) to the SortedKMerFile closed:
                    kc_count_file (pread into pinned blocks, PCIe upload, GPU
                    decode, count), kc_finish, kc_write_output. Each step writes
                    a new output file, deleted right after the step (outside
                    its interval); the input file is written untimed into the
                    first of $TMPDIR, /tmp, /dev/shm, ... with room for it
                    (statvfs). N = 1 by default (--e2e at N > 1);
  host_memory     : the FASTQ in (pageable) host memory, one kc_count_fastq
                    call, output file written;
  reference_chunks: the same reads as the reference's chunks (concatenated
                    sequences of 7.8 MB at gpuMemoryLimit=1e8,
                    KMerCounter.cpp:193-212) through ~960 kc_count_chunk calls
                    vs one kc_count_chunk call of all of them, output in HBM;
  cpu_baseline    : the CPU port of the reference pipeline on a bounded sample
                    (rank 0, after the timed region, at every N).

N GPUs (one process per GPU, torch.distributed; RCCL = backend nccl): rank r
counts reads [r R, (r+1) R) of the one read stream (weak scaling).
  --exchange alltoall (default at N > 1): the sorted runs are
    exchanged by key-space owner (RCCL all-to-all) and merged on the device;
    rank r owns the r-th key range (in the e2e leg it writes it as its own part
    file); the parts in rank order are the node's SortedKMerFile.
  --exchange files (default of --config 3; cfg3 as BASELINE.json states it:
    read-shard, no RCCL, host KMerFileMerger k-way merge): every rank writes
    its sorted run as a SortedKMerFile, then every rank merges one key range
    of all N files on the host (kc_merge_part_create: one k-way level, the
    range cut into sub-ranges merged by the rank's share of the CPUs) and
    writes it at its offset of the one output file (--files-merge rank0:
    rank 0 merges everything, kc_merge_files); the step includes the run
    files and the merge.
  --exchange none (read-shard variant over RCCL): the runs are gathered to
    rank 0's GPU (RCCL) and merged there (device merge path), rank 0 writes
    the file.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5] [--reads R]
                    [--value device|e2e] [--e2e|--no-e2e] [--no-cpu] [--no-variants] [--workdir DIR]
                    [--exchange alltoall|none|files]
                    [--min-read-length M]

Prints one JSON line on rank 0 (contract in the task statement); a failure
prints one line with an `error` field instead and exits 1.
"""
import argparse
import importlib.util
import json
import os
import sys
import threading
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


def usable_cpus():
    """CPUs this process may use: the affinity mask, capped by the cgroup CPU
    quota (the GPU box shows 256 CPUs but grants 16)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(kca, reads, L, k, genome, seed, threads):
    """The CPU port of the reference pipeline (oracle refcpu) on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: timed as the CPU baseline only

    fq = kca.synth_fastq(reads, L, seed, genome_length=genome)
    t0 = time.perf_counter()
    distinct, windows = oracle.refcpu_count_only(fq, k, gpu_memory_limit=100000000, threads=threads)
    dt = time.perf_counter() - t0
    return windows / dt, windows, distinct, dt


def cpu_baselines(kca, reads, L, k, genome, seed):
    cores = usable_cpus()
    v, win, distinct, dt = cpu_baseline(kca, reads, L, k, genome, seed, cores)
    v1, _, _, dt1 = cpu_baseline(kca, reads, L, k, genome, seed, 1)
    return {"value": v, "unit": "k-mers/s", "cores": cores, "kind": "port",
            "sample": f"{reads} reads x {L} bp of the same workload ({win} k-mers, {distinct} distinct): oracle "
                      f"refcpu = the reference count path on the CPU (readData chunking at gpuMemoryLimit=1e8, "
                      f"bitEncode/extractKMers/reduceKMers restated, hash insert into a sharded-lock table standing "
                      f"in for TBB), timed up to the complete table as the reference's DumpResults writes in hash "
                      f"order; {cores} threads = the CPUs this process may use (cgroup quota of the "
                      f"{os.cpu_count()} visible), {dt:.2f} s; same sample at 1 thread: {dt1:.2f} s",
            "value_t1": v1}


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
    return {"value": windows / dt, "unit": "k-mers/s", "cores": 1, "kind": "oracle-spec",
            "sample": f"{reads} reads of {lmin}..{L} bp of the same workload ({windows} k-mers, "
                      f"{len(out) // (8 * ((k + 31) // 32) + 4)} distinct): the oracle's specification form "
                      f"(count_fastq_varlen: each read as a reference chunk of its own length, sorted output), not "
                      f"a port of a reference pipeline (the reference has none for mixed read lengths); 1 thread, "
                      f"{dt:.2f} s"}


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


class Dist:
    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        self.device = self.local
        if self.world > 1:
            import torch
            import torch.distributed as dist_mod

            ndev = max(1, torch.cuda.device_count())
            self.device = self.local % ndev  # rehearsal: ranks may share a GPU
            torch.cuda.set_device(self.device)
            # nccl (= RCCL) by default; KC_BENCH_BACKEND=gloo rehearses several
            # ranks on one GPU (RCCL refuses duplicate devices)
            dist_mod.init_process_group(backend=os.environ.get("KC_BENCH_BACKEND", "nccl"))
            self.dist = dist_mod

    def xdev(self):
        import torch
        if self.dist.get_backend() == "gloo":
            return torch.device("cpu")
        return torch.device("cuda", self.device)

    def barrier_sync(self):
        if self.dist is not None:
            import torch
            gpu = torch.cuda.is_available()
            if gpu:
                torch.cuda.synchronize()
            self.dist.barrier()
            if gpu:
                torch.cuda.synchronize()

    def max(self, v):
        return max_over_ranks(self.dist, float(v), self.xdev() if self.dist is not None else None)

    def sum(self, v):
        if self.dist is None:
            return v
        import torch
        t = torch.tensor([float(v)], dtype=torch.float64, device=self.xdev())
        self.dist.all_reduce(t)
        return float(t.item())

    def all_gather_int(self, v):
        if self.dist is None:
            return [v]
        import torch
        t = torch.tensor([int(v)], dtype=torch.int64, device=self.xdev())
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [int(x.item()) for x in out]


def gather_runs_to_rank0(kca, ctx, D):
    """cfg3 (read-shard, --exchange none): every rank's sorted run to rank 0's
    GPU (one all-to-all in which only rank 0 receives), merged there by merge
    path (kc_merge_runs_device). Returns rank 0's merged record count."""
    import torch

    dev = D.xdev()
    n = ctx.finish()
    rs = ctx.rs
    send = torch.empty(n * rs, dtype=torch.uint8, device=dev)
    ctx.export_records(send)
    counts = D.all_gather_int(n)
    recv_sizes = [c * rs for c in counts] if D.rank == 0 else [0] * D.world
    send_sizes = [n * rs if o == 0 else 0 for o in range(D.world)]
    recv = torch.empty(sum(recv_sizes), dtype=torch.uint8, device=dev)
    D.dist.all_to_all_single(recv, send, recv_sizes, send_sizes)
    if recv.is_cuda:
        torch.cuda.current_stream(recv.device).synchronize()
    del send
    if D.rank == 0:
        return ctx.merge_runs(recv, counts)
    return 0


# --exchange files, shared merge: key-range parts per rank (rounds, at least
# this many); the last round's write is the only one not overlapped with merging
FILES_MERGE_ROUNDS = 4


def merge_threads(D):
    """Host threads one rank may use: the usable CPUs shared by the node's local ranks."""
    local = int(os.environ.get("LOCAL_WORLD_SIZE", str(D.world)))
    return max(1, usable_cpus() // max(1, local))


def host_merge_runs(kca, ctx, D, run_dir, out_path, k, threads=0, where="ranks", timing=None):
    """cfg3 as BASELINE.json states it (read-shard, no RCCL, host
    KMerFileMerger k-way merge; KMerFileMergeHandler.cpp:41-123,
    KMerFileMerger.cpp:49-96): every rank writes its sorted run as a
    SortedKMerFile into run_dir (kc_write_output), then the N run files are
    merged into out_path.
      where="ranks" (default): the merge is shared by the ranks, as the
        reference runs its merge groups concurrently: the key space is cut into
        N x FILES_MERGE_ROUNDS ranges (kc_merge_part_create; the boundary keys
        come from the files by one deterministic rule, so no rank sends another
        any records) and rank r merges ranges r, r + N, ... in key order; after
        each round the ranks all-gather their merged sizes (one integer each
        over the process group: control, not data) and each writes its range at
        its offset of the one output file (kc_merge_part_write) while it merges
        its next one.
      where="rank0": rank 0 merges all N files alone (kc_merge_files).
    `threads` per rank (default: the usable CPUs shared by the node's ranks).
    The barriers only order the ranks. The files are overwritten in place each
    step. `timing` (a dict, optional) accumulates this rank's seconds in
    run_file / merge / write. Returns (records in the node's output, output
    bytes this rank wrote)."""
    tm = timing if timing is not None else {}
    t0 = time.perf_counter()
    run = os.path.join(run_dir, f"kc_cfg3.run{D.rank}")
    ctx.write_output(run)
    D.barrier_sync()
    t1 = time.perf_counter()
    tm["run_file"] = tm.get("run_file", 0.0) + (t1 - t0)
    runs = [os.path.join(run_dir, f"kc_cfg3.run{r}") for r in range(D.world)]
    thr = threads or merge_threads(D)
    if where == "rank0":
        n, mine = 0, 0
        if D.rank == 0:
            kca.merge_files(runs, out_path, k, D.world, threads or usable_cpus())
            mine = os.path.getsize(out_path)
            n = mine // ctx.rs
        D.barrier_sync()
        tm["merge"] = tm.get("merge", 0.0) + (time.perf_counter() - t1)
        return n, mine
    # the key space in world x R parts, rank r merging parts r, r + N, ... in
    # key order (rounds): after each round the ranks all-gather the round's
    # sizes, which fixes the round's offsets, and a rank writes its part of
    # round i (a background thread; the library releases the GIL) while it
    # merges its part of round i + 1, so only the last round's write is not
    # overlapped
    R = max(FILES_MERGE_ROUNDS, 16 // D.world)  # (the last round's part: ~1/16 of the output at any N)
    parts = D.world * R
    total, mine = 0, 0
    writing = None  # (thread, part, errors) of the previous round
    t_merge = 0.0

    def finish_write(w):
        w[0].join()
        w[1].close()
        if w[2]:
            raise w[2][0]

    for i in range(R):
        t = time.perf_counter()
        part = kca.MergePart(runs, k, i * D.world + D.rank, parts, thr)
        sizes = D.all_gather_int(part.nbytes)
        t_merge += time.perf_counter() - t
        off = total + sum(sizes[:D.rank])
        total += sum(sizes)
        if writing is not None:
            finish_write(writing)
        errs = []

        def write(p=part, o=off, cut=total if i == R - 1 else 0, e=errs):
            try:
                p.write(out_path, o, cut)
            except Exception as ex:  # raised again on the main thread
                e.append(ex)

        th = threading.Thread(target=write)
        th.start()
        writing = (th, part, errs)
        mine += part.nbytes
    t2 = time.perf_counter()
    finish_write(writing)
    D.barrier_sync()
    t3 = time.perf_counter()
    tm["merge"] = tm.get("merge", 0.0) + t_merge
    tm["write"] = tm.get("write", 0.0) + (t3 - t2)
    return total // ctx.rs, mine


def write_node_output(kca, ctx, D, path, exchange):
    """The node's SortedKMerFile from the ranks' finished runs (see the module
    docstring). Returns output bytes written by this rank.

    N > 1, key-space exchange: rank r owns the r-th key range after the
    exchange and writes it as its own part file `path.part<r>`; the parts in
    rank order are the node's SortedKMerFile (the final merge is a
    concatenation). One file per rank because buffered writes into one file
    are serialised by its inode (~10 GB/s on the GPU box), separate files are
    not. N > 1, read-shard: rank 0 merges every rank's run on its GPU and
    writes the one file."""
    if D.world == 1:
        ctx.write_output(path)
        return ctx.finish() * ctx.rs
    if exchange == "alltoall":
        n = kca.keyspace_exchange(ctx, D.dist, D.xdev())
        ctx.write_output(f"{path}.part{D.rank}")
        return n * ctx.rs
    if exchange == "files":
        _, mine = host_merge_runs(kca, ctx, D, os.path.dirname(path) or ".", path, ctx.k,
                                  where=getattr(D, "files_merge", "ranks"))
        return mine
    n = gather_runs_to_rank0(kca, ctx, D)
    if D.rank == 0:
        ctx.write_output(path)
    return n * ctx.rs


def pick_workdir(explicit, need_bytes):
    """Directory for the e2e leg's input and output files: --workdir, else the
    first of $TMPDIR, /tmp, /dev/shm, /var/tmp and the repository that has
    `need_bytes` free (os.statvfs). Returns (dir, free bytes, tried)."""
    cands = [explicit] if explicit else [os.environ.get("TMPDIR"), "/tmp", "/dev/shm", "/var/tmp", ROOT]
    tried = {}
    for d in cands:
        if not d or d in tried or not os.path.isdir(d) or not os.access(d, os.W_OK):
            continue
        st = os.statvfs(d)
        tried[d] = st.f_bavail * st.f_frsize
        if tried[d] >= need_bytes:
            return d, tried[d], tried
    return None, 0, tried


def write_input_file(ctx, ptr, nbytes, path, piece=256 << 20):
    """The device FASTQ to a file through one bounded host buffer (the host
    never holds the whole input)."""
    import numpy as np

    buf = np.empty(min(piece, max(1, nbytes)), dtype=np.uint8)
    with open(path, "wb") as f:
        for off in range(0, nbytes, piece):
            n = min(piece, nbytes - off)
            ctx.copy_to_host_addr(buf.ctypes.data, ptr + off, n)
            f.write(memoryview(buf)[:n])
    del buf


def main(args, D, state):
    import numpy as np

    kca = load_pkg()
    k, L = args.k, args.L
    W = (k + 31) // 32
    varlen = 0 < args.min_read_length < L
    ctx = kca.Context(kmer_length=k, line_length=L, device=D.device, gpu_memory_limit=args.mem,
                      engine=args.engine, variable_length=varlen)
    state["ctx"] = ctx
    first = shard_first(D.rank, args.reads)
    lmin = args.min_read_length if varlen else 0
    ptr, nbytes = ctx.synth_device(args.reads, L, args.seed, args.genome, 0.0, first, lmin)
    state["ptr"] = ptr
    exchange = args.exchange if D.world > 1 else "none"
    D.files_merge = args.files_merge
    run_dir = None
    files_tm = {}
    if exchange == "files":
        # the ranks' run files and rank 0's merged file (SortedKMerFile each)
        local_ranks = int(os.environ.get("LOCAL_WORLD_SIZE", str(D.world)))
        est = int(nbytes * 0.3) + (64 << 20)
        run_dir, free, tried = pick_workdir(args.workdir, local_ranks * est + (est if D.local == 0 else 0) * 2)
        if run_dir is None:
            raise RuntimeError(f"--exchange files: no directory with room for the run files ({tried})")
        state.setdefault("files", []).extend(
            [os.path.join(run_dir, f"kc_cfg3.run{D.rank}")] + ([os.path.join(run_dir, "kc_cfg3.out")]
                                                              if D.rank == 0 else []))

    def windows_of_step(st):
        return st["windows"] if varlen else args.reads * (L - k + 1)

    # ---- device-resident step: the FASTQ in HBM -> sorted records in HBM -------
    # (the contract's `value`: inputs resident in HBM when the timed region starts)
    xch_ms = [0.0]

    def dev_step():
        ctx.reset()
        ctx.count_fastq_device(ptr, nbytes)
        n = ctx.finish()
        if exchange == "alltoall":
            t = time.perf_counter()
            n = kca.keyspace_exchange(ctx, D.dist, D.xdev())
            xch_ms[0] += (time.perf_counter() - t) * 1e3
        elif exchange == "none" and D.world > 1:
            t = time.perf_counter()
            n = gather_runs_to_rank0(kca, ctx, D)
            xch_ms[0] += (time.perf_counter() - t) * 1e3
        elif exchange == "files":
            t = time.perf_counter()
            n, _ = host_merge_runs(kca, ctx, D, run_dir, os.path.join(run_dir, "kc_cfg3.out"), k,
                                   where=args.files_merge, timing=files_tm)
            xch_ms[0] += (time.perf_counter() - t) * 1e3
        return n

    for _ in range(args.warmup):
        dev_step()
    D.barrier_sync()
    xch_ms[0] = 0.0
    files_tm.clear()
    acc = {"insert_ms": 0.0, "finish_ms": 0.0, "decode_ms": 0.0, "dedup_ms": 0.0, "presplit_ms": 0.0, "launches": 0,
           "part_ms": [0.0] * 5, "finish_group_ms": 0.0, "records": 0}
    t0 = time.perf_counter()
    n_rec = 0
    for _ in range(args.steps):
        n_rec = dev_step()
        st = ctx.stats()
        acc["insert_ms"] += st["insert_ms"]
        acc["launches"] += st["insert_launches"]
        acc["finish_ms"] += st["finish_ms"]
        acc["decode_ms"] += st["decode_ms"]
        acc["dedup_ms"] += st.get("dedup_ms", 0.0)
        acc["presplit_ms"] += st.get("presplit_ms", 0.0)
        acc["finish_group_ms"] += st.get("finish_group_ms", 0.0)
        acc["records"] += st["output_records"]
        acc["part_ms"] = [a + b for a, b in zip(acc["part_ms"], st["part_ms"])]
    D.barrier_sync()
    dev_el = D.max(time.perf_counter() - t0)
    st = ctx.stats()
    windows_per_gpu = windows_of_step(st)
    if D.world > 1 and varlen:
        windows_per_gpu = D.sum(windows_per_gpu) / D.world
    dev_value = windows_per_gpu * D.world * args.steps / dev_el
    roofline = device_roofline(args, st, acc, windows_per_gpu, nbytes, dev_el, varlen, k, L, W)
    device_resident = {
        "value": dev_value, "ms_per_step": dev_el / args.steps * 1e3,
        "breakdown_ms_per_step": {"fastq_index": acc["decode_ms"] / args.steps,
                                  "finish": acc["finish_ms"] / args.steps,
                                  "finish_grouping (in finish)": round(acc["finish_group_ms"] / args.steps, 3),
                                  "exchange_rank0": xch_ms[0] / args.steps,
                                  "exchange": exchange,
                                  **({"files_merge": args.files_merge, "merge_threads_per_rank": merge_threads(D),
                                      "files_ms_rank0": {key: round(v / args.steps * 1e3, 2)
                                                         for key, v in files_tm.items()}}
                                     if exchange == "files" else {}),
                                  "partition_passes": [round(x / args.steps, 3) for x in acc["part_ms"]],
                                  "p5a_dedup": round(acc["dedup_ms"] / args.steps, 3),
                                  "p3b_presplit (in partition_passes[2])": round(acc["presplit_ms"] / args.steps, 3)},
    }
    stats_dev = st

    # ---- end-to-end: FASTQ file in -> SortedKMerFile closed (PCIe-inclusive) ----
    e2e = None
    run_e2e = args.e2e if args.e2e is not None else (D.world == 1)
    if run_e2e:
        try:
            e2e = e2e_leg(kca, ctx, D, args, state, ptr, nbytes, exchange, windows_of_step)
        except Exception as ex:  # reported in the line; the device figure stands
            e2e = {"error": f"{type(ex).__name__}: {ex}"}
    elif D.world > 1:
        e2e = {"skipped": "N > 1: the file-to-file leg runs with --e2e (each rank writes its own 15.7 GB input file)"}

    # ---- host-memory input and the reference's chunks (N = 1) --------------------
    variants = {}
    if D.world == 1 and not args.no_variants and not varlen:
        try:
            variants = host_variants(kca, ctx, args, state, nbytes, k, L)
        except Exception as ex:
            variants = {"error": f"{type(ex).__name__}: {ex}"}
    for p in list(state.get("files", [])):
        _unlink(p)
    state["files"] = []

    cpu = None
    # rank 0 times the CPU port after the timed region, at every N (the other
    # ranks wait at the closing barrier)
    if D.rank == 0 and not args.no_cpu:
        if varlen:
            cpu = cpu_baseline_varlen(kca, max(1, args.cpu_reads // 10), L, args.min_read_length, k, args.genome,
                                      args.seed)
        else:
            cpu = cpu_baselines(kca, args.cpu_reads, L, k, args.genome, args.seed)

    src = (f"sampled from a {args.genome} bp random genome" if args.genome else "of iid uniform bases")
    lens = f"{args.min_read_length}..{L} bp (variable-length, KC_FLAG_VARLEN)" if varlen else f"{L} bp"
    base = f"k={k}, {args.reads} x {lens} reads per GPU {src} (seed {args.seed})"
    cfg_tag = f"cfg{args.config}{'v' if varlen else ''}"
    path_desc = "FASTQ in HBM -> sorted SortedKMerFile records in HBM (device-resident)"
    if D.world == 1:
        workload, parallelism = f"{cfg_tag}: {base}; {path_desc}", "single GPU"
    elif exchange == "alltoall":
        workload = (f"cfg4 pattern at {D.world} GPUs: {base}; {path_desc}; key-space all-to-all of the sorted "
                    f"(key, count) records (RCCL) + per-GPU merge: rank r owns the r-th key range "
                    f"(rank-order concatenation = the SortedKMerFile)")
        parallelism = f"read-shard count + key-space all-to-all x{D.world}"
    elif exchange == "files":
        by = ("shared by the ranks: rank r merges the r-th key range of every run file (kc_merge_part_create) "
              "and writes it at its offset of the one output file" if args.files_merge == "ranks"
              else "on rank 0 alone (kc_merge_files)")
        workload = (f"cfg3 at {D.world} GPUs as BASELINE.json states it: {base}; read-shard, no RCCL on the data "
                    f"path: each rank's sorted run written as a SortedKMerFile, then the host k-way merge "
                    f"(KMerFileMerger semantics) into the node's SortedKMerFile, {by}; step = count + run files + "
                    f"merge")
        parallelism = (f"read-shard x{D.world} + host k-way merge "
                       f"{'by key range on every rank' if args.files_merge == 'ranks' else 'on rank 0'}")
    else:
        workload = (f"cfg3 pattern at {D.world} GPUs: {base}; {path_desc}; runs gathered to rank 0's GPU "
                    f"(RCCL) and merged there by merge path")
        parallelism = f"read-shard x{D.world} + device merge on rank 0"

    if args.value == "e2e":
        if not e2e or "value" not in e2e:
            raise RuntimeError(f"--value e2e but the end-to-end leg did not run: {e2e}")
        value, ms = e2e["value"], e2e["ms_per_step"]
    else:
        value, ms = dev_value, dev_el / args.steps * 1e3
    if D.rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "k-mers/s", "n_gpus": D.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": workload, "k": k, "read_length": L, "reads_per_gpu": args.reads,
                       "parallelism": parallelism, "gpu_memory_limit": args.mem, "value": args.value},
            "roofline": roofline,
            "path_frac": roofline["path_frac"],
            "cpu_baseline": cpu,
            "device_resident": device_resident,
            "end_to_end": e2e,
            "host_variants": variants or None,
            "engine": args.engine,
            "engines_used": {1: "skm", 2: "key-prefix partition", 3: "skm + key-prefix",
                             4: "table"}.get(stats_dev.get("engines_used", 0), str(stats_dev.get("engines_used"))),
            "distinct_kmers_per_gpu": n_rec, "spilled_kmers": stats_dev["spilled_kmers"],
            "spill_runs": stats_dev["spill_runs"], "key_passes": stats_dev.get("key_passes", 0),
        }
        print(json.dumps(line), flush=True)
    ctx.free_device(ptr)
    state.pop("ptr", None)
    ctx.close()
    if D.dist is not None:
        D.dist.barrier()
        D.dist.destroy_process_group()


def _unlink(p):
    try:
        os.unlink(p)
    except OSError:
        pass


def e2e_leg(kca, ctx, D, args, state, ptr, nbytes, exchange, windows_of_step):
    """The file-to-file step: kc_reset; kc_count_file (pinned read-ahead blocks,
    PCIe upload, GPU decode + count); kc_finish; kc_write_output (device ->
    pinned -> output file, closed). The input file is written untimed (page
    cache). Every step writes a new output file, which is deleted right after
    the step, outside the step's timed interval; the steps are timed one by one
    (barrier + synchronize on both sides) and summed, so at most one output
    file exists at a time whatever --steps is."""
    out_est = int(nbytes * 0.3) + (64 << 20)  # records <= ~22% of the FASTQ bytes at cfg2/cfg5
    # every rank of this node writes its own input file and output part into
    # the same directory: room for all of them (at N = 8, cfg2: ~160 GB)
    local_ranks = int(os.environ.get("LOCAL_WORLD_SIZE", str(D.world)))
    need = local_ranks * (nbytes + 2 * out_est) + (1 << 30)
    if exchange == "files":
        need += local_ranks * out_est  # each rank's run file (kc_cfg3.run<r>) next to the output
    workdir, free, tried = pick_workdir(args.workdir, need)
    if workdir is None:
        return {"skipped": f"no directory with {need / 1e9:.1f} GB free for the input file and one output file",
                "free_bytes": tried}
    tag = os.getpid() if D.world == 1 else f"r{D.rank}"
    in_path = os.path.join(workdir, f"kc_bench_in.{tag}.fq")
    out_path = os.path.join(workdir, f"kc_bench_out.{os.getpid() if D.world == 1 else 'node'}.bin")
    state.setdefault("files", []).append(in_path)
    run_file = os.path.join(workdir, f"kc_cfg3.run{D.rank}")  # written by host_merge_runs (exchange files)
    if exchange == "files":
        state["files"].append(run_file)
    write_input_file(ctx, ptr, nbytes, in_path)
    state["in_path"] = in_path
    varlen = 0 < args.min_read_length < args.L
    phase = {"count_file": 0.0, "finish": 0.0, "output": 0.0}
    out_bytes = [0]

    def step(path):
        t0 = time.perf_counter()
        ctx.reset()
        ctx.count_file(in_path, args.L if varlen else 0)
        t1 = time.perf_counter()
        ctx.finish()
        t2 = time.perf_counter()
        out_bytes[0] = write_node_output(kca, ctx, D, path, exchange)
        t3 = time.perf_counter()
        return t1 - t0, t2 - t1, t3 - t2

    def cleanup(path):
        for q in (path, f"{path}.part{D.rank}"):
            if D.rank == 0 or q != path:
                _unlink(q)

    total = 0.0
    for i in range(args.warmup + args.steps):
        path = f"{out_path}.{i}"
        state["files"].extend([path, f"{path}.part{D.rank}"])
        D.barrier_sync()
        t0 = time.perf_counter()
        ph = step(path)
        D.barrier_sync()
        dt = D.max(time.perf_counter() - t0)
        cleanup(path)  # outside the step's interval
        if i >= args.warmup:
            total += dt
            for key, v in zip(phase, ph):
                phase[key] += v
    st = ctx.stats()
    win = D.sum(windows_of_step(st))
    in_b = D.sum(nbytes)
    step_s = total / args.steps
    ph = {key: v / args.steps * 1e3 for key, v in phase.items()}
    _unlink(in_path)
    state["files"].remove(in_path)
    if exchange == "files":
        _unlink(run_file)
        state["files"].remove(run_file)
    state.pop("in_path", None)
    return {"value": win / step_s, "ms_per_step": step_s * 1e3,
            "path": ("FASTQ file (page cache) -> pinned blocks -> PCIe -> GPU decode + count -> sorted records -> "
                     "PCIe -> SortedKMerFile closed"),
            "phases_ms_rank0": {key: round(v, 2) for key, v in ph.items()},
            "input_bytes": int(in_b), "output_bytes": int(D.sum(out_bytes[0])),
            # PCIe / file rates of rank 0's phases (count_file includes the GPU decode and counting of
            # whatever fits no flush before it; the output phase is D2H + file write)
            "input_GBps_rank0": round(nbytes / (ph["count_file"] / 1e3) / 1e9, 2),
            "output_GBps_rank0": round(out_bytes[0] / (ph["output"] / 1e3) / 1e9, 2) if ph["output"] else None,
            "workdir": workdir, "workdir_free_GB": round(free / 1e9, 1),
            "timing": "steps timed one by one (barrier + sync both sides, max over ranks) and summed; each step's "
                      "output file deleted between steps"}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5],
                    help="SURVEY §8d preset: 2 = k=31, 50M x 150 bp from a 250 Mbp genome (the metric's "
                         "config); 3 = cfg3's shard, 50M reads per GPU (400M over 8 GPUs, seed 3), read-shard "
                         "(--exchange none at N > 1); 4 = cfg4's shard, 125M reads per GPU (1B over 8 GPUs, "
                         "seed 4), key-space all-to-all at N > 1; "
                         "5 = k=55, 20M x 150 bp iid reads (~1.9e9 distinct, high cardinality) with a "
                         "48 GiB working set: the keys outgrow one batch and are counted in key-range passes "
                         "(the spill -> sort -> merge path)")
    ap.add_argument("--value", default="device", choices=["device", "e2e"],
                    help="value = the device-resident rate (the FASTQ resident in HBM when the timed region "
                         "starts: the contract's definition, default) or the file-to-file rate (e2e)")
    ap.add_argument("--mode", default=None, choices=["e2e", "device"], help="alias of --value (round-3 scripts)")
    ap.add_argument("--e2e", dest="e2e", action="store_true", default=None,
                    help="run the file-to-file leg (default: at N = 1 only)")
    ap.add_argument("--no-e2e", dest="e2e", action="store_false")
    ap.add_argument("--reads", type=int, default=None, help="reads per GPU")
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--L", type=int, default=150)
    ap.add_argument("--genome", type=int, default=None, help="0 = iid uniform reads")
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--mem", type=int, default=None, help="gpuMemoryLimit per GPU (bytes)")
    ap.add_argument("--engine", default="auto", choices=["auto", "skm", "partition", "table"])
    ap.add_argument("--cpu-reads", type=int, default=1_000_000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-variants", action="store_true", help="skip the host_memory / reference_chunks lines")
    ap.add_argument("--workdir", default=None, help="input/output files (default: $TMPDIR, /tmp, /dev/shm, ... "
                                                    "whichever has the space)")
    ap.add_argument("--files-merge", default="ranks", choices=["ranks", "rank0"],
                    help="--exchange files: the run files' k-way merge shared by the ranks (each merges one key "
                         "range of every file and writes it at its offset of the one output file; default) or "
                         "done by rank 0 alone")
    ap.add_argument("--min-read-length", type=int, default=0,
                    help="variable-length reads of M..L bases (KC_FLAG_VARLEN); 0 = every read has L bases")
    ap.add_argument("--exchange", default=None, choices=["alltoall", "none", "files"],
                    help="N>1: key-space all-to-all (cfg4, RCCL), read-shard + RCCL gather and device merge on "
                         "rank 0 (none), or read-shard + run files + host k-way merge on rank 0 (files: cfg3 as "
                         "stated, no RCCL)")
    args = ap.parse_args(argv)
    if args.mode:
        args.value = args.mode
        if args.mode == "e2e" and args.e2e is None:
            args.e2e = True
    preset = {2: dict(reads=50_000_000, k=31, genome=250_000_000, seed=2, mem=160 << 30),
              3: dict(reads=50_000_000, k=31, genome=250_000_000, seed=3, mem=160 << 30, exchange="files"),
              4: dict(reads=125_000_000, k=31, genome=250_000_000, seed=4, mem=160 << 30, exchange="alltoall"),
              5: dict(reads=20_000_000, k=55, genome=0, seed=5, mem=48 << 30)}[args.config]
    preset.setdefault("exchange", "alltoall")
    for key, v in preset.items():
        if getattr(args, key) is None:
            setattr(args, key, v)
    return args


def run():
    """Entry point: any failure still prints one JSON line (rank 0) with an
    `error` field, and removes the files the run wrote."""
    import traceback

    args = None
    state = {"files": []}
    D = None
    try:
        args = parse_args()
        D = Dist()
        main(args, D, state)
        return 0
    except BaseException as ex:  # noqa: B902 - report everything, then fail
        tb = traceback.format_exc()
        rank = int(os.environ.get("RANK", "0"))
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": None, "unit": "k-mers/s",
                              "n_gpus": int(os.environ.get("WORLD_SIZE", "1")),
                              "steps": getattr(args, "steps", None), "warmup": getattr(args, "warmup", None),
                              "error": f"{type(ex).__name__}: {ex}", "traceback_tail": tb[-2000:]}), flush=True)
        try:
            sys.stderr.write(tb)
            sys.stderr.flush()
        except OSError:
            pass
        return 1
    finally:
        for p in state.get("files", []):
            _unlink(p)
        try:
            if state.get("ptr") and state.get("ctx"):
                state["ctx"].free_device(state["ptr"])
        except Exception:
            pass


def device_roofline(args, st, acc, windows_step, nbytes, dev_el, varlen, k, L, W):
    """Per-kernel rooflines of the device-resident step. Each main kernel is
    priced by its own algorithmic HBM bytes; `roofline` is the
    kernel with the largest per-step time; achieved = algorithmic bytes per
    launch / its HIP-event launch time on the ctx stream. `path_frac` is
    SURVEY §8d's whole-path figure: k-mers/s per GPU x (FASTQ bytes per k-mer
    + 8W + 8) over the device-resident step."""
    G = (L + 15) // 16
    steps = args.steps
    part_ms = acc["part_ms"]
    recs_step = st["output_records"]
    kernels = {}
    used = st.get("engines_used", 0)
    if used & 1:
        rec_step = st["keys"] or 1  # records handed out by F per step
        rb = 8 * (W + 1)
        nw = L - k + 1
        ng = max((L + 15) // 16 + 1, (nw - 1) // 16 + 5) | 1
        hooks = os.environ.get("KC_TEST_HOOKS") == "1"  # the library reads KC_NO_F3/F2 only then
        f3 = (W == 1 and 19 <= k <= 32 and (320 + 64) * 8 + 256 + 256 * ng <= 40 * 1024
              and not (hooks and os.environ.get("KC_NO_F3")))
        f2 = W == 1 and 18 <= k <= 32 and (nw + 7) // 8 <= 64 and not (hooks and os.environ.get("KC_NO_F2"))
        fname = f"skm_front3_k<{k}>" if f3 else (f"skm_front2_k<1,{k}>" if f2 else f"skm_front_k<{W}>")
        dd_step = st.get("dedup_records", 0)
        specs = [
            ("F", fname, part_ms[1], acc["launches"], windows_step, "k-mers",
             (G * 6) / max(1, L - k + 1) + rb * rec_step / windows_step),
            ("S", f"rp_scatter_k<{W + 1},false>", part_ms[2], 2 * steps * st["batches"], 2 * rec_step, "records",
             2 * rb + 1),
        ]
        if acc["dedup_ms"] > 0:
            specs += [
                ("P5a", "count_rec_k", acc["dedup_ms"], steps * st["batches"], rec_step, "records",
                 rb + (rb + 4) * dd_step / rec_step),
                ("P5", f"count_skm_k<{W}>", part_ms[4], steps * st["batches"], max(1, dd_step), "distinct records",
                 (rb + 4) + (8 * W + 4) * recs_step / max(1, dd_step)),
            ]
        else:
            specs.append(("P5", f"count_skm_k<{W}>", part_ms[4], steps * st["batches"], rec_step, "records",
                          rb + (8 * W + 4) * recs_step / rec_step))
        if acc["finish_ms"] > 0 and acc["records"] > 0:
            # kc_finish: two grouping passes over the (key, count) records (read
            # and write 8W + 4 B each, plus the digit byte written by one pass and
            # read by the next's histogram) and the LDS segment sort writing the
            # SortedKMerFile records (8W + 4 in, 8W + 4 out)
            specs.append(("finish", f"rp_scatter_k<{W},true> x2 + seg_sort_k<{W}> (+ histograms, bounds)",
                          acc["finish_ms"], steps, acc["records"] / steps, "distinct records",
                          6 * (8 * W + 4) + 3))
    elif used & 2:
        keys_step = st["keys"] or windows_step
        p5_per_step = max(1, st["p5_launches"])
        # P3 runs once per read batch, or once per key-range pass (a batch
        # counted by key ranges: each pass partitions only its own keys, while
        # P2 walks every window of the batch per pass)
        nb = max(1, st.get("key_passes", 0) or st["batches"])
        pre_b = st.get("presplit_batches", 0)
        pre_ms = acc["presplit_ms"]
        specs = [
            ("P2", f"count_front<{W},2,true,1024>", part_ms[1], acc["launches"], windows_step,
             "k-mers", (G * 6) / max(1, L - k + 1) + 8 * W * keys_step / max(1, windows_step)),
            ("P3", f"rp_scatter_k<{W},false>", part_ms[2] - pre_ms, steps * nb, keys_step, "keys",
             16 * W),
        ]
        if pre_b:
            # P3b: word 0 read for the regional histogram + one scatter pass
            specs.append(("P3b", f"rp_scatter_k<{W},false> + rp_upsweep_k", pre_ms, steps * pre_b,
                          keys_step * pre_b / nb, "keys", 8 + 16 * W))
        if st.get("sorted_run_batches", 0):
            # P5s: keys read once, records written (packed, or SoA + segment copy)
            specs.append(("P5", f"sort_runs_k<{W}>", part_ms[4], steps * p5_per_step, keys_step, "keys",
                          8 * W + (8 * W + 4) * recs_step / max(1, keys_step)))
        else:
            specs.append(("P5", f"count_buckets<{W}>", part_ms[4], steps * p5_per_step, keys_step, "keys",
                          8 * W + (8 * W + 4) * recs_step / max(1, keys_step)))
    else:
        specs = [("insert", f"count_front<{W},0,false,256>", acc["insert_ms"], acc["launches"], windows_step,
                  "k-mers", nbytes / windows_step + 8 * W + 8)]
    for tag, name, ms_total, nl, units_step, unit_name, bpu in specs:
        nl = max(1, nl)
        avg = ms_total / nl
        units = units_step * steps / nl
        ach = bpu * units / (avg / 1e3) / 1e9 if avg > 0 else 0.0
        kernels[tag] = {"kernel": name, "avg_launch_ms": round(avg, 3), "ms_per_step": round(ms_total / steps, 3),
                        "units_per_launch": int(units), "unit": unit_name,
                        "algorithmic_bytes_per_unit": round(bpu, 3), "achieved": round(ach, 2),
                        "frac": round(ach / HBM_PEAK_GBS, 4)}
    dom = max(kernels, key=lambda t: kernels[t]["ms_per_step"])
    d = kernels[dom]
    t_bytes = None
    # the committed PMC summaries (cfg2: pmc_count_kmers.json, cfg5:
    # pmc_cfg5.json), used when they are of this workload (reads, k)
    for fname in ("pmc_count_kmers.json", "pmc_cfg5.json"):
        try:
            traffic = json.load(open(os.path.join(ROOT, "profiles", fname)))
        except (OSError, ValueError):
            continue
        if not varlen and traffic.get("reads_per_gpu") == args.reads and traffic.get("k") == k:
            # (a composite entry is keyed by its first kernel, the one the PMC passes measured)
            t_bytes = traffic.get("kernels", {}).get(d["kernel"].split(" ")[0], {}).get("bytes_per_launch")
            break
    b_path = nbytes / windows_step + 8 * W + 8
    path_achieved = b_path * windows_step / (dev_el / steps) / 1e9
    return {"bound": "hbm", "achieved": d["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": d["frac"], "traffic": t_bytes, "kernel": f"{dom}: {d['kernel']}",
            "avg_launch_ms": d["avg_launch_ms"], "units_per_launch": d["units_per_launch"],
            "unit_of_work": d["unit"], "algorithmic_bytes_per_unit": d["algorithmic_bytes_per_unit"],
            "path_achieved": round(path_achieved, 2), "path_frac": round(path_achieved / HBM_PEAK_GBS, 4),
            "path_bytes_per_kmer": round(b_path, 3), "kernels": kernels,
            "note": "dominant kernel = largest device time per step; path_* = SURVEY §8d bytes per k-mer over the "
                    "device-resident step"}


def host_variants(kca, ctx, args, state, nbytes, k, L):
    """host_memory: the FASTQ from pageable host memory in one kc_count_fastq
    call -> output file (deleted right after). reference_chunks: the same
    reads as the reference's chunks (sequences only, 7.8 MB each at
    gpuMemoryLimit=1e8) through kc_count_chunk, against one kc_count_chunk of
    all of them (records left in HBM in both). N = 1 only; the host copies are
    freed before the next one is made."""
    import numpy as np

    res = {}
    win = args.reads * (L - k + 1)

    def one(step, reps=1, after=lambda: None):
        step()  # warm
        after()
        best = None
        for _ in range(reps):
            t = time.perf_counter()
            step()
            dt = time.perf_counter() - t
            after()  # outside the interval
            best = dt if best is None else min(best, dt)
        return best

    workdir, _, tried = pick_workdir(args.workdir, int(nbytes * 0.3) + (2 << 30))
    if workdir is None:
        res["host_memory"] = {"skipped": "no directory with room for one output file", "free_bytes": tried}
    else:
        host = np.empty(nbytes, dtype=np.uint8)
        ctx.copy_to_host_addr(host.ctypes.data, state["ptr"], nbytes)
        out = os.path.join(workdir, f"kc_bench_out.{os.getpid()}.host")
        state.setdefault("files", []).append(out)

        def host_step():
            ctx.reset()
            ctx.count_fastq_host(host.ctypes.data, nbytes)
            ctx.write_output(out)

        dt = one(host_step, after=lambda: _unlink(out))
        del host
        res["host_memory"] = {"value": win / dt, "ms_per_step": dt * 1e3,
                              "path": "FASTQ in pageable host memory -> pinned ring -> PCIe -> GPU decode + count -> "
                                      "SortedKMerFile closed"}
    # the reference's chunk layout: concatenated sequences
    sptr, sbytes = ctx.synth_device(args.reads, L, args.seed, args.genome, 0.0, 0, 0, layout=1)
    seqs = np.empty(sbytes, dtype=np.uint8)
    ctx.copy_to_host_addr(seqs.ctypes.data, sptr, sbytes)
    ctx.free_device(sptr)
    # KMerCounter::GetChunkSize at the reference's default gpuMemoryLimit (main.cpp:28)
    kb = (k + 3) // 4
    per = ((kb + 7) // 8 + 1) * 8 * (L - k + 1)
    cs = L * ((100000000 - L) // (per - 1))
    base = seqs.ctypes.data

    def chunks_step():
        ctx.reset()
        for off in range(0, sbytes, cs):
            ctx.count_chunk_host(base + off, min(cs, sbytes - off), L)
        ctx.finish()

    def block_step():
        ctx.reset()
        ctx.count_chunk_host(base, sbytes, L)
        ctx.finish()

    # best of 3 after a warm run, both ways alike (a single host-side rep
    # varies by tens of ms from run to run on the shared host)
    tc = one(chunks_step, reps=3)
    tb = one(block_step, reps=3)
    res["reference_chunks"] = {"chunk_bytes": cs, "chunks": (sbytes + cs - 1) // cs,
                               "value_chunks": win / tc, "ms_chunks": tc * 1e3,
                               "value_one_block": win / tb, "ms_one_block": tb * 1e3,
                               "chunks_over_block_time": round(tc / tb, 3)}
    del seqs
    return res


if __name__ == "__main__":
    sys.exit(run())
