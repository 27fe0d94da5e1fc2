"""kmer-counter_amd — Python mirror of the reference's count-path interface
over the C ABI of libkc_hip.so (include/kc.h).

The reference's host interface is C++ (Options, KMerCounter, KMerPrinter:
Options.h:21-57, KMerCounter.h:70-75, KMerPrinter.h); this module mirrors it
with the same names and argument meanings so tests read like the reference's
usage, and adds `Context`, a thin wrapper of one device context (kc_ctx).

Nothing here computes k-mers: every count goes through the HIP kernels in
libkc_hip.so. If the library is missing the import of `lib()` raises — there
is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import re
import subprocess
from typing import List, Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
# KC_LIB: tuning experiments only (tools/build_variant.sh builds variants of
# the same sources under kmer-counter_amd/variants/)
LIB_PATH = os.environ.get("KC_LIB") or os.path.join(_HERE, "libkc_hip.so")
CLI_PATH = os.path.join(_HERE, "kmer-counter")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "kc.h")

KC_OK = 0
KC_ERR_ARG = 1
KC_ERR_HIP = 2
KC_ERR_NOMEM = 3
KC_ERR_FORMAT = 4
KC_ERR_IO = 5
KC_ERR_STATE = 6
KC_ERR_NODEVICE = 7
KC_ERR_INTERNAL = 8

KC_INPUT_AUTO = 0
KC_INPUT_FASTQ = 1
KC_INPUT_EXACT = 2
_INPUT_MODES = {"auto": KC_INPUT_AUTO, "fastq": KC_INPUT_FASTQ, "exact": KC_INPUT_EXACT}


class KcError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"kc status {status}: {msg}")
        self.status = status


class _Config(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int32),
        ("reserved0", ctypes.c_int32),
        ("kmer_length", ctypes.c_int64),
        ("line_length", ctypes.c_int64),
        ("gpu_memory_limit", ctypes.c_uint64),
        ("table_bytes", ctypes.c_uint64),
        ("temp_dir", ctypes.c_char_p),
        ("flags", ctypes.c_uint32),
        ("lds_slots", ctypes.c_uint32),
    ]


class Stats(ctypes.Structure):
    _fields_ = [
        ("reads", ctypes.c_uint64),
        ("windows", ctypes.c_uint64),
        ("valid_kmers", ctypes.c_uint64),
        ("table_capacity", ctypes.c_uint64),
        ("table_used", ctypes.c_uint64),
        ("spilled_kmers", ctypes.c_uint64),
        ("spill_runs", ctypes.c_uint64),
        ("output_records", ctypes.c_uint64),
        ("insert_launches", ctypes.c_uint64),
        ("insert_ms", ctypes.c_double),
        ("decode_ms", ctypes.c_double),
        ("finish_ms", ctypes.c_double),
        ("last_count_ms", ctypes.c_double),
        ("part_ms", ctypes.c_double * 5),
        ("batches", ctypes.c_uint64),
        ("keys", ctypes.c_uint64),
        ("p5_launches", ctypes.c_uint64),
        ("engines_used", ctypes.c_uint32),
        ("reserved1", ctypes.c_uint32),
        ("dedup_ms", ctypes.c_double),
        ("dedup_records", ctypes.c_uint64),
        ("presplit_ms", ctypes.c_double),
        ("presplit_batches", ctypes.c_uint64),
        ("sorted_run_batches", ctypes.c_uint64),
        ("key_passes", ctypes.c_uint64),
        ("finish_group_ms", ctypes.c_double),
    ]

    def as_dict(self):
        d = {f: getattr(self, f) for f, _ in self._fields_}
        d["part_ms"] = list(self.part_ms)
        return d


class _Synth(ctypes.Structure):
    _fields_ = [
        ("n_reads", ctypes.c_uint64),
        ("read_length", ctypes.c_int64),
        ("seed", ctypes.c_uint64),
        ("genome_length", ctypes.c_uint64),
        ("n_rate", ctypes.c_double),
        ("first_read", ctypes.c_uint64),
        ("min_read_length", ctypes.c_int64),
        ("layout", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
    ]


_lib = None


def header_functions() -> List[str]:
    """Names of every function declared in include/kc.h."""
    text = open(HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(kc_[a-z0-9_]+)\s*\(", text)))


def lib() -> ctypes.CDLL:
    """Loads libkc_hip.so (built in-tree by __graft_entry__.build / make)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run `make -C kmer-counter_amd` (no CPU fallback exists)")
    L = ctypes.CDLL(LIB_PATH)
    vp, u64, i64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_uint32
    P = ctypes.POINTER
    sig = {
        "kc_create": ([P(vp), P(_Config)], ctypes.c_int),
        "kc_destroy": ([vp], None),
        "kc_strerror": ([ctypes.c_int], ctypes.c_char_p),
        "kc_last_error": ([vp], ctypes.c_char_p),
        "kc_abi_version": ([], ctypes.c_int32),
        "kc_device_count": ([], ctypes.c_int32),
        "kc_reset": ([vp], ctypes.c_int),
        "kc_count_chunk": ([vp, ctypes.c_char_p, i64, i64], ctypes.c_int),
        "kc_count_chunk_device": ([vp, vp, i64, i64], ctypes.c_int),
        "kc_count_fastq": ([vp, ctypes.c_char_p, u64, i64, P(u64)], ctypes.c_int),
        "kc_count_fastq_device": ([vp, vp, u64, i64, P(u64)], ctypes.c_int),
        "kc_check_fastq": ([vp, ctypes.c_char_p, u64, i64, P(u64)], ctypes.c_int),
        "kc_finish": ([vp, P(u64)], ctypes.c_int),
        "kc_copy_records": ([vp, vp, u64], ctypes.c_int),
        "kc_device_records": ([vp, P(vp), P(u64)], ctypes.c_int),
        "kc_write_output": ([vp, ctypes.c_char_p, u32, u32], ctypes.c_int),
        "kc_write_runs": ([vp, ctypes.c_char_p, P(u32)], ctypes.c_int),
        "kc_get_stats": ([vp, P(Stats)], ctypes.c_int),
        "kc_merge_files": ([P(ctypes.c_char_p), u32, ctypes.c_char_p, i64, u32, u32], ctypes.c_int),
        "kc_synth_fastq_bytes": ([P(_Synth)], u64),
        "kc_synth_fastq_host": ([P(_Synth), vp, u64], ctypes.c_int),
        "kc_synth_fastq_device": ([vp, P(_Synth), P(vp), P(u64)], ctypes.c_int),
        "kc_synth_free": ([vp, vp], ctypes.c_int),
        "kc_copy_to_host": ([vp, vp, vp, u64], ctypes.c_int),
        "kc_owner_counts": ([vp, u32, P(u64)], ctypes.c_int),
        "kc_merge_records_device": ([vp, vp, u64], ctypes.c_int),
        "kc_copy_device": ([vp, vp, vp, u64], ctypes.c_int),
        "kc_exchange_contexts": ([P(vp), u32], ctypes.c_int),
        "kc_merge_runs_device": ([vp, vp, P(u64), u32], ctypes.c_int),
        "kc_checkpoint": ([vp], ctypes.c_int),
        "kc_rollback": ([vp], ctypes.c_int),
        "kc_commit": ([vp], ctypes.c_int),
        "kc_count_file": ([P(vp), u32, ctypes.c_char_p, i64, u32, P(u64)], ctypes.c_int),
        "kc_write_output_at": ([vp, ctypes.c_char_p, u64], ctypes.c_int),
        "kc_gather_contexts": ([P(vp), u32], ctypes.c_int),
        "kc_merge_part_create": ([P(ctypes.c_char_p), u32, i64, u32, u32, u32, P(vp), P(u64)], ctypes.c_int),
        "kc_merge_part_write": ([vp, ctypes.c_char_p, u64, u64], ctypes.c_int),
        "kc_merge_part_destroy": ([vp], None),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def _spec(n_reads, read_length, seed, genome_length=0, n_rate=0.0, first_read=0, min_read_length=0, layout=0):
    return _Synth(n_reads, read_length, seed, genome_length, n_rate, first_read, min_read_length, layout, 0)


def synth_fastq(n_reads: int, read_length: int, seed: int, genome_length: int = 0, n_rate: float = 0.0,
                first_read: int = 0, min_read_length: int = 0, layout: int = 0) -> bytes:
    """Synthetic FASTQ text (SURVEY §8d generator) produced by the library's host generator
    (layout 1: the sequences only, concatenated — a reference chunk)."""
    L = lib()
    sp = _spec(n_reads, read_length, seed, genome_length, n_rate, first_read, min_read_length, layout)
    n = L.kc_synth_fastq_bytes(ctypes.byref(sp))
    buf = ctypes.create_string_buffer(n + 1)
    st = L.kc_synth_fastq_host(ctypes.byref(sp), buf, n + 1)
    if st:
        raise KcError(st, L.kc_strerror(st).decode())
    return buf.raw[:n]


def merge_files(inputs: List[str], output: str, kmer_length: int, fan_in: int = 2, threads: int = 2) -> None:
    L = lib()
    arr = (ctypes.c_char_p * max(1, len(inputs)))(*[p.encode() for p in inputs])
    st = L.kc_merge_files(arr, len(inputs), output.encode(), kmer_length, fan_in, threads)
    if st:
        raise KcError(st, L.kc_strerror(st).decode())


class MergePart:
    """One part of a host k-way merge shared by `parts` processes over the same
    run files (kc_merge_part_create): cfg3's ranks each merge one key range of
    every rank's run file, then write it at its offset of the one output file
    (the offsets are the prefix sums of the parts' sizes, gathered by the
    caller). Use as a context manager or call close()."""

    def __init__(self, inputs: List[str], kmer_length: int, part: int, parts: int, threads: int = 1):
        self._L = lib()
        arr = (ctypes.c_char_p * max(1, len(inputs)))(*[p.encode() for p in inputs])
        h = ctypes.c_void_p()
        n = ctypes.c_uint64()
        st = self._L.kc_merge_part_create(arr, len(inputs), kmer_length, part, parts, threads, ctypes.byref(h),
                                          ctypes.byref(n))
        if st:
            raise KcError(st, self._L.kc_strerror(st).decode())
        self._h = h
        self.nbytes = int(n.value)

    def write(self, output: str, offset: int, file_bytes: int = 0) -> None:
        st = self._L.kc_merge_part_write(self._h, output.encode(), offset, file_bytes)
        if st:
            raise KcError(st, self._L.kc_strerror(st).decode())

    def close(self) -> None:
        if self._h:
            self._L.kc_merge_part_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """One device context (kc_ctx): the GPU table of one device."""

    def __init__(self, kmer_length: int, line_length: int = 0, device: int = 0,
                 gpu_memory_limit: int = 100000000, table_bytes: int = 0, temp_dir: Optional[str] = None,
                 quiet: bool = True, engine: str = "auto", lds_slots: int = 0, variable_length: bool = False):
        self._L = lib()
        self.k = kmer_length
        self.W = (kmer_length + 31) // 32
        self.rs = 8 * self.W + 4
        self._device = device
        self._tmp = temp_dir.encode() if temp_dir else None
        engine_flags = {"auto": 0, "table": 2, "skm": 4, "partition": 8}
        if engine not in engine_flags:
            raise ValueError("engine must be 'auto', 'skm', 'partition' or 'table'")
        flags = (1 if quiet else 0) | engine_flags[engine] | (16 if variable_length else 0)
        cfg = _Config(device, 0, kmer_length, line_length or kmer_length, int(gpu_memory_limit), int(table_bytes),
                      self._tmp, flags, int(lds_slots))
        h = ctypes.c_void_p()
        st = self._L.kc_create(ctypes.byref(h), ctypes.byref(cfg))
        if st:
            raise KcError(st, self._L.kc_strerror(st).decode())
        self._h = h

    def _chk(self, st: int):
        if st:
            raise KcError(st, f"{self._L.kc_strerror(st).decode()}: {self._L.kc_last_error(self._h).decode()}")

    def close(self):
        if getattr(self, "_h", None):
            self._L.kc_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        self._chk(self._L.kc_reset(self._h))

    def count_chunk(self, chunk: bytes, line_length: int):
        self._chk(self._L.kc_count_chunk(self._h, chunk, len(chunk), line_length))

    def count_chunk_device(self, ptr: int, size: int, line_length: int):
        self._chk(self._L.kc_count_chunk_device(self._h, ctypes.c_void_p(ptr), size, line_length))

    def count_fastq(self, data: bytes, line_length: int = 0) -> int:
        n = ctypes.c_uint64()
        self._chk(self._L.kc_count_fastq(self._h, data, len(data), line_length, ctypes.byref(n)))
        return n.value

    def check_fastq(self, data: bytes, line_length: int = 0) -> int:
        n = ctypes.c_uint64()
        self._chk(self._L.kc_check_fastq(self._h, data, len(data), line_length, ctypes.byref(n)))
        return n.value

    def count_chunk_host(self, addr: int, size: int, line_length: int):
        """kc_count_chunk on raw host memory (e.g. a numpy array's address)."""
        self._chk(self._L.kc_count_chunk(self._h, ctypes.cast(addr, ctypes.c_char_p), size, line_length))

    def count_fastq_host(self, addr: int, size: int, line_length: int = 0) -> int:
        """kc_count_fastq on raw host memory (e.g. a numpy array's address)."""
        n = ctypes.c_uint64()
        self._chk(self._L.kc_count_fastq(self._h, ctypes.cast(addr, ctypes.c_char_p), size, line_length,
                                         ctypes.byref(n)))
        return n.value

    def copy_to_host_addr(self, addr: int, ptr: int, n: int):
        """Device -> host copy into raw host memory (e.g. a numpy array's address)."""
        self._chk(self._L.kc_copy_to_host(self._h, ctypes.c_void_p(addr), ctypes.c_void_p(ptr), n))

    def count_fastq_device(self, ptr: int, size: int, line_length: int = 0) -> int:
        n = ctypes.c_uint64()
        self._chk(self._L.kc_count_fastq_device(self._h, ctypes.c_void_p(ptr), size, line_length, ctypes.byref(n)))
        return n.value

    def count_file(self, path: str, line_length: int = 0, mode: str = "auto") -> int:
        """kc_count_file on this context alone; returns the reads counted."""
        return count_file([self], path, line_length, mode)

    def checkpoint(self):
        self._chk(self._L.kc_checkpoint(self._h))

    def rollback(self):
        self._chk(self._L.kc_rollback(self._h))

    def commit(self):
        self._chk(self._L.kc_commit(self._h))

    def synth_device(self, n_reads, read_length, seed, genome_length=0, n_rate=0.0, first_read=0,
                     min_read_length=0, layout=0):
        """Generates synthetic FASTQ directly in device memory; returns (ptr, nbytes)."""
        sp = _spec(n_reads, read_length, seed, genome_length, n_rate, first_read, min_read_length, layout)
        p = ctypes.c_void_p()
        n = ctypes.c_uint64()
        self._chk(self._L.kc_synth_fastq_device(self._h, ctypes.byref(sp), ctypes.byref(p), ctypes.byref(n)))
        return p.value, n.value

    def free_device(self, ptr: int):
        self._chk(self._L.kc_synth_free(self._h, ctypes.c_void_p(ptr)))

    def copy_to_host(self, ptr: int, n: int) -> bytes:
        buf = ctypes.create_string_buffer(max(1, n))
        self._chk(self._L.kc_copy_to_host(self._h, buf, ctypes.c_void_p(ptr), n))
        return buf.raw[:n]

    def finish(self) -> int:
        n = ctypes.c_uint64()
        self._chk(self._L.kc_finish(self._h, ctypes.byref(n)))
        return n.value

    def records(self) -> bytes:
        """Sorted table run (SortedKMerFile bytes); requires no spill runs."""
        n = self.finish()
        buf = ctypes.create_string_buffer(max(1, n * self.rs))
        self._chk(self._L.kc_copy_records(self._h, buf, n * self.rs))
        return buf.raw[: n * self.rs]

    def device_records(self):
        """(device pointer, bytes) of the finished table run's packed records."""
        p = ctypes.c_void_p()
        n = ctypes.c_uint64()
        self._chk(self._L.kc_device_records(self._h, ctypes.byref(p), ctypes.byref(n)))
        return p.value or 0, n.value

    def owner_counts(self, world: int) -> List[int]:
        """Records of the finished table run per key-space owner (kc_owner_counts)."""
        arr = (ctypes.c_uint64 * world)()
        self._chk(self._L.kc_owner_counts(self._h, world, arr))
        return list(arr)

    def export_records(self, dst) -> int:
        """Copy the finished table run's packed records into the torch uint8
        tensor `dst` (device or host); returns the record count."""
        n = self.finish()
        nb = n * self.rs
        if dst.numel() < nb:
            raise ValueError("destination too small")
        if dst.is_cuda:
            ptr, _ = self.device_records()
            self._chk(self._L.kc_copy_device(self._h, ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(ptr), nb))
        else:
            self._chk(self._L.kc_copy_records(self._h, ctypes.c_void_p(dst.data_ptr()), nb))
        return n

    def merge_records(self, src, n_records: int) -> int:
        """Replace the table run by the sorted, summed merge of n_records packed
        records held in the torch uint8 tensor `src` (host tensors are staged
        to this ctx's device first); returns the merged record count."""
        if n_records * self.rs > src.numel():
            raise ValueError("source too small")
        if not src.is_cuda:
            import torch

            src = src.to(torch.device("cuda", self._device))
        self._chk(self._L.kc_merge_records_device(self._h, ctypes.c_void_p(src.data_ptr()), n_records))
        return self.finish()

    def merge_runs(self, src, run_counts) -> int:
        """Like merge_records when `src` holds len(run_counts) sorted runs one
        after another (kc_merge_runs_device: pairwise merge path)."""
        n = int(sum(run_counts))
        if n * self.rs > src.numel():
            raise ValueError("source too small")
        if not src.is_cuda:
            import torch

            src = src.to(torch.device("cuda", self._device))
        arr = (ctypes.c_uint64 * max(1, len(run_counts)))(*[int(x) for x in run_counts])
        self._chk(self._L.kc_merge_runs_device(self._h, ctypes.c_void_p(src.data_ptr()), arr, len(run_counts)))
        return self.finish()

    def write_output(self, path: str, fan_in: int = 2, threads: int = 2):
        self.finish()
        self._chk(self._L.kc_write_output(self._h, path.encode(), fan_in, threads))

    def write_output_at(self, path: str, offset: int):
        """The finished table run into an existing file at `offset` (kc_write_output_at)."""
        self.finish()
        self._chk(self._L.kc_write_output_at(self._h, path.encode(), offset))

    def write_runs(self, prefix: str) -> List[str]:
        self.finish()
        n = ctypes.c_uint32()
        self._chk(self._L.kc_write_runs(self._h, prefix.encode(), ctypes.byref(n)))
        return [f"{prefix}.{i}" for i in range(n.value)]

    def output_bytes(self, tmpdir: str) -> bytes:
        """Final SortedKMerFile bytes (table run merged with spill runs)."""
        path = os.path.join(tmpdir, f"kc_out_{id(self)}.bin")
        self.write_output(path)
        with open(path, "rb") as f:
            data = f.read()
        os.unlink(path)
        return data

    def stats(self) -> dict:
        s = Stats()
        self._chk(self._L.kc_get_stats(self._h, ctypes.byref(s)))
        return s.as_dict()


def count_file(ctxs, path: str, line_length: int = 0, mode: str = "auto") -> int:
    """kc_count_file: a FASTQ file read in pinned blocks and dealt to the
    contexts (read-shard); mode auto | fastq | exact (include/kc.h)."""
    L = lib()
    arr = (ctypes.c_void_p * len(ctxs))(*[c._h.value for c in ctxs])
    n = ctypes.c_uint64()
    st = L.kc_count_file(arr, len(ctxs), path.encode(), line_length, _INPUT_MODES[mode], ctypes.byref(n))
    if st:
        raise KcError(st, f"{L.kc_strerror(st).decode()}: {L.kc_last_error(ctxs[0]._h).decode()}")
    return n.value


def owner_of(key0: int, world: int) -> int:
    """Key-space owner of a key: ((word0 >> 32) * world) >> 32,
    the top log2(world) bits of word 0 when world is a power of two; monotone
    in the key, so owner order is SortedKMerFile order (kc.h kc_owner_counts)."""
    return ((key0 >> 32) * world) >> 32


def exchange_contexts(ctxs) -> None:
    """kc_exchange_contexts: the key-space exchange between contexts of one
    process; afterwards ctxs[o] holds the keys with owner_of(key) == o."""
    L = lib()
    arr = (ctypes.c_void_p * len(ctxs))(*[c._h.value for c in ctxs])
    st = L.kc_exchange_contexts(arr, len(ctxs))
    if st:
        raise KcError(st, f"{L.kc_strerror(st).decode()}: {L.kc_last_error(ctxs[0]._h).decode()}")


def gather_contexts(ctxs) -> None:
    """kc_gather_contexts: every context's run merged on ctxs[0]'s device."""
    L = lib()
    arr = (ctypes.c_void_p * len(ctxs))(*[c._h.value for c in ctxs])
    st = L.kc_gather_contexts(arr, len(ctxs))
    if st:
        raise KcError(st, f"{L.kc_strerror(st).decode()}: {L.kc_last_error(ctxs[0]._h).decode()}")


def keyspace_exchange(run, dist, device) -> int:
    """Key-space partition step of cfg4: every rank has counted its
    own reads into a finished sorted run; rank o ends up owning the keys with
    owner_of(key) == o, summed over all ranks, so the ranks' outputs
    concatenated in rank order are the whole node's SortedKMerFile.

    `run` is a Context (or anything with finish/owner_counts/export_records/
    merge_records and rs); `dist` an initialised torch.distributed (RCCL on
    GPUs: `device` is the rank's cuda device and the records never leave HBM;
    gloo: `device` is cpu and the records are staged through host memory).
    One all-to-all of world u64 counts, then one all-to-all of the packed
    records (12 B per record at k<=32). Returns the rank's merged record count.
    """
    import torch

    world = dist.get_world_size()
    rs = run.rs
    n = run.finish()
    counts = run.owner_counts(world)
    send = torch.empty(n * rs, dtype=torch.uint8, device=device)
    run.export_records(send)
    sc = torch.tensor(counts, dtype=torch.int64, device=device)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc)
    rcounts = [int(x) for x in rc.tolist()]
    m = sum(rcounts)
    recv = torch.empty(m * rs, dtype=torch.uint8, device=device)
    dist.all_to_all_single(recv, send, [c * rs for c in rcounts], [c * rs for c in counts])
    if recv.is_cuda:
        torch.cuda.current_stream(recv.device).synchronize()  # RCCL ran on torch's stream
    del send
    # what arrived is one sorted slice per source rank, in rank order
    if hasattr(run, "merge_runs"):
        return run.merge_runs(recv, rcounts)
    return run.merge_records(recv, m)


class Options:
    """Mirror of the reference's Options (Options.h:21-57) with the defaults
    main.cpp:27-30 installs over Options() (Options.cpp:16-22)."""

    def __init__(self):
        self._inputFileDirectory = "/home/jayangad/data/1"
        self._gpuMemoryLimit = 100000000
        self._kmerLength = 32
        self._tempFileLocation = "/tmp/1"
        self._outputFile = "/tmp/2/output.bin"
        self._noOfMergersAtOnce = 2
        self._noOfMergeThreads = 2

    def SetInputFileDirectory(self, d): self._inputFileDirectory = d
    def GetInputFileDirectory(self): return self._inputFileDirectory
    def SetGpuMemoryLimit(self, v): self._gpuMemoryLimit = int(v)
    def GetGpuMemoryLimit(self): return self._gpuMemoryLimit
    def SetKmerLength(self, v): self._kmerLength = int(v)
    def GetKmerLength(self): return self._kmerLength
    def setOutputFile(self, v): self._outputFile = v
    def getOutputFile(self): return self._outputFile
    def setTempFileLocation(self, v): self._tempFileLocation = v
    def getTempFileLocation(self): return self._tempFileLocation
    def setNoOfMergersAtOnce(self, v): self._noOfMergersAtOnce = int(v)
    def getNoOfMergersAtOnce(self): return self._noOfMergersAtOnce
    def setNoOfMergeThreads(self, v): self._noOfMergeThreads = int(v)
    def getNoOfMergeThreads(self): return self._noOfMergeThreads

    def argv(self) -> List[str]:
        return [f"kmerLength={self._kmerLength}", f"gpuMemoryLimit={self._gpuMemoryLimit}",
                f"inputFileLocation={self._inputFileDirectory}", f"tempFileLocation={self._tempFileLocation}",
                f"outputFile={self._outputFile}", f"noOfMergersAtOnce={self._noOfMergersAtOnce}",
                f"noOfMergeThreads={self._noOfMergeThreads}"]


class KMerCounter:
    """Mirror of KMerCounter (KMerCounter.h:70-75): Start() counts every file of
    the input directory and writes the SortedKMerFile output, by running the
    native `kmer-counter` CLI (same key=value arguments)."""

    def __init__(self, options: Options, extra_args: Optional[List[str]] = None):
        self._options = options
        self._extra = list(extra_args or [])

    def Start(self) -> subprocess.CompletedProcess:
        if not os.path.exists(CLI_PATH):
            raise ImportError(f"{CLI_PATH} is missing: run `make -C kmer-counter_amd`")
        r = subprocess.run([CLI_PATH] + self._options.argv() + self._extra, capture_output=True, text=True)
        if r.returncode != 0:
            raise KcError(KC_ERR_INTERNAL, r.stderr.strip())
        return r


class KMerPrinter:
    """Mirror of KMerPrinter (KMerPrinter.h): `kmer-counter print in out k`."""

    def __init__(self, inputFilename: str, outputFilename: str, kmerlength: int):
        self._args = [inputFilename, outputFilename, str(kmerlength)]

    def print(self) -> str:
        r = subprocess.run([CLI_PATH, "print"] + self._args, capture_output=True, text=True, check=True)
        return r.stdout
