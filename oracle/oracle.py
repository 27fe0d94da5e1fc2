"""ctypes binding of the CPU oracle (oracle/kc_oracle.c) and of the reference
programs built from /root/reference sources into oracle/_ref/.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg — never by the product (kmer-counter_amd/).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_DIR = os.path.join(HERE, "_ref")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", HERE, os.path.basename(LIB) and LIB], check=True,
                           stdout=subprocess.DEVNULL)
        L = ctypes.CDLL(LIB)
        i64, u64, vp = ctypes.c_int64, ctypes.c_uint64, ctypes.c_void_p
        P = ctypes.POINTER
        L.oracle_chunk_size.argtypes = [i64, i64, i64]
        L.oracle_chunk_size.restype = i64
        L.oracle_count_fastq.argtypes = [ctypes.c_char_p, i64, i64, i64, ctypes.c_int, P(vp)]
        L.oracle_count_fastq.restype = i64
        L.oracle_refcpu_count.argtypes = [vp, i64, i64, i64, ctypes.c_int, P(vp), P(u64)]
        L.oracle_refcpu_count.restype = i64
        L.oracle_refcpu_run.argtypes = [vp, i64, i64, i64, ctypes.c_int, vp, P(u64)]
        L.oracle_refcpu_run.restype = i64
        L.oracle_free.argtypes = [vp]
        L.oracle_acc_new.argtypes = [i64]
        L.oracle_acc_new.restype = vp
        L.oracle_acc_free.argtypes = [vp]
        L.oracle_acc_add_chunk_spec.argtypes = [vp, ctypes.c_char_p, i64, i64]
        L.oracle_acc_add_chunk_ref.argtypes = [vp, ctypes.c_char_p, i64, i64]
        L.oracle_acc_finish.argtypes = [vp, P(vp)]
        L.oracle_acc_finish.restype = i64
        L.oracle_reader_new.argtypes = [ctypes.c_char_p, i64]
        L.oracle_reader_new.restype = vp
        L.oracle_reader_next.argtypes = [vp, i64, ctypes.c_char_p]
        L.oracle_reader_next.restype = i64
        L.oracle_reader_done.argtypes = [vp]
        L.oracle_reader_done.restype = ctypes.c_int
        L.oracle_reader_line_length.argtypes = [vp]
        L.oracle_reader_line_length.restype = i64
        L.oracle_reader_free.argtypes = [vp]
        L.oracle_window_checksum.argtypes = [vp, i64, i64, ctypes.c_int, P(u64)]
        L.oracle_window_checksum.restype = ctypes.c_int
        L.oracle_records_checksum.argtypes = [vp, i64, i64, ctypes.c_int, P(u64)]
        L.oracle_records_checksum.restype = ctypes.c_int
        _lib = L
    return _lib


def _take(ptr, n: int) -> bytes:
    """n bytes at a C pointer (ctypes.string_at takes a C int size: <= 2 GiB)."""
    return (ctypes.c_char * n).from_address(ptr.value if hasattr(ptr, "value") else ptr).raw


def rs_of(k: int) -> int:
    return 8 * ((k + 31) // 32) + 4


def chunk_size(L: int, k: int, limit: int) -> int:
    return lib().oracle_chunk_size(L, k, limit)


def count_fastq(data: bytes, k: int, gpu_memory_limit: int = 100000000, mode: str = "spec") -> bytes:
    """Sorted SortedKMerFile bytes of the reference count path over one FASTQ file."""
    L = lib()
    out = ctypes.c_void_p()
    n = L.oracle_count_fastq(data, len(data), k, gpu_memory_limit, 1 if mode == "ref" else 0, ctypes.byref(out))
    if n < 0:
        raise ValueError("bad oracle arguments")
    res = _take(out, n * rs_of(k)) if n else b""
    L.oracle_free(out)
    return res


def count_chunks(chunks, k: int, mode: str = "spec") -> bytes:
    """Sorted bytes for a list of (chunk_bytes, L) — processKMers + hash per chunk."""
    L = lib()
    acc = L.oracle_acc_new(k)
    for data, ll in chunks:
        if mode == "ref":
            L.oracle_acc_add_chunk_ref(acc, data, len(data), ll)
        else:
            L.oracle_acc_add_chunk_spec(acc, data, len(data), ll)
    out = ctypes.c_void_p()
    n = L.oracle_acc_finish(acc, ctypes.byref(out))
    res = _take(out, n * rs_of(k)) if n else b""
    L.oracle_free(out)
    L.oracle_acc_free(acc)
    return res


def fastq_sequences(data: bytes):
    """Sequence lines (line 2 of every 4-line record) of well-formed FASTQ."""
    lines = data.split(b"\n")
    return [lines[i] for i in range(1, len(lines) - 1, 4)]


def count_fastq_varlen(data: bytes, k: int, mode: str = "spec") -> bytes:
    """Variable-length reads (KC_FLAG_VARLEN): every read
    counted as a reference chunk of that one read with L = its own length
    (processKMers semantics per read, GPUHandler.cu:397-466; a read shorter
    than k contributes nothing). Runs of equal-length reads share a chunk."""
    chunks, run, run_len = [], [], -1
    for s in fastq_sequences(data):
        if len(s) != run_len and run:
            chunks.append((b"".join(run), run_len))
            run = []
        run_len = len(s)
        run.append(s)
    if run:
        chunks.append((b"".join(run), run_len))
    return count_chunks([(c, ll) for c, ll in chunks if ll >= k], k, mode)


def refcpu(data: bytes, k: int, gpu_memory_limit: int = 100000000, threads: int = 1):
    """The reference pipeline on the CPU (chunker + ref-structured encode/extract
    + adjacent reduce + sharded-lock hash + sort). `data`: bytes, a numpy uint8
    array or (address, nbytes). Returns (bytes, windows)."""
    L = lib()
    out = ctypes.c_void_p()
    win = ctypes.c_uint64()
    keep = data
    addr, nb = _addr(data)
    n = L.oracle_refcpu_count(addr, nb, k, gpu_memory_limit, threads, ctypes.byref(out), ctypes.byref(win))
    del keep
    if n < 0:
        raise ValueError("bad oracle arguments")
    res = _take(out, n * rs_of(k)) if n else b""
    L.oracle_free(out)
    return res, win.value


def refcpu_count_only(data: bytes, k: int, gpu_memory_limit: int = 100000000, threads: int = 1):
    """refcpu up to the complete hash table (no sorted dump). Returns
    (distinct keys, windows)."""
    L = lib()
    win = ctypes.c_uint64()
    keep = data
    addr, nb = _addr(data)
    n = L.oracle_refcpu_run(addr, nb, k, gpu_memory_limit, threads, None, ctypes.byref(win))
    del keep
    if n < 0:
        raise ValueError("bad oracle arguments")
    return n, win.value


def _addr(buf):
    """(address, nbytes) of bytes / a numpy array / (address, nbytes)."""
    if isinstance(buf, tuple):
        return buf
    if isinstance(buf, bytes):
        return ctypes.cast(ctypes.c_char_p(buf), ctypes.c_void_p).value, len(buf)
    return buf.ctypes.data, buf.nbytes


def window_checksum(fastq, k: int, threads: int = 1) -> dict:
    """Size-independent parity property (kc_oracle.c, "window checksums"):
    over every valid window of well-formed 4-line FASTQ (spec form, each read at
    its own length) the sums of two 64-bit key hashes, plus windows, valid
    windows, whether any window was invalid (key 0^W present) and reads.
    `fastq`: bytes, a numpy uint8 array or (address, nbytes)."""
    keep = fastq  # the buffer must outlive the call
    addr, n = _addr(fastq)
    out = (ctypes.c_uint64 * 6)()
    if lib().oracle_window_checksum(addr, n, k, threads, out) != 0:
        raise ValueError("bad oracle arguments")
    del keep
    return {"h1": out[0], "h2": out[1], "windows": out[2], "valid": out[3], "hole": bool(out[4]), "reads": out[5]}


def records_checksum(recs, k: int, threads: int = 1) -> dict:
    """The matching sums over SortedKMerFile records: sum count*h1, sum
    count*h2, sum count, and the adjacent pairs that are not strictly
    ascending. `recs`: bytes, a numpy uint8 array or (address, nbytes)."""
    keep = recs
    addr, n = _addr(recs)
    out = (ctypes.c_uint64 * 4)()
    if lib().oracle_records_checksum(addr, n // rs_of(k), k, threads, out) != 0:
        raise ValueError("bad oracle arguments")
    del keep
    return {"h1": out[0], "h2": out[1], "count": out[2], "unordered": out[3]}


def chunks_of(data: bytes, chunk: int):
    """[(chunk_bytes, L)] the reference reader produces for one in-memory file."""
    L = lib()
    r = L.oracle_reader_new(data, len(data))
    ll = L.oracle_reader_line_length(r)
    out = []
    buf = ctypes.create_string_buffer(max(chunk, 0) + 1)
    while not L.oracle_reader_done(r):
        n = L.oracle_reader_next(r, chunk, buf)
        if n > 0 and n >= ll:
            out.append((buf.raw[:n], ll))
    L.oracle_reader_free(r)
    return out


# ---- reference programs (oracle/_ref, built from /root/reference) ----------

def have_ref(name: str) -> bool:
    return os.access(os.path.join(REF_DIR, name), os.X_OK)


def ref_chunks(input_dir: str, chunk: int):
    """Chunks the reference's own InputFileHandler/FASTQFileReader produce."""
    with tempfile.NamedTemporaryFile(delete=False) as t:
        path = t.name
    try:
        subprocess.run([os.path.join(REF_DIR, "ref_reader"), input_dir, str(chunk), path], check=True,
                       stdout=subprocess.DEVNULL, timeout=600)
        data = open(path, "rb").read()
    finally:
        os.unlink(path)
    out, i = [], 0
    while i < len(data):
        size = int.from_bytes(data[i:i + 8], "little", signed=True)
        ll = int.from_bytes(data[i + 8:i + 16], "little", signed=True)
        out.append((data[i + 16:i + 16 + size], ll))
        i += 16 + size
    return out


class RefHang(RuntimeError):
    """The reference's merge handler did not finish (its Run loop waits for
    fan_in files forever once fewer remain, KMerFileMergeHandler.cpp:54-84)."""


def ref_merge(runs, out_path: str, k: int, fan_in: int = 2, threads: int = 2, timeout: float = 30) -> bytes:
    """Merges sorted run files with the reference's own KMerFileMergeHandler."""
    if os.path.exists(out_path):
        os.unlink(out_path)  # the reference appends (KMerFileMerger.cpp:129)
    try:
        subprocess.run([os.path.join(REF_DIR, "ref_merge"), out_path, str(k), str(fan_in), str(threads)] + list(runs),
                       check=True, stdout=subprocess.DEVNULL, timeout=timeout)
    except subprocess.TimeoutExpired as e:
        raise RefHang(str(e)) from None
    return open(out_path, "rb").read()


def ref_print(path: str, k: int) -> str:
    r = subprocess.run([os.path.join(REF_DIR, "ref_print"), path, "ignored", str(k)], check=True,
                       capture_output=True, text=True, timeout=600)
    return r.stdout
