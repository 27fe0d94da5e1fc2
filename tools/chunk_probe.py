"""Splits the reference-chunk bench variant into its phases: the 960
kc_count_chunk calls (host side) and kc_finish, against one call of all the
reads; prints ms per phase. Run on the GPU box."""
import time
import numpy as np
import importlib.util, os, sys
sys.path.insert(0, os.getcwd())
spec = importlib.util.spec_from_file_location("kca", os.path.join("kmer-counter_amd", "__init__.py"))
kca = importlib.util.module_from_spec(spec); spec.loader.exec_module(kca)
L, k, reads = 150, 31, 50_000_000
ctx = kca.Context(kmer_length=k, line_length=L, gpu_memory_limit=160 << 30)
sptr, sbytes = ctx.synth_device(reads, L, 2, 250_000_000, 0.0, 0, 0, layout=1)
seqs = np.empty(sbytes, dtype=np.uint8)
ctx.copy_to_host_addr(seqs.ctypes.data, sptr, sbytes)
ctx.free_device(sptr)
kb = (k + 3) // 4
per = ((kb + 7) // 8 + 1) * 8 * (L - k + 1)
cs = L * ((100000000 - L) // (per - 1))
base = seqs.ctypes.data
for rep in range(3):
    for name, pieces in (("chunks", [(o, min(cs, sbytes - o)) for o in range(0, sbytes, cs)]), ("block", [(0, sbytes)])):
        ctx.reset()
        t0 = time.perf_counter()
        for o, n in pieces:
            ctx.count_chunk_host(base + o, n, L)
        t1 = time.perf_counter()
        ctx.finish()
        t2 = time.perf_counter()
        print(f"{name:7s} calls {1e3*(t1-t0):8.2f} ms  finish {1e3*(t2-t1):8.2f} ms  total {1e3*(t2-t0):8.2f}", flush=True)
# host memcpy rate alone (pageable -> pageable, one thread)
dst = np.empty(cs, dtype=np.uint8)
t0 = time.perf_counter()
for o in range(0, 200 * cs, cs):
    dst[:] = seqs[o:o + cs]
print(f"numpy memcpy 1 thread: {200*cs/(time.perf_counter()-t0)/1e9:.1f} GB/s")
