#!/usr/bin/env python3
"""Host-phase probe of the end-to-end path on the GPU box (KC_TRACE output to
stderr): cfg2 input file -> count_file -> finish -> write_output, the output
written to a new path and over an existing file."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from conftest import load_pkg  # noqa: E402

kca = load_pkg()
reads = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
wd = os.environ.get("TMPDIR", "/tmp")
ctx = kca.Context(kmer_length=31, line_length=150, gpu_memory_limit=160 << 30)
ptr, nb = ctx.synth_device(reads, 150, 2, 250_000_000, 0.0, 0)
host = np.empty(nb, dtype=np.uint8)
ctx.copy_to_host_addr(host.ctypes.data, ptr, nb)
inp = os.path.join(wd, "kc_probe_in.fq")
t = time.perf_counter()
host.tofile(inp)
print(f"input file written: {nb / 1e9:.2f} GB in {time.perf_counter() - t:.2f} s", flush=True)
for rep in range(2):
    t0 = time.perf_counter()
    ctx.reset()
    ctx.count_file(inp)
    t1 = time.perf_counter()
    n = ctx.finish()
    t2 = time.perf_counter()
    out = os.path.join(wd, f"kc_probe_out{rep}.bin")
    ctx.write_output(out)
    t3 = time.perf_counter()
    ctx.write_output(out)  # over the existing file
    t4 = time.perf_counter()
    os.unlink(out)
    ctx.write_output(out)  # a new file again
    t5 = time.perf_counter()
    print(f"rep {rep}: count_file {1e3 * (t1 - t0):.1f} ms ({nb / (t1 - t0) / 1e9:.1f} GB/s), finish "
          f"{1e3 * (t2 - t1):.1f} ms, write new {1e3 * (t3 - t2):.1f} ms, over existing {1e3 * (t4 - t3):.1f} ms, "
          f"new again {1e3 * (t5 - t4):.1f} ms ({n * 12 / 1e9:.2f} GB)", flush=True)
    os.unlink(out)
t = time.perf_counter()
ctx.reset()
ctx.count_fastq_host(host.ctypes.data, nb)
print(f"count_fastq from pageable host memory: {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
os.unlink(inp)
ctx.free_device(ptr)
ctx.close()
