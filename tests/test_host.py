"""Host-side checks that need no GPU: the C ABI library loads and exports every
symbol of include/kc.h, the synthetic generator spec, the host merge against
the reference's own merger, the print subcommand against the reference's own
printer, and the CLI option surface."""
import os
import random
import subprocess

import numpy as np
import pytest

import kmer_ref_py as kp


def test_library_exports_header_symbols(kca):
    L = kca.lib()
    names = kca.header_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing
    assert L.kc_abi_version() == 7
    assert L.kc_strerror(4) == b"malformed FASTQ block"


EXPERIMENT_KNOBS = ("KC_F_SKIP", "KC_P2_SKIP", "KC_P5_SKIP", "KC_SEG_SKIP", "KC_SKM_MMIN")


def test_release_library_ignores_timing_ablations(kca):
    """The stage-skipping timing knobs (outputs invalid after the skipped
    stage) exist only in experiment builds (-DKC_EXPERIMENTS,
    tools/build_variant.sh): the release library does not even hold their
    names, so no environment variable can change what it counts."""
    blob = open(kca.LIB_PATH, "rb").read()
    assert [k for k in EXPERIMENT_KNOBS if k.encode() in blob] == []


def test_no_device_is_an_error_not_a_fallback(kca):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(kca.KcError) as e:
        kca.Context(kmer_length=31, line_length=150)
    assert e.value.status == kca.KC_ERR_NODEVICE


MASK = (1 << 64) - 1


def _splitmix(x):
    x = (x + 0x9E3779B97F4A7C15) & MASK
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & MASK
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & MASK
    return x ^ (x >> 31)


def _rand(seed, stream, i):
    return _splitmix((_splitmix(seed ^ ((stream * 0xD1342543DE82EF95) & MASK)) + i) & MASK)


def _py_record(i, L, seed, genome, n_thr):
    pos = _rand(seed, 1, i) % (genome - L + 1) if genome else 0
    s = []
    for j in range(L):
        if genome:
            g = pos + j
            c = (_rand(seed, 2, g >> 5) >> (2 * (g & 31))) & 3
        else:
            c = (_rand(seed, 4, i * ((L + 31) // 32) + (j >> 5)) >> (2 * (j & 31))) & 3
        ch = "ACGT"[c]
        if n_thr and (_rand(seed, 3, i * L + j) >> 11) < n_thr:
            ch = "N"
        s.append(ch)
    return f"@r{i}\n{''.join(s)}\n+\n{'I' * L}\n"


@pytest.mark.parametrize("L,seed,genome,n_rate,first", [(100, 1, 0, 0.002, 0), (150, 2, 5000, 0.0, 0),
                                                        (150, 3, 100000, 0.01, 98)])
def test_synth_generator_spec(kca, L, seed, genome, n_rate, first):
    n = 7
    got = kca.synth_fastq(n, L, seed, genome_length=genome, n_rate=n_rate, first_read=first).decode()
    n_thr = int(n_rate * 2 ** 53) if n_rate > 0 else 0
    want = "".join(_py_record(i, L, seed, genome, n_thr) for i in range(first, first + n))
    assert got == want


def _run_file(path, recs, W):
    with open(path, "wb") as f:
        for key, c in recs:
            for w in key:
                f.write(int(w).to_bytes(8, "little"))
            f.write(int(c).to_bytes(4, "little"))


def _random_runs(rng, nruns, per, W, dup_frac=0.2, space=1 << 20):
    runs = []
    for _ in range(nruns):
        keys = sorted(tuple(rng.randrange(space) for _ in range(W)) for _ in range(per))
        recs = []
        for key in keys:
            recs.append((key, rng.randrange(1, 5)))
            if rng.random() < dup_frac:  # equal consecutive records inside a run are folded on read
                recs.append((key, rng.randrange(1, 5)))
        runs.append(recs)
    return runs


def _expected(runs, W):
    acc = {}
    for r in runs:
        for key, c in r:
            acc[key] = (acc.get(key, 0) + c) & 0xFFFFFFFF
    out = bytearray()
    for key in sorted(acc):
        for w in key:
            out += int(w).to_bytes(8, "little")
        out += acc[key].to_bytes(4, "little")
    return bytes(out)


@pytest.mark.parametrize("k,nruns,fan,thr", [(31, 1, 2, 2), (31, 2, 2, 2), (31, 5, 2, 2), (55, 4, 3, 2),
                                             (31, 9, 4, 3), (100, 3, 2, 1)])
def test_merge_matches_reference_merger(kca, orc, tmp_path, k, nruns, fan, thr):
    W = (k + 31) // 32
    rng = random.Random(k * 31 + nruns)
    runs = _random_runs(rng, nruns, 3000, W, space=5000 if W == 1 else 40)
    paths = []
    for i, r in enumerate(runs):
        p = tmp_path / f"run{i}"
        _run_file(p, r, W)
        paths.append(str(p))
    out = tmp_path / "merged.bin"
    kca.merge_files(paths, str(out), k, fan, thr)
    mine = out.read_bytes()
    assert mine == _expected(runs, W)
    if orc.have_ref("ref_merge"):
        try:
            ref = orc.ref_merge(paths, str(tmp_path / "ref.bin"), k, fan, thr, timeout=20)
        except orc.RefHang:
            # e.g. 9 runs, fan-in 4: two merges leave 3 files < fan-in and the
            # handler sleeps forever; compare against one reference merger
            ref = orc.ref_merge(paths, str(tmp_path / "ref.bin"), k, len(paths) + 1, 1)
        assert ref == mine


@pytest.mark.parametrize("k,nruns,thr,rr", [(31, 8, 4, 500), (31, 3, 16, 64), (55, 5, 3, 300), (100, 2, 2, 50),
                                            (31, 1, 4, 100)])
def test_merge_key_ranges_parallel(kca, orc, tmp_path, monkeypatch, k, nruns, thr, rr):
    """The last merge level by key ranges (kc_io.cpp merge_runs_parallel):
    small ranges (KC_MERGE_RANGE_RECS) put many range edges among duplicate
    keys inside and across runs, and a long stretch of one repeated key that
    no edge may split; the bytes equal the single-threaded merge's and the
    reference merger's."""
    monkeypatch.setenv("KC_MERGE_RANGE_RECS", str(rr))
    W = (k + 31) // 32
    rng = random.Random(k * 7 + nruns + rr)
    runs = _random_runs(rng, nruns, 4000, W, dup_frac=0.3, space=6000 if W == 1 else 50)
    key = runs[0][len(runs[0]) // 2][0]
    runs[0] = sorted(runs[0] + [(key, 3)] * (5 * rr))  # one key repeated across several ranges' worth
    paths = []
    for i, r in enumerate(runs):
        p = tmp_path / f"run{i}"
        _run_file(p, r, W)
        paths.append(str(p))
    out = tmp_path / "merged.bin"
    (tmp_path / "merged.bin").write_bytes(b"x" * 10_000_000)  # an older, larger file is overwritten and cut
    kca.merge_files(paths, str(out), k, max(2, nruns), thr)
    mine = out.read_bytes()
    assert mine == _expected(runs, W)
    one = tmp_path / "one.bin"
    kca.merge_files(paths, str(one), k, max(2, nruns), 1)
    assert one.read_bytes() == mine
    if orc.have_ref("ref_merge"):
        assert orc.ref_merge(paths, str(tmp_path / "ref.bin"), k, len(paths) + 1, 1) == mine


@pytest.mark.parametrize("k,nruns,parts,thr,rr", [(31, 8, 2, 3, 400), (31, 8, 8, 2, 100), (31, 12, 3, 4, 300),
                                                  (31, 20, 5, 2, 200), (21, 2, 7, 1, 1 << 20), (55, 4, 3, 2, 150),
                                                  (100, 3, 4, 2, 80), (31, 1, 3, 2, 100), (31, 5, 1, 4, 100)])
def test_merge_parts_concatenate(kca, orc, tmp_path, monkeypatch, k, nruns, parts, thr, rr):
    """The merge shared by `parts` processes (kc_merge_part_create /
    kc_merge_part_write, cfg3's ranks): every part computed from the same
    files on its own (no exchange), written at the prefix sum of the parts'
    sizes into one file holding an older, larger file's bytes; the result
    equals merge_files' bytes and the reference merger's. Runs with in-run
    duplicates, a key repeated for several ranges' worth, an empty run, u32
    count wrap; 1 to 20 runs (the one-word merge's 4/8/16-lane forms and its
    fallback) and more parts than some runs have distinct keys."""
    monkeypatch.setenv("KC_MERGE_RANGE_RECS", str(rr))
    W = (k + 31) // 32
    rng = random.Random(k * 13 + nruns * 5 + parts)
    runs = _random_runs(rng, nruns, 2500, W, dup_frac=0.2, space=4000 if W == 1 else 40)
    key = runs[0][len(runs[0]) // 3][0]
    runs[0] = sorted(runs[0] + [(key, 0xFFFFFFF0)] * (3 * min(rr, 400)))
    if nruns > 2:
        runs[1] = []
    paths = []
    for i, r in enumerate(runs):
        p = tmp_path / f"run{i}"
        _run_file(p, r, W)
        paths.append(str(p))
    want = _expected(runs, W)
    one = tmp_path / "one.bin"
    kca.merge_files(paths, str(one), k, max(2, nruns), 1)
    assert one.read_bytes() == want
    out = tmp_path / "parts.bin"
    out.write_bytes(b"y" * (len(want) + 777_777))
    ps = [kca.MergePart(paths, k, p, parts, thr) for p in range(parts)]
    sizes = [p.nbytes for p in ps]
    assert sum(sizes) == len(want)
    for i in reversed(range(parts)):  # any order
        ps[i].write(str(out), sum(sizes[:i]), sum(sizes))
        ps[i].close()
    assert out.read_bytes() == want
    if parts > 1 and nruns > 1 and rr < 1 << 20:
        assert max(sizes) < 0.75 * len(want)  # the boundaries split the key space
    if orc.have_ref("ref_merge"):  # (the reference merger dereferences NULL on an empty run)
        full = [q for q, r in zip(paths, runs) if r]
        assert orc.ref_merge(full, str(tmp_path / "ref.bin"), k, len(full) + 1, 1) == want


def test_merge_part_bad_args(kca, tmp_path):
    p = tmp_path / "r"
    p.write_bytes(b"")
    with pytest.raises(kca.KcError):
        kca.MergePart([str(p)], 31, 2, 2)
    with pytest.raises(kca.KcError):
        kca.MergePart([str(tmp_path / "missing")], 31, 0, 1)
    with kca.MergePart([str(p)], 31, 0, 1) as mp:
        assert mp.nbytes == 0
        with pytest.raises(kca.KcError):
            mp.write(str(tmp_path / "o"), 5, 4)  # past the file size


def test_merge_large_runs_cross_cache_refill(kca, orc, tmp_path):
    """Runs above the reference's 1M-record cache (SortedKMerFile.cpp:29)."""
    rng = np.random.default_rng(3)
    paths, allk, allc = [], [], []
    for i in range(2):
        keys = np.sort(rng.integers(0, 1 << 62, size=1_200_000, dtype=np.uint64))
        keys[1::7] = keys[0::7][: len(keys[1::7])]  # in-run duplicates
        keys.sort()
        cnt = rng.integers(1, 1000, size=keys.size, dtype=np.uint32)
        rec = np.zeros(keys.size, dtype=[("k", "<u8"), ("c", "<u4")])
        rec["k"], rec["c"] = keys, cnt
        p = tmp_path / f"big{i}"
        rec.tofile(p)
        paths.append(str(p))
        allk.append(keys)
        allc.append(cnt)
    out = tmp_path / "m.bin"
    kca.merge_files(paths, str(out), 31, 2, 2)
    k = np.concatenate(allk)
    c = np.concatenate(allc).astype(np.uint64)
    order = np.argsort(k, kind="stable")
    k, c = k[order], c[order]
    uk, start = np.unique(k, return_index=True)
    sums = (np.add.reduceat(c, start) & 0xFFFFFFFF).astype(np.uint32)
    want = np.zeros(uk.size, dtype=[("k", "<u8"), ("c", "<u4")])
    want["k"], want["c"] = uk, sums
    assert out.read_bytes() == want.tobytes()
    if orc.have_ref("ref_merge"):
        assert orc.ref_merge(paths, str(tmp_path / "r.bin"), 31, 2, 2) == out.read_bytes()


@pytest.mark.parametrize("k", [21, 31, 55, 100])
def test_print_matches_reference_printer(kca, orc, tmp_path, k):
    W = (k + 31) // 32
    rng = random.Random(k)
    recs = [(tuple(rng.randrange(1 << 64) for _ in range(W)), rng.randrange(1 << 32)) for _ in range(25000)]
    p = tmp_path / "x.bin"
    _run_file(p, recs, W)
    with open(p, "ab") as f:
        f.write(b"\x01\x02\x03")  # trailing partial record
    mine = kca.KMerPrinter(str(p), "ignored", k).print()
    lines = mine.splitlines()
    assert lines[0] == "### kmer-counter application ###"
    if orc.have_ref("ref_print"):
        assert "\n".join(lines[1:]) + "\n" == orc.ref_print(str(p), k)


def test_cli_options_surface(kca, tmp_path):
    """getOptions (main.cpp:25-70): prefix matching, echo lines, last wins."""
    r = subprocess.run([kca.CLI_PATH, "kmerLength=21", "gpuMemoryLimit=5000000", f"inputFileLocation={tmp_path}",
                        "tempFileLocation=/tmp/x", f"outputFile={tmp_path}/o.bin", "noOfMergersAtOnce=3",
                        "noOfMergeThreads=4", "kmerLength=25", "bogus=1"], capture_output=True, text=True)
    out = r.stdout.splitlines()
    assert out[0] == "### kmer-counter application ###"
    assert out[1:9] == ["Updating KmerLength=21", "Updating Gpu Memory Limit=5000000",
                        f"Updating Input File Location='{tmp_path}'", "Updating Temp File Location='/tmp/x'",
                        f"Updating Output File='{tmp_path}/o.bin'", "Updating No Of Mergers At Once='3'",
                        "Updating No Of Merge Threads='4'", "Updating KmerLength=25"]


@pytest.mark.parametrize("arg", ["readLengths=varaible", "outputFormat=dmup", "inputMode=fast", "exchange=all"])
def test_cli_rejects_unknown_mode_values(kca, tmp_path, arg):
    """Additive keys take only their listed values: a typo is an error, not a
    silent switch to another mode (parsing runs before any device is opened)."""
    r = subprocess.run([kca.CLI_PATH, "kmerLength=21", f"inputFileLocation={tmp_path}", arg],
                       capture_output=True, text=True)
    assert r.returncode == 1 and "expected" in r.stderr


def test_cli_rejects_variable_lengths_in_exact_mode(kca, tmp_path):
    r = subprocess.run([kca.CLI_PATH, "kmerLength=21", "readLengths=variable", "inputMode=exact"],
                       capture_output=True, text=True)
    assert r.returncode == 1 and "inputMode=exact" in r.stderr


def test_python_options_mirror_reference_defaults(kca, orc):
    o = kca.Options()
    assert (o.GetKmerLength(), o.getNoOfMergersAtOnce(), o.getNoOfMergeThreads()) == (32, 2, 2)
    assert o.GetGpuMemoryLimit() == 100000000  # main.cpp:28 overrides Options() (1e7)
    if orc.have_ref("ref_options"):
        import subprocess as sp
        r = sp.run([os.path.join(orc.REF_DIR, "ref_options")], capture_output=True, text=True, check=True)
        d = dict(line.split("=") for line in r.stdout.split())
        assert int(d["kmerLength"]) == o.GetKmerLength()
        assert int(d["noOfMergersAtOnce"]) == o.getNoOfMergersAtOnce()
        assert int(d["noOfMergeThreads"]) == o.getNoOfMergeThreads()


def test_pool_par_memcpy_stress(tmp_path):
    """kc_stage's copy pool: par_memcpy of mixed sizes (100 B .. 64 MiB + odd
    tails) back to back through a 16-thread Pool, byte-exact (a worker that
    joined a finished job must not take pieces of the next one)."""
    import shutil
    import subprocess
    if not shutil.which("g++") or not os.path.exists("/opt/rocm/lib/libamdhip64.so"):
        pytest.skip("g++ or the HIP runtime library missing")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "pool_stress")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(root, "kmer-counter_amd", "csrc"),
                    "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", "-pthread",
                    os.path.join(root, "tools", "pool_stress.cpp"),
                    os.path.join(root, "kmer-counter_amd", "csrc", "kc_stage.cpp"), "-L/opt/rocm/lib",
                    "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib", "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "ok" in out.stdout, out.stdout + out.stderr
