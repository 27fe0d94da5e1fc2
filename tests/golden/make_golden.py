"""Regenerates the golden fixtures in tests/golden/ (committed).

Inputs are small FASTQ files made here with Python's `random` (fixed seeds).
Expected outputs are the SortedKMerFile bytes of the reference count path,
computed by the C oracle (oracle/kc_oracle.c, spec form) and required to be
identical to (a) the oracle's ref-structured form, (b) the oracle's
multi-threaded refcpu pipeline and (c) the pure-Python statement in
tests/kmer_ref_py.py before they are written. MANIFEST.json holds the sha256
of every file.

Usage: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(HERE))
import oracle  # noqa: E402
import kmer_ref_py  # noqa: E402


def fastq(reads, hdr=lambda i: f"@r{i}"):
    return "".join(f"{hdr(i)}\n{s}\n+\n{'I' * len(s)}\n" for i, s in enumerate(reads))


def iid(rng, n, L, n_rate=0.0, alphabet="ACGT"):
    out = []
    for _ in range(n):
        s = [rng.choice(alphabet) for _ in range(L)]
        if n_rate:
            s = ["N" if rng.random() < n_rate else c for c in s]
        out.append("".join(s))
    return out


def genome_reads(rng, n, L, G):
    g = "".join(rng.choice("ACGT") for _ in range(G))
    return [g[p:p + L] for p in (rng.randrange(G - L + 1) for _ in range(n))]


def cases():
    rng = random.Random(20161021)
    yield "cfg1_k21_L100", 21, fastq(iid(rng, 600, 100, 0.002))
    yield "genome_k31_L150", 31, fastq(genome_reads(rng, 600, 150, 20000))
    yield "genome_k55_L150", 55, fastq(genome_reads(rng, 400, 150, 20000))
    special = ["A" * 100, "N" * 100, "T" * 100, "ACGT" * 25, "acgt" * 25,
               "A" * 50 + "N" + "C" * 49, "N" + "G" * 99, "G" * 99 + "N", "AAAAC" * 20]
    yield "special_k31_L100", 31, fastq(special + iid(rng, 50, 100, 0.05))
    yield "special_k32_L100", 32, fastq(special + iid(rng, 50, 100, 0.05))
    yield "special_k21_L100", 21, fastq(special + iid(rng, 50, 100, 0.05))
    yield "k29_L90_nrate", 29, fastq(iid(rng, 300, 90, 0.01))
    yield "k64_L130", 64, fastq(iid(rng, 200, 130, 0.003))
    yield "k1_L33", 1, fastq(iid(rng, 100, 33, 0.02))
    yield "k100_L101", 100, fastq(iid(rng, 100, 101, 0.001))
    mixed = ["".join(c if rng.random() > 0.01 else rng.choice("acgtNRY") for c in s) for s in iid(rng, 100, 70)]
    yield "mixedcase_k31_L70", 31, fastq(mixed)


def main():
    manifest = {}
    for name, k, text in cases():
        data = text.encode()
        want = oracle.count_fastq(data, k, mode="spec")
        assert want == oracle.count_fastq(data, k, mode="ref"), name
        assert want == oracle.refcpu(data, k, threads=3)[0], name
        py = kmer_ref_py.to_bytes(kmer_ref_py.count_reads(kmer_ref_py.fastq_reads(text), k), k)
        assert want == py, name
        fq, out = f"{name}.fq", f"{name}.k{k}.bin"
        open(os.path.join(HERE, fq), "wb").write(data)
        open(os.path.join(HERE, out), "wb").write(want)
        manifest[name] = {"k": k, "fastq": fq, "expected": out,
                          "sha256_fastq": hashlib.sha256(data).hexdigest(),
                          "sha256_expected": hashlib.sha256(want).hexdigest(),
                          "records": len(want) // oracle.rs_of(k)}
        print(name, k, manifest[name]["records"])
    json.dump(manifest, open(os.path.join(HERE, "MANIFEST.json"), "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
