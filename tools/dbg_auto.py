import sys, os
sys.path.insert(0, "tests"); import conftest
kca = conftest.load_pkg()
fq = kca.synth_fastq(160_000, 150, seed=77)
with kca.Context(kmer_length=31, line_length=150, engine="auto") as ctx:
    ctx.count_fastq(fq)
    print(ctx.stats()["engines_used"], ctx.stats()["keys"], ctx.stats()["batches"])
