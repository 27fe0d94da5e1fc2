import sys, os
sys.path.insert(0, os.getcwd() + "/tests")
from conftest import load_pkg
kca = load_pkg()
ctx = kca.Context(kmer_length=31, line_length=150)
ctx.count_fastq(kca.synth_fastq(100, 150, seed=1))
import torch
print("torch avail after ctx:", torch.cuda.is_available(), torch.cuda.device_count())
t = torch.empty(10, device="cuda:0")
print("ok", t.device)
