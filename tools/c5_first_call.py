import os, sys, time
sys.path.insert(0, os.getcwd())
import torch
import rogtk_amd
from rogtk_amd import bam as B, synth_bam
path = "/tmp/rogtk_c5.bam"
synth_bam.synth_bam(path, 4_000_000, level=6, threads=16)
torch.cuda.init()
t = time.perf_counter(); tab = B.bam_umi_cluster(path, umi_len=12, max_distance=1, source="sequence", mode="htslib", n_threads=16); print("whole file", time.perf_counter() - t, flush=True)
os.environ["ROGTK_BAM_TIMING"] = "1"
for i in range(3):
    t = time.perf_counter()
    tab4 = B.bams_umi_cluster([path], umi_len=12, max_distance=1, source="sequence", mode="htslib", n_threads=16, ranges_per_file=4)
    print(f"call {i}: {time.perf_counter() - t:.3f} s", flush=True)
