"""Device time of the sampler-table generation (ctl_sampler_generate: one
sampler_kernel launch per pass), averaged over 200 passes with HIP events on
the call's stream.  CTL_LIB selects the library (A/B)."""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch
import cudatracerlib_amd as ctl

pt = ctl.PathTracer(0)
s = torch.cuda.current_stream()
for p in range(20):
    pt.generate_samples(p, s.cuda_stream)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
for p in range(200):
    pt.generate_samples(1000 + p, s.cuda_stream)
e1.record(s)
torch.cuda.synchronize()
print(f"sampler tables: {e0.elapsed_time(e1) / 200 * 1e3:.1f} us per pass ({os.environ.get('CTL_LIB', 'in-tree')})")
pt.close()
