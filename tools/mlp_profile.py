import torch, sys
sys.path.insert(0, '.')
from long_context_biomedical_imaging_amd import blocks
M, D, H = 131072, 384, 1536
mb = blocks.MLPBlock(D, H).cuda()
xm = torch.randn(M, D, device="cuda", requires_grad=True)
gy = torch.randn(M, D, device="cuda").to(torch.bfloat16)
def step():
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = mb(xm)
    y.backward(gy)
blocks.FUSED_MLP = True
for _ in range(3): step()
torch.cuda.synchronize()
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA, torch.profiler.ProfilerActivity.CPU]) as prof:
    for _ in range(3): step()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25, max_name_column_width=60))
