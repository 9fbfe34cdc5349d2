"""torch.addmm (hipBLASLt) on the fp32 ViT shapes, for a rocprofv3 kernel-name / timing trace."""
import torch

for (N, K) in [(1536, 512), (2048, 512), (512, 2048), (512, 512)]:
    x = torch.randn(32768, K, device="cuda")
    w = torch.randn(N, K, device="cuda") / K ** 0.5
    b = torch.randn(N, device="cuda")
    for _ in range(5):
        torch.addmm(b, x, w.t())
torch.cuda.synchronize()
print("done")
