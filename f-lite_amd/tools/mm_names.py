import torch
a = torch.randn(8192, 8192, device="cuda").bfloat16(); b = torch.randn(8192, 8192, device="cuda").bfloat16()
for _ in range(3): torch.mm(a, b.t())
a = torch.randn(8224, 3072, device="cuda").bfloat16(); b = torch.randn(24576, 3072, device="cuda").bfloat16()
for _ in range(3): torch.mm(a, b.t())
torch.cuda.synchronize()
