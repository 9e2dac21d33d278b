import torch, sys
dev = torch.device("cuda", 0)
for (M, N, K) in [(32000, 512, 2048), (32000, 2048, 512), (32000, 1536, 512), (32000, 512, 512)]:
    A = torch.randn(M, K, device=dev).bfloat16()
    W = torch.randn(N, K, device=dev).bfloat16()
    for _ in range(5):
        torch.matmul(A, W.t())
torch.cuda.synchronize()
